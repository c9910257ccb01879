/** \file fvhip_api.cpp
 * \brief Implementation of the C-ABI in include/fvhip.h: device-resident discretisation,
 *   host<->device plumbing with the reference's cell numbering, kernel timing, mesh builder.
 * No exception crosses the ABI; errors become a nonzero return and fvhip_last_error().
 */
#include "ctx.hpp"

#include <cmath>

namespace fvhip_detail {

fvhip_ctx::GroupExchange groupExchange(const fvhip_group_s* g)
{
	// in-process exchange: pack everywhere, then copy each neighbour's packed rows into the ghost block
	return [g](const fvhip_ctx::ArrayOf& arr_of, int width, int layers) {
		const std::vector<fvhip_ctx*>& hs = g->hs;
		const size_t n = hs.size();
		std::vector<fvhip_ctx*> byrank(n);
		for(fvhip_ctx* h : hs) byrank[h->rank] = h;
		for(size_t i = 0; i < n; i++) if(hs[i]->halo()) { HC(hipSetDevice(hs[i]->device)); hs[i]->pack(arr_of(i), width); }
		for(size_t i = 0; i < n; i++) HC(hipStreamSynchronize(hs[i]->stream));
		for(size_t i = 0; i < n; i++) {
			fvhip_ctx* h = hs[i];
			const Layout& L = h->L;
			for(size_t k = 0; k < L.nbr_rank.size(); k++) {
				fvhip_ctx* q = byrank[L.nbr_rank[k]];
				const Layout& Q = q->L;
				size_t kk = 0;
				while(kk < Q.nbr_rank.size() && Q.nbr_rank[kk] != h->rank) kk++;
				if(kk == Q.nbr_rank.size()) throw std::logic_error("halo lists are not symmetric");
				const int cnt = h->ghostCount(k, layers);
				if(cnt != q->sendCount(kk, layers)) throw std::logic_error("halo sizes differ");
				if(cnt == 0) continue;
				HC(hipMemcpyAsync(arr_of(i) + static_cast<size_t>(width)*(L.ncell + L.ghost_start[k]),
				                  q->d_sendbuf + static_cast<size_t>(width)*Q.send_start[kk],
				                  sizeof(double)*width*static_cast<size_t>(cnt), hipMemcpyDeviceToDevice, h->stream));
			}
		}
		for(size_t i = 0; i < n; i++) HC(hipStreamSynchronize(hs[i]->stream));
	};
}

}

extern "C" {

const char* fvhip_last_error(void) { return g_err.c_str(); }
const char* fvhip_version(void) { return "fvhip 0.1 (gfx950)"; }
int fvhip_device_count(void) {
	int n = 0;
	if(hipGetDeviceCount(&n) != hipSuccess) return 0;
	return n;
}

/// what FlowFV_base's constructor builds from the config (flow_spatial.cpp:45-50, 320): the factories
/// return nullptr for an unknown flux or reconstruction name (afactory.cpp:79-81, 208-211) and the
/// first residual then dereferences it; here the handle is refused instead. An unknown gradient
/// scheme is the reference's ZeroGradients (afactory.cpp:123-127) and stays allowed.
static void checkConfig(const fvhip_flow_config* cfg)
{
	if(cfg->nbc < 0 || cfg->nbc > MAXBC) throw std::invalid_argument("too many boundary conditions");
	if(cfg->nbc > 0 && (!cfg->bc_type || !cfg->bc_tag || !cfg->bc_vals)) throw std::invalid_argument("null argument");
	if(cfg->conv_numflux < 0 || cfg->conv_numflux > 6) throw std::invalid_argument("unknown flux"); // afactory.cpp:78-80
	if(cfg->conv_numflux_jac < 0 || cfg->conv_numflux_jac > 6) throw std::invalid_argument("unknown Jacobian flux");
	if(cfg->reconstruction < 0 || cfg->reconstruction > 4)
		throw std::invalid_argument("Invalid reconstruction");                              // afactory.cpp:208-211
	// Venkatakrishnan's eps^2 = (K clength)^3 (limitedlinearreconstruction.cpp:222): K = 0 makes phi 0/0
	// wherever a cell's neighbours all equal it; the reference never parses K (controlparser.cpp:227-232)
	if(cfg->reconstruction == FVHIP_REC_VENKATAKRISHNAN && !(cfg->limiter_param > 0 && std::isfinite(cfg->limiter_param)))
		throw std::invalid_argument("Venkatakrishnan limiter: limiter_param (K) must be finite and > 0");
	if(cfg->reconstruction == FVHIP_REC_WENO && !(cfg->limiter_param >= 0 && std::isfinite(cfg->limiter_param)))
		throw std::invalid_argument("WENO: limiter_param (lambda) must be finite and >= 0");
	for(int i = 0; i < cfg->nbc; i++) {
		const int t = cfg->bc_type[i];
		if(t == FVHIP_BC_PERIODIC || t < 0 || t > 7) throw std::invalid_argument("BC type not implemented yet!"); // abc.cpp:493-494
	}
}

/// device-resident discretisation of a (possibly partitioned) topology
static fvhip_ctx* createCtx(const MeshTopo& T, const fvhip_flow_config* cfg, int device)
{
	checkConfig(cfg);
	std::unique_ptr<fvhip_ctx> h(new fvhip_ctx());
	h->device = device;
	HC(hipSetDevice(device));
	HC(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
	h->cfg = *cfg;
	h->bc_type.assign(cfg->bc_type, cfg->bc_type + cfg->nbc);
	h->bc_tag.assign(cfg->bc_tag, cfg->bc_tag + cfg->nbc);
	h->bc_vals.assign(cfg->bc_vals, cfg->bc_vals + 2*cfg->nbc);
	h->cfg.bc_type = h->bc_type.data(); h->cfg.bc_tag = h->bc_tag.data(); h->cfg.bc_vals = h->bc_vals.data();

	h->L = buildLayout(T, h->cfg, true);
	Layout& L = h->L;
	auto& o = h->owned;
	DevMesh& M = h->M;
	M.ncell = L.ncell + L.nghost; M.nown = L.ncell; M.nbface = L.nbface;
	M.npatch = static_cast<int>(L.patch_cell.size()) - 1;
	M.nslot = static_cast<int>(L.slot_L.size());
	M.patch_cell = upload(L.patch_cell, o);
	M.patch_slot = upload(L.patch_slot, o);
	M.slot_LR = reinterpret_cast<const int2*>(upload(pack2(L.slot_L, L.slot_R), o));
	M.slot_n = reinterpret_cast<const double2*>(upload(L.slot_n, o));
	M.slot_len = upload(L.slot_len, o);
	M.slot_gr = reinterpret_cast<const double2*>(upload(L.slot_gr, o));
	M.cell_slots = reinterpret_cast<const int4*>(upload(L.cell_slots, o));
	M.cell_nbr = reinterpret_cast<const int4*>(upload(L.cell_nbr_local, o));
	M.cell_face = reinterpret_cast<const int4*>(upload(L.cell_face_local, o));
	M.cell_nbr_fo = reinterpret_cast<const int4*>(upload(L.cell_nbr_fo, o));
	M.rc = reinterpret_cast<const double2*>(upload(L.rc, o));
	M.area = upload(L.area, o);
	M.wls_V = reinterpret_cast<const double4*>(upload(L.wls_V, o));
	M.venk_eps2 = upload(L.venk_eps2, o);
	M.bf_L = upload(L.bf_L, o);
	M.bf_bc = upload(L.bf_bc, o);
	M.bf_n = reinterpret_cast<const double2*>(upload(L.bf_n, o));
	M.bf_rcbp = reinterpret_cast<const double2*>(upload(L.bf_rcbp, o));
	if(!L.fz_ext_start.empty()) {
		M.fz_ext_start = upload(L.fz_ext_start, o);
		M.fz_ext = upload(L.fz_ext, o);
		M.fz_n1 = upload(L.fz_n1, o);
		M.fz_g_start = upload(L.fz_g_start, o);
		M.fz_gnbr = reinterpret_cast<const int4*>(upload(L.fz_gnbr, o));
		M.fz_slot_lr16 = upload(L.fz_slot_lr16, o);
		M.fz_gnbr16 = reinterpret_cast<const uint2*>(upload(L.fz_gnbr16, o));
		M.fz_gbf_start = upload(L.fz_gbf_start, o);
		M.fz_gbf = upload(L.fz_gbf, o);
		M.fz_cslot16 = reinterpret_cast<const uint2*>(upload(L.fz_cslot16, o));
		M.fz_max_cells = L.fz_max_cells;
	}
	M.gg_n = static_cast<int>(L.gg_cells.size());
	M.gg_cells = upload(L.gg_cells, o);
	M.gg_nbr = reinterpret_cast<const int4*>(upload(L.gg_nbr, o));
	M.gg_V = reinterpret_cast<const double4*>(upload(L.gg_V, o));
	M.gg_gp = reinterpret_cast<const double2*>(upload(L.gg_gp, o));
	M.gg_eps2 = upload(L.gg_eps2, o);
	M.xb_bc = upload(L.xb_bc, o);
	M.xb_n = reinterpret_cast<const double2*>(upload(L.xb_n, o));
	M.xb_rcbp = reinterpret_cast<const double2*>(upload(L.xb_rcbp, o));
	if(!L.pipe_patch.empty()) h->d_pipe_patch = upload(L.pipe_patch, o);
	if(L.nghost > 0 && !L.fz_order.empty()) h->d_fz_order = upload(L.fz_order, o);
	h->d_perm = upload(L.perm, o);
	h->nsend = static_cast<int>(L.send_cells.size());
	h->nborder = static_cast<int>(L.border_cells.size());
	if(h->nborder > 0) h->d_border = upload(L.border_cells, o);
	if(h->nsend > 0) {
		h->d_send = upload(L.send_cells, o);
		h->d_sendbuf = dalloc(8*static_cast<size_t>(h->nsend), o);
	}
	if(!L.trace_conn.empty()) {
		if(static_cast<int>(L.trace_conn.size()) != h->nsend) throw std::logic_error("per-rank mesh: trace lists differ");
		h->d_trace_conn = upload(L.trace_conn, o);
		h->d_tracebuf = dalloc(4*static_cast<size_t>(L.nghost), o);
	}

	DevPhys& P = h->P;
	P.gas = gd::make_gas(cfg->gamma, cfg->Minf, cfg->Tinf, cfg->Reinf, cfg->Pr);
	// free stream, aphysics.cpp:43-58 (sideslip 0)
	const double beta = 0;
	P.uinf[0] = 1.0;
	P.uinf[1] = std::cos(cfg->aoa)*std::cos(beta);
	P.uinf[2] = std::sin(cfg->aoa)*std::cos(beta);
	const double pinf = (1.0/(cfg->gamma*cfg->Minf*cfg->Minf));
	P.uinf[3] = pinf/(cfg->gamma-1.0) + 0.5*1.0*1.0;
	P.nbc = cfg->nbc;
	for(int i = 0; i < cfg->nbc; i++) P.bc[i] = gd::BCDev{cfg->bc_type[i], cfg->bc_vals[2*i], cfg->bc_vals[2*i+1]};
	P.limiter_param = cfg->limiter_param;

	const size_t N = static_cast<size_t>(L.ncell), NT = N + static_cast<size_t>(L.nghost);
	const size_t nb = static_cast<size_t>(L.nbface);
	h->d_u = dalloc(4*NT, o); h->d_r = dalloc(4*N, o); h->d_dtm = dalloc(N, o);
	h->d_up = dalloc(4*NT, o); h->d_grad = dalloc(8*NT, o);
	h->d_ubc = dalloc(4*nb, o); h->d_ug = dalloc(4*nb, o);
	if(cfg->reconstruction == FVHIP_REC_WENO) h->d_lgrad = dalloc(8*NT, o);
	if(cfg->reconstruction == FVHIP_REC_BARTHJESPERSEN || cfg->reconstruction == FVHIP_REC_VENKATAKRISHNAN)
		h->d_phi = dalloc(4*NT, o);

	return h.release();
}

int fvhip_create(const fvhip_mesh* mesh, const fvhip_flow_config* cfg, int device, fvhip_handle* out)
{
	return guard([&] {
		if(!mesh || !cfg || !out) throw std::invalid_argument("null argument");
		if(mesh->nconnface > 0) {
			// one rank's subdomain: its rank comes with the communicator (or fvhip_set_rank)
			fvhip_ctx* h = createCtx(topoFromRankMesh(*mesh), cfg, device);
			h->rankmesh = true; h->rank = -1; h->nparts = 0;
			*out = h;
			return;
		}
		*out = createCtx(topoFromMesh(*mesh), cfg, device);
	});
}

int fvhip_set_rank(fvhip_handle h, int rank, int nranks)
{
	return guard([&] {
		need(h, "handle");
		if(!h->rankmesh) throw std::invalid_argument("fvhip_set_rank: not a per-rank mesh handle");
		if(rank < 0 || rank >= nranks) throw std::invalid_argument("rank out of range");
		for(int q : h->L.nbr_rank)
			if(q < 0 || q >= nranks || q == rank) throw std::invalid_argument("connectivity faces name rank "
			                                                                  + std::to_string(q));
		h->rank = rank; h->nparts = nranks;
	});
}

int fvhip_create_partitioned(const fvhip_mesh* mesh, const fvhip_flow_config* cfg, const int* part, int nparts,
                             int rank, int device, fvhip_handle* out)
{
	return guard([&] {
		if(!mesh || !cfg || !part || !out) throw std::invalid_argument("null argument");
		if(rank < 0 || rank >= nparts) throw std::invalid_argument("rank out of range");
		for(int e = 0; e < mesh->nelem; e++)
			if(part[e] < 0 || part[e] >= nparts) throw std::invalid_argument("partition entry out of range");
		fvhip_ctx* h = createCtx(extractPartition(*mesh, part, rank), cfg, device);
		h->rank = rank; h->nparts = nparts;
		*out = h;
	});
}

int fvhip_find_lines(const fvhip_mesh* mesh, double threshold, int* nlines, int* ncells, int* start, int* cells)
{
	return guard([&] {
		need(mesh, "mesh");
		const std::vector<std::vector<int>> lines = findLinesReference(*mesh, threshold);
		int n = 0;
		if(start) start[0] = 0;
		for(size_t i = 0; i < lines.size(); i++) {
			if(cells) std::copy(lines[i].begin(), lines[i].end(), cells + n);
			n += static_cast<int>(lines[i].size());
			if(start) start[i+1] = n;
		}
		if(nlines) *nlines = static_cast<int>(lines.size());
		if(ncells) *ncells = n;
	});
}

int fvhip_partition_rcb(const fvhip_mesh* mesh, int nparts, int* part)
{
	return guard([&] {
		need(mesh, "mesh"); need(part, "part");
		const std::vector<int> p = partitionRCB(mesh->rc, mesh->nelem, nparts);
		std::memcpy(part, p.data(), p.size()*sizeof(int));
	});
}

int fvhip_partition_graph(const fvhip_mesh* mesh, int nparts, int* part)
{
	return guard([&] {
		need(mesh, "mesh"); need(part, "part");
		const std::vector<int> p = partitionGraph(*mesh, nparts);
		std::memcpy(part, p.data(), p.size()*sizeof(int));
	});
}

int fvhip_partition_graph_weighted(const fvhip_mesh* mesh, int nparts, const int* weight, int* part)
{
	return guard([&] {
		need(mesh, "mesh"); need(part, "part");
		const std::vector<int> p = partitionGraph(*mesh, nparts, weight);
		std::memcpy(part, p.data(), p.size()*sizeof(int));
	});
}

long long fvhip_partition_edge_cut(const fvhip_mesh* mesh, const int* part)
{
	long long c = -1;
	if(guard([&] { need(mesh, "mesh"); need(part, "part"); c = edgeCut(*mesh, part); })) return -1;
	return c;
}

int fvhip_partition_info(const fvhip_mesh* mesh, const int* part, int rank, int* counts, int* cell_global,
                         int* nbr_rank, int* ghost_start, int* send_start, int* send_global)
{
	return guard([&] {
		need(mesh, "mesh"); need(part, "part"); need(counts, "counts");
		const MeshTopo T = extractPartition(*mesh, part, rank);
		const int nnbr = static_cast<int>(T.nbr_rank.size());
		counts[0] = T.nown; counts[1] = T.nghost; counts[2] = T.nbface; counts[3] = T.naface;
		counts[4] = nnbr; counts[5] = static_cast<int>(T.send_cells.size());
		if(cell_global) std::memcpy(cell_global, T.cell_global.data(), T.cell_global.size()*sizeof(int));
		if(nbr_rank) for(int k = 0; k < nnbr; k++) nbr_rank[k] = T.nbr_rank[k];
		if(ghost_start) for(int k = 0; k <= nnbr; k++) ghost_start[k] = nnbr ? T.ghost_start[k] : 0;
		if(send_start) for(int k = 0; k <= nnbr; k++) send_start[k] = T.send_start[k];
		if(send_global) for(size_t i = 0; i < T.send_cells.size(); i++) send_global[i] = T.cell_global[T.send_cells[i]];
	});
}

int fvhip_partition_halo_layers(const fvhip_mesh* mesh, const int* part, int rank, int* ghost_l1_end,
                                int* send_l1_end)
{
	return guard([&] {
		const MeshTopo T = extractPartition(*mesh, part, rank);
		for(size_t k = 0; k < T.nbr_rank.size(); k++) {
			if(ghost_l1_end) ghost_l1_end[k] = T.ghost_l1_end[k];
			if(send_l1_end) send_l1_end[k] = T.send_l1_end[k];
		}
	});
}

int fvhip_comm_unique_id(void* id128)
{
	return guard([&] {
		need(id128, "unique id");
		ncclUniqueId id;
		NC(ncclGetUniqueId(&id));
		std::memcpy(id128, &id, sizeof(id));
	});
}

int fvhip_comm_init(fvhip_handle h, int nranks, int rank, const void* id128)
{
	return guard([&] {
		need(h, "handle"); need(id128, "unique id");
		if(h->rankmesh && h->rank < 0 && fvhip_set_rank(h, rank, nranks)) throw std::runtime_error(g_err);
		if(nranks != h->nparts || rank != h->rank)
			throw std::invalid_argument("communicator does not match the handle's partition");
		HC(hipSetDevice(h->device));
		ncclUniqueId id;
		std::memcpy(&id, id128, sizeof(id));
		NC(ncclCommInitRank(&h->comm, nranks, id, rank));
	});
}

int fvhip_group_create(fvhip_handle* hs, int n, fvhip_group* out)
{
	return guard([&] {
		need(hs, "handles"); need(out, "group");
		if(n < 1) throw std::invalid_argument("a group needs one handle per rank of one partition");
		std::unique_ptr<fvhip_group_s> g(new fvhip_group_s());
		std::vector<int> seen(n, 0);
		for(int i = 0; i < n; i++) {
			if(!hs[i] || hs[i]->nparts != n || hs[i]->rank < 0 || hs[i]->rank >= n || seen[hs[i]->rank]++)
				throw std::invalid_argument("a group needs one handle per rank of one partition");
			g->hs.push_back(hs[i]);
		}
		for(fvhip_ctx* h : g->hs) h->in_group = true;
		*out = g.release();
	});
}

int fvhip_group_destroy(fvhip_group g) { return guard([&] { if(!g) return; for(fvhip_ctx* h : g->hs) h->in_group = false; delete g; }); }

int fvhip_group_compute_residual_device(fvhip_group g, const double* const* d_u, double* const* d_r,
                                        int gettimesteps, double* const* d_dtm, int flags)
{
	return guard([&] {
		need(g, "group");
		needEach(d_u, g->hs.size(), "u"); needEach(d_r, g->hs.size(), "residual"); if(gettimesteps) needEach(d_dtm, g->hs.size(), "dtm");
		const size_t n = g->hs.size();
		std::vector<const double*> us(d_u, d_u + n);
		std::vector<double*> rs(d_r, d_r + n), dts(n, nullptr);
		if(gettimesteps) dts.assign(d_dtm, d_dtm + n);
		fvhip_ctx::residual_seq(g->hs, us, rs, gettimesteps != 0, dts, (flags & FVHIP_RES_OVERWRITE) != 0,
		                        groupExchange(g));
		for(size_t i = 0; i < n; i++) HC(hipStreamSynchronize(g->hs[i]->stream));
	});
}

int fvhip_trace_exchange_device(fvhip_handle h, const double* d_left, double* d_right, int width)
{
	return guard([&] {
		need(h, "handle");
		need(d_left, "left trace"); need(d_right, "right trace");
		HC(hipSetDevice(h->device));
		h->trace_exchange_rccl(d_left, d_right, width);
		HC(hipStreamSynchronize(h->stream));
	});
}

int fvhip_group_trace_exchange_device(fvhip_group g, const double* const* d_left, double* const* d_right, int width)
{
	return guard([&] {
		need(g, "group");
		needEach(d_left, g->hs.size(), "left trace"); needEach(d_right, g->hs.size(), "right trace");
		const std::vector<fvhip_ctx*>& hs = g->hs;
		const size_t n = hs.size();
		std::vector<fvhip_ctx*> byrank(n);
		for(fvhip_ctx* h : hs) byrank[h->rank] = h;
		for(size_t i = 0; i < n; i++) { HC(hipSetDevice(hs[i]->device)); hs[i]->trace_pack(d_left[i], width, hs[i]->stream); }
		for(size_t i = 0; i < n; i++) HC(hipStreamSynchronize(hs[i]->stream));
		for(size_t i = 0; i < n; i++) {
			fvhip_ctx* h = hs[i];
			const Layout& L = h->L;
			HC(hipSetDevice(h->device));
			for(size_t k = 0; k < L.nbr_rank.size(); k++) {
				fvhip_ctx* q = byrank[L.nbr_rank[k]];
				const Layout& Q = q->L;
				size_t kk = 0;
				while(kk < Q.nbr_rank.size() && Q.nbr_rank[kk] != h->rank) kk++;
				if(kk == Q.nbr_rank.size()) throw std::logic_error("halo lists are not symmetric");
				const int cnt = L.ghost_start[k+1] - L.ghost_start[k];
				if(cnt != Q.send_start[kk+1] - Q.send_start[kk]) throw std::logic_error("halo sizes differ");
				if(cnt == 0) continue;
				HC(hipMemcpyAsync(h->d_tracebuf + static_cast<size_t>(width)*L.ghost_start[k],
				                  q->d_sendbuf + static_cast<size_t>(width)*Q.send_start[kk],
				                  sizeof(double)*width*static_cast<size_t>(cnt), hipMemcpyDeviceToDevice, h->stream));
			}
			h->trace_unpack(d_right[i], width, h->stream);
		}
		for(size_t i = 0; i < n; i++) HC(hipStreamSynchronize(hs[i]->stream));
	});
}

int fvhip_destroy(fvhip_handle h) { return guard([&]{ delete h; }); }

int fvhip_compute_residual_device(fvhip_handle h, const double* d_u, double* d_r, int gettimesteps,
                                  double* d_dtm, int flags)
{
	return guard([&] {
		need(h, "handle");
		need(d_u, "u"); need(d_r, "residual"); if(gettimesteps) need(d_dtm, "dtm");
		HC(hipSetDevice(h->device));
		h->use_staged = (flags & FVHIP_RES_STAGED) != 0;
		h->use_pipe = (flags & FVHIP_RES_PIPELINED) != 0;
		if(flags & FVHIP_RES_HALO_READY) h->residual_halo_ready(d_u, d_r, gettimesteps != 0, d_dtm, (flags & FVHIP_RES_OVERWRITE) != 0);
		else h->residual(d_u, d_r, gettimesteps != 0, d_dtm, (flags & FVHIP_RES_OVERWRITE) != 0);
		h->use_staged = h->use_pipe = false;
	});
}

/// host array in reference order -> device array in internal order, on the handle's stream: the rows are
/// copied as they are (one contiguous transfer) and reordered by k_gather over d_perm on the device
static void uploadInternal(fvhip_ctx* h, const double* host_ref, double* d_internal, int width) {
	const size_t n = static_cast<size_t>(h->L.ncell)*width;
	if(n == 0) return;
	double* raw = h->rawScratch(n);
	HC(hipMemcpyAsync(raw, host_ref, n*sizeof(double), hipMemcpyHostToDevice, h->stream));
	exact::launch_gather_cells(h->d_perm, raw, d_internal, h->L.ncell, width, h->stream);
	HC(hipGetLastError());
}
/// device array in internal order -> host array in reference order (k_scatter, then one transfer);
/// returns when the host array holds the values
static void downloadReference(fvhip_ctx* h, const double* d_internal, double* host_ref, int width) {
	const size_t n = static_cast<size_t>(h->L.ncell)*width;
	if(n == 0) return;
	double* raw = h->rawScratch(n);
	exact::launch_scatter_cells(h->d_perm, d_internal, raw, h->L.ncell, width, h->stream);
	HC(hipGetLastError());
	HC(hipMemcpyAsync(host_ref, raw, n*sizeof(double), hipMemcpyDeviceToHost, h->stream));
	HC(hipStreamSynchronize(h->stream));
}
/// host-side reordering of rows already on the host (internal -> reference)
static void fromInternal(fvhip_ctx* h, const double* src, double* dst, int width) {
	const int N = h->L.ncell;
	for(int c = 0; c < N; c++)
		std::memcpy(dst + static_cast<size_t>(h->L.perm[c])*width, src + static_cast<size_t>(c)*width, width*sizeof(double));
}

int fvhip_compute_residual(fvhip_handle h, const double* u, double* r, int gettimesteps, double* dtm)
{
	return guard([&] {
		need(h, "handle");
		need(u, "u"); need(r, "residual"); if(gettimesteps) need(dtm, "dtm");
		HC(hipSetDevice(h->device));
		uploadInternal(h, u, h->d_u, 4);
		uploadInternal(h, r, h->d_r, 4);
		h->residual(h->d_u, h->d_r, gettimesteps != 0, h->d_dtm, false);
		downloadReference(h, h->d_r, r, 4);
		if(gettimesteps) downloadReference(h, h->d_dtm, dtm, 1);
	});
}

int fvhip_get_gradients(fvhip_handle h, const double* u, double* grads)
{
	return guard([&] {
		need(h, "handle");
		need(u, "u"); need(grads, "grads");
		HC(hipSetDevice(h->device));
		uploadInternal(h, u, h->d_u, 4);
		h->exchange_rccl(h->d_u, 4);   // ghost rows for the border cells (partitioned handles)
		// ghost states from cell values, then the gradient scheme on CONSERVED variables
		exact::launch_prep(h->M, h->P, h->d_u, h->d_up, h->d_ubc, h->d_ug, false, h->stream);
		switch(h->cfg.gradientscheme) {
			case FVHIP_GRAD_LEASTSQUARES: exact::launch_grad_wls(h->M, h->d_u, h->d_ubc, h->d_grad, h->stream); break;
			case FVHIP_GRAD_GREENGAUSS: exact::launch_grad_gg(h->M, h->d_u, h->d_ubc, h->d_grad, h->stream); break;
			default: exact::launch_fill(h->d_grad, 0.0, 8LL*h->L.ncell, h->stream);
		}
		HC(hipGetLastError());
		downloadReference(h, h->d_grad, grads, 8);
	});
}

int fvhip_surface_data_device(fvhip_handle h, const double* d_u, int marker, double* funcs, double* faces,
                              int* nfaces)
{
	return guard([&] {
		need(h, "handle");
		need(d_u, "u"); need(funcs, "funcs");
		if(!funcs) throw std::invalid_argument("funcs must not be NULL");
		HC(hipSetDevice(h->device));
		fvhip_ctx::SurfCache& c = h->surfaceFaces(marker);
		double* u = const_cast<double*>(d_u);
		h->exchange_rccl(u, 4);   // ghost rows for the border cells' gradients (partitioned handles)
		// getGradients (flow_spatial.cpp:95-112): ghost states, then the scheme on conserved variables
		exact::launch_prep(h->M, h->P, u, h->d_up, h->d_ubc, h->d_ug, false, h->stream);
		switch(h->cfg.gradientscheme) {
			case FVHIP_GRAD_LEASTSQUARES: exact::launch_grad_wls(h->M, u, h->d_ubc, h->d_grad, h->stream); break;
			case FVHIP_GRAD_GREENGAUSS: exact::launch_grad_gg(h->M, u, h->d_ubc, h->d_grad, h->stream); break;
			default: exact::launch_fill(h->d_grad, 0.0, 8LL*h->L.ncell, h->stream);
		}
		// flowDirectionVector(aoa) with zero side-slip and getFreestreamPressure, on the host as there
		const double aoa = h->cfg.aoa;
		const double wx = std::cos(aoa)*std::cos(0.0), wy = std::sin(aoa)*std::cos(0.0);      // mathutils.hpp:67-75
		const double pinf = 1.0/(h->cfg.gamma*h->cfg.Minf*h->cfg.Minf);                          // aphysics_defs.hpp:465-467
		launch_surface(c.S, u, h->d_grad, h->P.gas, pinf, wx, wy, c.faceout, c.contrib, c.sums, h->stream);
		HC(hipGetLastError());
		if(h->comm) NC(ncclAllReduce(c.sums, c.sums, 4, ncclDouble, ncclSum, h->comm, h->stream));   // :297-299
		double s[4];
		HC(hipMemcpyAsync(s, c.sums, sizeof s, hipMemcpyDeviceToHost, h->stream));
		if(faces && c.S.n > 0)
			HC(hipMemcpyAsync(faces, c.faceout, 4*static_cast<size_t>(c.S.n)*sizeof(double), hipMemcpyDeviceToHost, h->stream));
		HC(hipStreamSynchronize(h->stream));
		funcs[0] = s[0]/s[3]; funcs[1] = s[1]/s[3]; funcs[2] = s[2]/s[3];                          // :302
		if(nfaces) *nfaces = c.S.n;
	});
}

/// this handle's owned-cell entropy sum (before the rank sum and the square root), on its stream
static double* entropySum(fvhip_ctx* h, const double* d_u)
{
	if(!h->d_ent) h->d_ent = dalloc(static_cast<size_t>(entropy_partials(h->L.ncell)) + 1, h->owned);
	// free-stream entropy on the host, as FlowOutput does (compute_freestream_state, aphysics.cpp:43-58)
	const double sinf = gd::pressure_cons(h->P.gas, h->P.uinf)/std::pow(h->P.uinf[0], h->cfg.gamma);
	double* out = h->d_ent + entropy_partials(h->L.ncell);
	launch_entropy(h->L.ncell, d_u, h->M.area, h->P.gas, sinf, h->d_ent, out, h->stream);
	HC(hipGetLastError());
	return out;
}

int fvhip_entropy_error_device(fvhip_handle h, const double* d_u, double* err)
{
	return guard([&] {
		need(h, "handle");
		need(d_u, "u");
		if(!err) throw std::invalid_argument("err must not be NULL");
		HC(hipSetDevice(h->device));
		double* out = entropySum(h, d_u);
		if(h->comm) NC(ncclAllReduce(out, out, 1, ncclDouble, ncclSum, h->comm, h->stream));   // mpi_all_reduce :49
		else if(h->halo()) throw std::runtime_error("partitioned handle: call fvhip_comm_init (or use a group) first");
		double s = 0;
		HC(hipMemcpyAsync(&s, out, sizeof s, hipMemcpyDeviceToHost, h->stream));
		HC(hipStreamSynchronize(h->stream));
		*err = std::sqrt(s);
	});
}

int fvhip_group_entropy_error_device(fvhip_group g, const double* const* d_u, double* err)
{
	return guard([&] {
		need(g, "group");
		needEach(d_u, g->hs.size(), "u");
		double tot = 0;
		for(size_t i = 0; i < g->hs.size(); i++) {          // rank order
			fvhip_ctx* h = g->hs[i];
			HC(hipSetDevice(h->device));
			double* out = entropySum(h, d_u[i]);
			double s = 0;
			HC(hipMemcpyAsync(&s, out, sizeof s, hipMemcpyDeviceToHost, h->stream));
			HC(hipStreamSynchronize(h->stream));
			tot += s;
		}
		*err = std::sqrt(tot);
	});
}

int fvhip_assemble_jacobian(fvhip_handle h, const double* u, double* diag, double* lower, double* upper)
{
	return guard([&] {
		need(h, "handle");
		need(u, "u"); need(diag, "diag"); if(h->L.ninface > 0) { need(lower, "lower"); need(upper, "upper"); }
		HC(hipSetDevice(h->device));
		const size_t N = static_cast<size_t>(h->L.ncell), Fi = static_cast<size_t>(h->L.ninface);
		uploadInternal(h, u, h->d_u, 4);
		h->exchange_rccl(h->d_u, 4);   // ghost rows: the cut-face blocks read them (partitioned handles)
		HC(hipStreamSynchronize(h->stream));
		if(!h->d_jdiag) {
			h->d_jdiag = dalloc(16*N, h->owned);
			h->d_jlo = dalloc(16*std::max<size_t>(Fi,1), h->owned);
			h->d_jup = dalloc(16*std::max<size_t>(Fi,1), h->owned);
		}
		h->assemble(h->d_u, h->d_jdiag, h->d_jlo, h->d_jup);
		// ADD_VALUES into the caller's blocks (the reference's caller zeroes them, aodesolver.cpp:456)
		std::vector<double> tmp(16*N), lo(16*Fi), up(16*Fi);
		if(Fi) {
			HC(hipMemcpyAsync(lo.data(), h->d_jlo, 16*Fi*sizeof(double), hipMemcpyDeviceToHost, h->stream));
			HC(hipMemcpyAsync(up.data(), h->d_jup, 16*Fi*sizeof(double), hipMemcpyDeviceToHost, h->stream));
		}
		downloadReference(h, h->d_jdiag, tmp.data(), 16);
		for(size_t k = 0; k < 16*N; k++) diag[k] += tmp[k];
		for(size_t k = 0; k < 16*Fi; k++) { lower[k] += lo[k]; upper[k] += up[k]; }
	});
}

int fvhip_assemble_jacobian_device(fvhip_handle h, const double* d_u, double* d_diag, double* d_lower, double* d_upper)
{
	return guard([&] {
		need(h, "handle");
		need(d_u, "u"); need(d_diag, "diag"); if(h->L.ninface > 0) { need(d_lower, "lower"); need(d_upper, "upper"); }
		HC(hipSetDevice(h->device));
		h->assemble(d_u, d_diag, d_lower, d_upper);
	});
}

int fvhip_add_pseudo_time_term_device(fvhip_handle h, double cfl, double* d_dtm, double* d_diag)
{
	return guard([&] {
		need(h, "handle");
		need(d_dtm, "dtm"); need(d_diag, "diag");
		HC(hipSetDevice(h->device));
		h->ensureJacobian();
		h->timed("k_pseudo_time", [&]{ launch_pseudo_time(h->L.ncell, h->M.area, cfl, d_dtm, d_diag, h->stream); });
		HC(hipGetLastError());
	});
}

int fvhip_block_apply_device(fvhip_handle h, const double* d_diag, const double* d_lower, const double* d_upper,
                             const double* d_x, double* d_y)
{
	return guard([&] {
		need(h, "handle");
		need(d_diag, "diag"); if(h->L.ninface > 0) { need(d_lower, "lower"); need(d_upper, "upper"); } need(d_x, "x"); need(d_y, "y");
		HC(hipSetDevice(h->device));
		h->ensureJacobian();
		h->timed("k_block_apply", [&]{ launch_block_apply(h->J, d_diag, d_lower, d_upper, d_x, d_y, h->stream); });
		HC(hipGetLastError());
	});
}

int fvhip_jacobian_pattern(fvhip_handle h, int* rowptr, int* colind)
{
	return guard([&] {
		need(h, "handle");
		need(rowptr, "rowptr"); need(colind, "colind");
		const int N = h->L.ncell, nb = h->L.nbface, Fi = h->L.ninface;
		// reference cell numbering: diagonal plus one block per interior face on each side
		std::vector<int> cnt(N, 1);
		for(int fi = 0; fi < Fi; fi++) { cnt[h->L.perm[h->L.if_L[fi]]]++; cnt[h->L.perm[h->L.if_R[fi]]]++; }
		rowptr[0] = 0;
		for(int c = 0; c < N; c++) rowptr[c+1] = rowptr[c] + cnt[c];
		std::vector<int> pos(rowptr, rowptr + N);
		for(int c = 0; c < N; c++) colind[pos[c]++] = c;
		for(int fi = 0; fi < Fi; fi++) {
			const int l = h->L.perm[h->L.if_L[fi]], r = h->L.perm[h->L.if_R[fi]];
			colind[pos[l]++] = r; colind[pos[r]++] = l;
		}
		for(int c = 0; c < N; c++) std::sort(colind + rowptr[c], colind + rowptr[c+1]);
		(void)nb;
	});
}

int fvhip_assemble_jacobian_bsr(fvhip_handle h, const double* u, const int* rowptr, const int* colind, double* vals)
{
	return guard([&] {
		need(h, "handle");
		need(u, "u"); need(rowptr, "rowptr"); need(colind, "colind"); need(vals, "vals");
		const int N = h->L.ncell, Fi = h->L.ninface;
		std::vector<double> diag(16*static_cast<size_t>(N)), lo(16*static_cast<size_t>(std::max(Fi,1))),
			up(16*static_cast<size_t>(std::max(Fi,1)));
		if(fvhip_assemble_jacobian(h, u, diag.data(), lo.data(), up.data())) throw std::runtime_error(g_err);
		auto find = [&](int row, int col) -> size_t {
			const int* b = colind + rowptr[row]; const int* e = colind + rowptr[row+1];
			const int* it = std::lower_bound(b, e, col);
			if(it == e || *it != col) throw std::runtime_error("Jacobian pattern does not match the mesh");
			return static_cast<size_t>(it - colind);
		};
		std::fill(vals, vals + 16*static_cast<size_t>(rowptr[N]), 0.0);
		for(int c = 0; c < N; c++) std::memcpy(vals + 16*find(c,c), &diag[16*static_cast<size_t>(c)], 16*sizeof(double));
		for(int fi = 0; fi < Fi; fi++) {
			const int l = h->L.perm[h->L.if_L[fi]], r = h->L.perm[h->L.if_R[fi]];
			std::memcpy(vals + 16*find(r,l), &lo[16*static_cast<size_t>(fi)], 16*sizeof(double));
			std::memcpy(vals + 16*find(l,r), &up[16*static_cast<size_t>(fi)], 16*sizeof(double));
		}
	});
}

int fvhip_matfree_set_state(fvhip_handle h, const double* u, const double* r, const double* mdt)
{
	return guard([&] {
		need(h, "handle");
		need(u, "u"); need(r, "residual"); need(mdt, "mdt");
		HC(hipSetDevice(h->device));
		const size_t N = static_cast<size_t>(h->L.ncell);
		if(!h->d_mf_u) { h->d_mf_u = dalloc(4*N, h->owned); h->d_mf_r = dalloc(4*N, h->owned); h->d_mf_mdt = dalloc(N, h->owned); }
		uploadInternal(h, u, h->d_mf_u, 4);
		uploadInternal(h, r, h->d_mf_r, 4);
		uploadInternal(h, mdt, h->d_mf_mdt, 1);
		HC(hipStreamSynchronize(h->stream));
		h->mf_u = h->d_mf_u; h->mf_r = h->d_mf_r; h->mf_mdt = h->d_mf_mdt;
	});
}

int fvhip_matfree_apply(fvhip_handle h, const double* x, double* y)
{
	return guard([&] {
		need(h, "handle");
		need(x, "x"); need(y, "y");
		HC(hipSetDevice(h->device));
		if(!h->d_mf_u) throw std::runtime_error("matrix-free operator: state not set");
		double *dx = h->d_u, *dy = h->d_r;   // scratch: the operator's state lives in d_mf_*
		uploadInternal(h, x, dx, 4);
		if(h->halo()) {
			// partitioned: the operator over all ranks (global |x|; ghost rows of the perturbed state
			// are exchanged inside the residual), as fvhip_matfree_apply_device does
			if(!h->comm) throw std::runtime_error("partitioned handle: call fvhip_comm_init first");
			sysMatfree({h}, fvhip_ctx::GroupExchange(), {dx}, {dy});
		} else h->matfree(dx, dy);
		downloadReference(h, dy, y, 4);
	});
}

int fvhip_matfree_set_state_device(fvhip_handle h, const double* d_u, const double* d_r, const double* d_mdt)
{
	return guard([&] { need(h, "handle"); h->mf_u = d_u; h->mf_r = d_r; h->mf_mdt = d_mdt; });
}

int fvhip_matfree_apply_device(fvhip_handle h, const double* d_x, double* d_y)
{
	return guard([&] {
		need(h, "handle");
		need(d_x, "x"); need(d_y, "y");
		HC(hipSetDevice(h->device));
		if(!h->halo()) { h->matfree(d_x, d_y); return; }
		if(!h->comm) throw std::runtime_error("partitioned handle: call fvhip_comm_init (or use a group) first");
		sysMatfree({h}, fvhip_ctx::GroupExchange(), {d_x}, {d_y});
	});
}

int fvhip_group_matfree_set_state_device(fvhip_group g, const double* const* d_u, const double* const* d_r,
                                         const double* const* d_mdt)
{
	return guard([&] {
		need(g, "group");
		needEach(d_u, g->hs.size(), "u"); needEach(d_r, g->hs.size(), "residual"); needEach(d_mdt, g->hs.size(), "dtm");
		for(size_t i = 0; i < g->hs.size(); i++) { g->hs[i]->mf_u = d_u[i]; g->hs[i]->mf_r = d_r[i]; g->hs[i]->mf_mdt = d_mdt[i]; }
	});
}

int fvhip_group_matfree_apply_device(fvhip_group g, const double* const* d_x, double* const* d_y)
{
	return guard([&] {
		need(g, "group");
		needEach(d_x, g->hs.size(), "x"); needEach(d_y, g->hs.size(), "y");
		const size_t n = g->hs.size();
		sysMatfree(g->hs, groupExchange(g), std::vector<const double*>(d_x, d_x + n), std::vector<double*>(d_y, d_y + n));
	});
}

int fvhip_matfree_set_eps(fvhip_handle h, double eps) { return guard([&] { need(h, "handle"); h->mf_eps = eps; }); }

int fvhip_to_internal(fvhip_handle h, const double* host_ref, double* d_internal, int width)
{
	return guard([&] {
		need(h, "handle");
		need(host_ref, "host array"); need(d_internal, "device array");
		if(width < 1) throw std::invalid_argument("width must be >= 1");
		HC(hipSetDevice(h->device));
		uploadInternal(h, host_ref, d_internal, width);
		HC(hipStreamSynchronize(h->stream));
	});
}
int fvhip_from_internal(fvhip_handle h, const double* d_internal, double* host_ref, int width)
{
	return guard([&] {
		need(h, "handle");
		need(d_internal, "device array"); need(host_ref, "host array");
		if(width < 1) throw std::invalid_argument("width must be >= 1");
		HC(hipSetDevice(h->device));
		downloadReference(h, d_internal, host_ref, width);
	});
}
int fvhip_get_permutation(fvhip_handle h, int* perm)
{
	return guard([&] { need(h, "handle"); need(perm, "perm"); std::memcpy(perm, h->L.perm.data(), h->L.perm.size()*sizeof(int)); });
}
int fvhip_device_alloc(fvhip_handle h, unsigned long long bytes, void** ptr)
{
	return guard([&] { need(h, "handle"); need(ptr, "ptr"); HC(hipSetDevice(h->device)); HC(hipMalloc(ptr, bytes)); });
}
int fvhip_device_free(fvhip_handle h, void* ptr)
{
	return guard([&] { need(h, "handle"); HC(hipSetDevice(h->device)); HC(hipFree(ptr)); });
}
int fvhip_synchronize(fvhip_handle h)
{
	return guard([&] { need(h, "handle"); HC(hipSetDevice(h->device)); HC(hipStreamSynchronize(h->stream)); });
}
void* fvhip_stream(fvhip_handle h) { return h ? static_cast<void*>(h->stream) : nullptr; }

int fvhip_profile(fvhip_handle h, int enable)
{
	return guard([&] {
		need(h, "handle");
		if(!enable && h->prof) h->collect();
		h->prof = enable != 0;
		if(enable) { h->collect(); h->acc.clear(); }
	});
}

int fvhip_kernel_times(fvhip_handle h, int maxk, char* names, int namelen, double* ms, int* counts)
{
	int n = 0;
	const int rc = guard([&] {
		need(h, "handle");
		if(maxk > 0) { need(names, "names"); need(ms, "ms"); need(counts, "counts"); }
		h->collect();
		for(auto& kv : h->acc) {
			if(n >= maxk) break;
			std::strncpy(names + static_cast<size_t>(n)*namelen, kv.first.c_str(), namelen-1);
			names[static_cast<size_t>(n)*namelen + namelen-1] = '\0';
			ms[n] = kv.second.first; counts[n] = kv.second.second;
			n++;
		}
	});
	return rc ? -1 : n;
}

/// layout statistics (include/fvhip.h fvhip_layout_stats / fvhip_layout_probe), n entries
static void layoutStats(const Layout& L, long long* s, int n)
{
	long long v[16] = {};
	v[0] = L.ncell; v[1] = L.naface; v[2] = static_cast<long long>(L.slot_L.size());
	v[3] = static_cast<long long>(L.patch_cell.size()) - 1; v[4] = L.max_slots; v[5] = L.nbface;
	v[6] = L.nghost; v[7] = static_cast<long long>(L.nbr_rank.size()); v[8] = static_cast<long long>(L.send_cells.size());
	v[9] = L.fz_ninner;
	// fused residual staging: ring-1 cells over all patches; patches staging more cells than a
	// block has threads (their staging takes two rounds); ring-2 cells; most rows one patch stages
	v[10] = static_cast<long long>(L.fz_ext.size()) - L.fz_ring2;
	const long long np = static_cast<long long>(L.patch_cell.size()) - 1;
	if(!L.fz_ext_start.empty())
		for(long long p = 0; p < np; p++) {
			const long long nl = (L.patch_cell[p+1] - L.patch_cell[p]) + (L.fz_ext_start[p+1] - L.fz_ext_start[p]);
			if(nl > SLOTS_MAX) v[11]++;
		}
	v[12] = L.fz_ring2;
	v[13] = L.fz_max_cells;
	v[14] = SLOTS_MAX;
	for(int i = 0; i < n && i < 16; i++) s[i] = v[i];
}

int fvhip_layout_stats(fvhip_handle h, long long* s)
{
	return guard([&] { need(h, "handle"); need(s, "stats"); layoutStats(h->L, s, 12); });
}

int fvhip_layout_probe(const fvhip_mesh* mesh, const fvhip_flow_config* cfg, long long* s)
{
	return guard([&] {
		if(!mesh || !cfg || !s) throw std::invalid_argument("null argument");
		checkConfig(cfg);
		const Layout L = buildLayout(topoFromMesh(*mesh), *cfg, true);
		layoutStats(L, s, 16);
	});
}

int fvhip_local_flux(int flux_type, const double* gas5, int nf, const double* ul, const double* ur,
                     const double* n, double* flux)
{
	return guard([&] {
		const gd::Gas G = gd::make_gas(gas5[0], gas5[1], gas5[2], gas5[3], gas5[4]);
		double *a, *b, *c, *d;
		HC(hipMalloc(&a, 4*sizeof(double)*nf + 8)); HC(hipMalloc(&b, 4*sizeof(double)*nf + 8));
		HC(hipMalloc(&c, 2*sizeof(double)*nf + 8)); HC(hipMalloc(&d, 4*sizeof(double)*nf + 8));
		HC(hipMemcpy(a, ul, 4*sizeof(double)*nf, hipMemcpyHostToDevice));
		HC(hipMemcpy(b, ur, 4*sizeof(double)*nf, hipMemcpyHostToDevice));
		HC(hipMemcpy(c, n, 2*sizeof(double)*nf, hipMemcpyHostToDevice));
		exact::launch_local_flux(flux_type, G, nf, a, b, c, d, nullptr);
		HC(hipGetLastError());
		HC(hipMemcpy(flux, d, 4*sizeof(double)*nf, hipMemcpyDeviceToHost));
		(void)hipFree(a); (void)hipFree(b); (void)hipFree(c); (void)hipFree(d);
	});
}

int fvhip_divsqrt_probe(int n, const double* a, const double* b, double* out)
{
	return guard([&] {
		double *da, *db, *dout;
		HC(hipMalloc(&da, sizeof(double)*n + 8)); HC(hipMalloc(&db, sizeof(double)*n + 8));
		HC(hipMalloc(&dout, 4*sizeof(double)*n + 8));
		HC(hipMemcpy(da, a, sizeof(double)*n, hipMemcpyHostToDevice));
		HC(hipMemcpy(db, b, sizeof(double)*n, hipMemcpyHostToDevice));
		exact::launch_divsqrt_probe(n, da, db, dout, nullptr);
		HC(hipGetLastError());
		HC(hipMemcpy(out, dout, 4*sizeof(double)*n, hipMemcpyDeviceToHost));
		(void)hipFree(da); (void)hipFree(db); (void)hipFree(dout);
	});
}

int fvhip_local_flux_jacobian(int flux_type, const double* gas5, int nf, const double* ul,
                              const double* ur, const double* n, double* dfdl, double* dfdr)
{
	return guard([&] {
		if(flux_type == FVHIP_FLUX_VANLEER) throw std::runtime_error(" ! VanLeerFlux: Not implemented!");
		if(flux_type == FVHIP_FLUX_AUSMPLUS) throw std::runtime_error(" ! AUSMPlusFlux: Not implemented!");
		if(flux_type < 0 || flux_type > 6) throw std::invalid_argument("unknown flux");
		const gd::Gas G = gd::make_gas(gas5[0], gas5[1], gas5[2], gas5[3], gas5[4]);
		double *a, *b, *c, *d, *e;
		HC(hipMalloc(&a, 4*sizeof(double)*nf + 8)); HC(hipMalloc(&b, 4*sizeof(double)*nf + 8));
		HC(hipMalloc(&c, 2*sizeof(double)*nf + 8)); HC(hipMalloc(&d, 16*sizeof(double)*nf + 8));
		HC(hipMalloc(&e, 16*sizeof(double)*nf + 8));
		HC(hipMemcpy(a, ul, 4*sizeof(double)*nf, hipMemcpyHostToDevice));
		HC(hipMemcpy(b, ur, 4*sizeof(double)*nf, hipMemcpyHostToDevice));
		HC(hipMemcpy(c, n, 2*sizeof(double)*nf, hipMemcpyHostToDevice));
		launch_local_jac(flux_type, G, nf, a, b, c, d, e, nullptr);
		HC(hipGetLastError());
		HC(hipMemcpy(dfdl, d, 16*sizeof(double)*nf, hipMemcpyDeviceToHost));
		HC(hipMemcpy(dfdr, e, 16*sizeof(double)*nf, hipMemcpyDeviceToHost));
		(void)hipFree(a); (void)hipFree(b); (void)hipFree(c); (void)hipFree(d); (void)hipFree(e);
	});
}

// ------------------------------------------------------------------------------------------------
// mesh builder
// ------------------------------------------------------------------------------------------------
struct fvmesh_s { MeshData raw; Mesh mesh; };

int fvmesh_read_gmsh(const char* path, fvmesh_handle* out)
{
	return guard([&] {
		std::unique_ptr<fvmesh_s> m(new fvmesh_s());
		m->raw = readGmsh2(path);
		m->mesh = buildMesh(m->raw);
		*out = m.release();
	});
}

int fvmesh_generate(int kind, int a, int b, int c, double x, double y, double z, fvmesh_handle* out)
{
	return guard([&] {
		std::unique_ptr<fvmesh_s> m(new fvmesh_s());
		if(kind == 0) m->raw = generateNacaOgrid(a, b, c, x, y, static_cast<int>(z));
		else if(kind == 1) m->raw = generateCylinderOgrid(a, b, x, y);
		else if(kind == 2) m->raw = generateFlatPlate(a, b, x, y, z);
		else if(kind == 3) m->raw = generateNacaCgrid(a, static_cast<int>(z), b, c, x, y);
		else throw std::invalid_argument("unknown mesh kind");
		m->mesh = buildMesh(m->raw);
		*out = m.release();
	});
}

int fvmesh_generate_hybrid(int nsurf, int nwake, int nquad, int nrows, double rfar,
                           double wallspacing, fvmesh_handle* out)
{
	return guard([&] {
		std::unique_ptr<fvmesh_s> m(new fvmesh_s());
		m->raw = generateNacaHybrid(nsurf, nwake, nquad, nrows, rfar, wallspacing);
		m->mesh = buildMesh(m->raw);
		*out = m.release();
	});
}

int fvmesh_amg_aggregates(fvmesh_handle m, double threshold, int* nagg, int* agg)
{
	return guard([&] {
		if(!m || !nagg) throw std::invalid_argument("null argument");
		if(!(threshold >= 0.0 && threshold < 1.0)) throw std::invalid_argument("threshold must be in [0, 1)");
		const Mesh& M = m->mesh;
		const int N = M.md.nelem, nb = M.md.nbface;
		// the cell graph over interior faces, columns ascending (ctx.hpp ensureAmg's graph in this cell order)
		std::vector<std::vector<std::pair<int,double>>> adj(static_cast<size_t>(N));
		for(int f = nb; f < M.naface - M.nconnface; f++) {
			const int L = M.intfac[4*static_cast<size_t>(f)], R = M.intfac[4*static_cast<size_t>(f)+1];
			if(R >= N) continue;
			const double dx = M.rc[2*static_cast<size_t>(L)] - M.rc[2*static_cast<size_t>(R)];
			const double dy = M.rc[2*static_cast<size_t>(L)+1] - M.rc[2*static_cast<size_t>(R)+1];
			const double w = M.facemetric[3*static_cast<size_t>(f)+2]/std::sqrt(dx*dx + dy*dy);
			adj[L].push_back({R, w}); adj[R].push_back({L, w});
		}
		AmgGraph g;
		g.n = N;
		g.rowptr.assign(static_cast<size_t>(N) + 1, 0);
		for(int c = 0; c < N; c++) {
			std::sort(adj[c].begin(), adj[c].end());
			g.dblk.push_back(c);
			for(const auto& e : adj[c]) { g.col.push_back(e.first); g.w.push_back(e.second); g.blk.push_back(0); }
			g.rowptr[c+1] = static_cast<int>(g.col.size());
		}
		const AmgLevelHost H = amgCoarsen(g, threshold);
		*nagg = H.n;
		if(agg) std::copy(H.agg.begin(), H.agg.end(), agg);
	});
}

int fvmesh_write_gmsh(fvmesh_handle m, const char* path) { return guard([&] { writeGmsh2(m->raw, path); }); }
int fvmesh_destroy(fvmesh_handle m) { return guard([&] { delete m; }); }

int fvmesh_partition_trivial(int nelem, int nranks, int* elemdist)
{
	return guard([&] {
		const std::vector<int> d = partitionTrivial(nelem, nranks);
		std::memcpy(elemdist, d.data(), d.size()*sizeof(int));
	});
}

int fvmesh_restrict(fvmesh_handle g, const int* elemdist, int rank, fvmesh_handle* out)
{
	return guard([&] {
		if(!g || !elemdist || !out) throw std::invalid_argument("null argument");
		std::unique_ptr<fvmesh_s> m(new fvmesh_s());
		m->mesh = restrictMesh(g->mesh, elemdist, rank);
		m->raw = m->mesh.md;
		*out = m.release();
	});
}

int fvmesh_global_elem_index(fvmesh_handle h, int* gidx)
{
	return guard([&] {
		const Mesh& M = h->mesh;
		for(int i = 0; i < M.md.nelem; i++) gidx[i] = M.globalElemIndex.empty() ? i : M.globalElemIndex[i];
	});
}

int fvmesh_view(fvmesh_handle h, fvhip_mesh* v)
{
	return guard([&] {
		const Mesh& M = h->mesh;
		v->nelem = M.md.nelem; v->npoin = M.md.npoin; v->nbface = M.md.nbface; v->naface = M.naface;
		v->nconnface = M.nconnface; v->maxnnode = M.md.maxnnode; v->maxnfael = M.md.maxnfael; v->nbtag = M.md.nbtag;
		v->coords = M.md.coords.data(); v->inpoel = M.md.inpoel.data(); v->nnode = M.md.nnode.data();
		v->esuel = M.esuel.data(); v->elemface = M.elemface.data(); v->intfac = M.intfac.data();
		v->btags = M.btags.data(); v->facemetric = M.facemetric.data(); v->area = M.area.data();
		v->rc = M.rc.data(); v->rcbp = M.rcbp.data(); v->gr = M.gr.data();
		v->connface = M.connface.empty() ? nullptr : M.connface.data();
	});
}

int fvmesh_raw_info(fvmesh_handle h, int* info)
{
	return guard([&] {
		info[0] = h->raw.npoin; info[1] = h->raw.nelem; info[2] = h->raw.maxnnode;
		info[3] = h->raw.nbface; info[4] = h->raw.nbtag;
	});
}

int fvmesh_raw_arrays(fvmesh_handle h, double* coords, int* inpoel, int* nnode, int* bface)
{
	return guard([&] {
		const MeshData& r = h->raw;
		std::memcpy(coords, r.coords.data(), r.coords.size()*sizeof(double));
		std::memcpy(inpoel, r.inpoel.data(), r.inpoel.size()*sizeof(int));
		std::memcpy(nnode, r.nnode.data(), r.nnode.size()*sizeof(int));
		std::memcpy(bface, r.bface.data(), r.bface.size()*sizeof(int));
	});
}

}
