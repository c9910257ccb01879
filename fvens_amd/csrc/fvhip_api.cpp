/** \file fvhip_api.cpp
 * \brief Implementation of the C-ABI in include/fvhip.h: device-resident discretisation,
 *   host<->device plumbing with the reference's cell numbering, kernel timing, mesh builder.
 * No exception crosses the ABI; errors become a nonzero return and fvhip_last_error().
 */
#include "../../include/fvhip.h"
#include "layout.hpp"
#include "kernels.hpp"
#include "jacobian.hpp"
#include "mesh.hpp"
#include "partition.hpp"
#include "halo.hpp"
#include "ode.hpp"
#include <rccl/rccl.h>

#include <hip/hip_runtime.h>
#include <cstring>
#include <algorithm>
#include <cmath>
#include <string>
#include <vector>
#include <map>
#include <stdexcept>
#include <memory>
#include <functional>

using namespace fvhip;

namespace {

thread_local std::string g_err;

struct HipError : std::runtime_error { using std::runtime_error::runtime_error; };

inline void hipCheck(hipError_t e, const char* what) {
	if(e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}
#define HC(x) hipCheck((x), #x)

inline void ncclCheck(ncclResult_t e, const char* what) {
	if(e != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(e));
}
#define NC(x) ncclCheck((x), #x)

template <typename F>
int guard(F&& f) {
	try { f(); return 0; }
	catch(const std::exception& e) { g_err = e.what(); return 1; }
	catch(...) { g_err = "unknown error"; return 1; }
}

template <typename T>
T* upload(const std::vector<T>& v, std::vector<void*>& owned) {
	if(v.empty()) return nullptr;
	void* p = nullptr;
	HC(hipMalloc(&p, v.size()*sizeof(T)));
	HC(hipMemcpy(p, v.data(), v.size()*sizeof(T), hipMemcpyHostToDevice));
	owned.push_back(p);
	return static_cast<T*>(p);
}

double* dalloc(size_t n, std::vector<void*>& owned) {
	if(n == 0) n = 1;
	void* p = nullptr;
	HC(hipMalloc(&p, n*sizeof(double)));
	owned.push_back(p);
	return static_cast<double*>(p);
}

/// interleave int pairs / 4-tuples for vector loads
std::vector<int> pack2(const std::vector<int>& a, const std::vector<int>& b) {
	std::vector<int> o(2*a.size());
	for(size_t i = 0; i < a.size(); i++) { o[2*i] = a[i]; o[2*i+1] = b[i]; }
	return o;
}

}

struct fvhip_ctx
{
	int device = 0;
	hipStream_t stream = nullptr;
	fvhip_flow_config cfg{};
	std::vector<int> bc_type, bc_tag;
	std::vector<double> bc_vals;
	Layout L;
	DevMesh M{};
	DevPhys P{};
	std::vector<void*> owned;
	int* d_perm = nullptr;
	// state scratch
	double *d_u = nullptr, *d_up = nullptr, *d_grad = nullptr, *d_lgrad = nullptr, *d_phi = nullptr;
	double *d_ubc = nullptr, *d_ug = nullptr, *d_r = nullptr, *d_dtm = nullptr;
	// mat-free state
	double *d_mf_u = nullptr, *d_mf_r = nullptr, *d_mf_mdt = nullptr, *d_mf_aux = nullptr, *d_mf_y = nullptr;
	double mf_eps = 1e-7;
	const double *mf_u = nullptr, *mf_r = nullptr, *mf_mdt = nullptr;   // device state of the operator
	double *d_part = nullptr, *d_pm = nullptr;
	double *d_rn_part = nullptr, *d_rn = nullptr;   // residual-norm reduction of the explicit driver
	// Jacobian
	JacMesh J{};
	bool jac_ready = false;
	double *d_jb = nullptr, *d_jlo = nullptr, *d_jup = nullptr, *d_jdiag = nullptr;
	std::vector<double> h_stage;
	// partitioned meshes: halo exchange with the neighbour ranks (RCCL, or in-process for a group)
	int rank = 0, nparts = 1;
	bool use_staged = false;      ///< force the staged (gradient + sweep) path even if fused applies
	ncclComm_t comm = nullptr;
	bool in_group = false;
	int* d_send = nullptr;
	int* d_border = nullptr;
	int nborder = 0;
	double* d_sendbuf = nullptr;
	int nsend = 0;
	// profiling
	bool prof = false;
	struct Rec { std::string name; hipEvent_t a, b; };
	std::vector<Rec> recs;
	std::map<std::string, std::pair<double,int>> acc;

	~fvhip_ctx() {
		(void)hipSetDevice(device);
		if(comm) (void)ncclCommDestroy(comm);
		for(auto& r : recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
		for(void* p : owned) (void)hipFree(p);
		if(stream) (void)hipStreamDestroy(stream);
	}

	template <typename F>
	void timed(const std::string& name, F&& launch) {
		if(!prof) { launch(); return; }
		Rec r; r.name = name;
		HC(hipEventCreate(&r.a)); HC(hipEventCreate(&r.b));
		HC(hipEventRecord(r.a, stream));
		launch();
		HC(hipEventRecord(r.b, stream));
		recs.push_back(r);
	}
	void collect() {
		HC(hipStreamSynchronize(stream));
		for(auto& r : recs) {
			float ms = 0;
			HC(hipEventElapsedTime(&ms, r.a, r.b));
			auto& a = acc[r.name]; a.first += ms; a.second += 1;
			(void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b);
		}
		recs.clear();
	}

	/// kernels of the selected numerics mode (exact: bitwise parity; fast: stated tolerance)
#define KOPS(fn) (cfg.fast_math ? fast::fn : exact::fn)
	int recKind() const {
		if(!cfg.order2) return SR_FIRST;
		return cfg.reconstruction == FVHIP_REC_VANALBADA ? SR_MUSCL : SR_LINEAR;
	}
	int viscKind() const {
		if(!cfg.viscous_sim) return SV_NONE;
		return cfg.const_visc ? SV_CONST : SV_SUTHERLAND;
	}

	bool halo() const { return !L.nbr_rank.empty(); }
	int ntotal() const { return L.ncell + L.nghost; }

	// --- residual stages (FlowFV::compute_residual, flow_spatial.cpp:636-816); between them the
	// ghost rows of u, of the gradients and of limiter data are exchanged on partitioned meshes ---
	void stage_gradients(const double* u) {
		if(L.nghost > 0)
			timed("k_ghost_prim", [&]{ launch_cons2prim_rows(P.gas, u, d_up, L.ncell, L.nghost, stream); });
		if(cfg.gradientscheme == FVHIP_GRAD_LEASTSQUARES) {
			timed("k_prep_grad_wls", [&]{ KOPS(launch_prep_grad_wls)(M, P, u, d_up, d_ubc, d_ug, d_grad, stream); });
		} else {
			timed("k_prep", [&]{ KOPS(launch_prep)(M, P, u, d_up, d_ubc, d_ug, true, stream); });
			if(cfg.gradientscheme == FVHIP_GRAD_GREENGAUSS)
				timed("k_grad_gg", [&]{ KOPS(launch_grad_gg)(M, d_up, d_ug, d_grad, stream); });
			else KOPS(launch_fill)(d_grad, 0.0, 8LL*ntotal(), stream);
		}
	}
	bool limited() const {
		return cfg.reconstruction == FVHIP_REC_BARTHJESPERSEN || cfg.reconstruction == FVHIP_REC_VENKATAKRISHNAN;
	}
	void stage_limiter() {
		const int venk = cfg.reconstruction == FVHIP_REC_VENKATAKRISHNAN;
		timed("k_limiter", [&]{ KOPS(launch_limiter)(M, P, venk, d_up, d_ug, d_grad, d_phi, stream); });
	}
	void stage_weno() { timed("k_weno", [&]{ KOPS(launch_weno)(M, P, d_grad, d_lgrad, stream); }); }
	void stage_sweep(const double* u, double* r, bool dt, double* dtm, bool overwrite) {
		const int rk = recKind();
		SweepBuffers B{};
		B.u = u; B.r = r; B.dtm = dtm; B.overwrite = overwrite ? 1 : 0;
		if(rk != SR_FIRST) {
			B.up = d_up; B.grad = d_grad; B.rgrad = d_grad; B.ubc = d_ubc; B.ug = d_ug;
			if(limited()) B.phi = d_phi;
			if(cfg.reconstruction == FVHIP_REC_WENO) B.rgrad = d_lgrad;
		}
		const char* nm = nullptr;
		// name is only known after launch; record under a generic label then rename
		timed("k_sweep", [&]{ nm = KOPS(launch_sweep)(M, P, B, cfg.conv_numflux, rk, viscKind(), dt, stream); });
		if(prof && !recs.empty() && recs.back().name == "k_sweep" && nm) recs.back().name = nm;
		HC(hipGetLastError());
	}

	void stage_border_gradients(const double* u) {
		timed("k_grad_wls_list", [&]{ KOPS(launch_grad_wls_list)(M, P, u, d_border, nborder, d_grad, stream); });
	}

	/// one-launch residual (WLS + MUSCL / unlimited linear, inviscid)
	bool fused() const { return !L.fz_ext_start.empty() && !use_staged; }
	void stage_fused(const double* u, double* r, bool dt, double* dtm, bool overwrite) {
		SweepBuffers B{};
		B.u = u; B.r = r; B.dtm = dtm; B.overwrite = overwrite ? 1 : 0;
		B.grad = d_grad;     // received gradients of ghost cells (partitioned meshes)
		const char* nm = nullptr;
		timed("k_residual_wls", [&]{ nm = KOPS(launch_residual_wls)(M, P, B, cfg.conv_numflux, recKind(), dt, stream); });
		if(prof && !recs.empty() && recs.back().name == "k_residual_wls" && nm) recs.back().name = nm;
		HC(hipGetLastError());
	}

	/// pack the rows of `arr` (width doubles per cell) that the neighbours hold as ghosts
	void pack(const double* arr, int width) {
		timed("k_pack", [&]{ launch_pack_rows(d_send, nsend, arr, width, d_sendbuf, stream); });
	}
	/// RCCL point-to-point exchange with every neighbour rank, on this handle's stream
	void exchange_rccl(double* arr, int width) {
		if(!halo()) return;
		if(!comm) throw std::runtime_error("partitioned handle: call fvhip_comm_init (or use a group) first");
		pack(arr, width);
		NC(ncclGroupStart());
		for(size_t k = 0; k < L.nbr_rank.size(); k++) {
			const int q = L.nbr_rank[k];
			const size_t ns = static_cast<size_t>(L.send_start[k+1] - L.send_start[k]);
			const size_t ng = static_cast<size_t>(L.ghost_start[k+1] - L.ghost_start[k]);
			NC(ncclSend(d_sendbuf + static_cast<size_t>(width)*L.send_start[k], width*ns, ncclDouble, q, comm, stream));
			NC(ncclRecv(arr + static_cast<size_t>(width)*(L.ncell + L.ghost_start[k]), width*ng, ncclDouble, q, comm, stream));
		}
		NC(ncclGroupEnd());
	}

	/// the device sweep: -r(u) added (or written) into r, time steps into dtm. On a partitioned
	/// mesh u must have room for the ghost rows (ncell+nghost rows), which this fills.
	void residual(const double* u, double* r, bool dt, double* dtm, bool overwrite) {
		std::vector<fvhip_ctx*> one{this};
		residual_seq(one, {u}, {r}, dt, {dtm}, overwrite, GroupExchange());
	}

	typedef std::function<double*(size_t)> ArrayOf;
	typedef std::function<void(const ArrayOf&, int)> GroupExchange;

	/// The residual as a sequence of stages over one or several handles (several: the ranks of a
	/// partition held by one process, exchanging through device copies, see fvhip_group_*)
	static void residual_seq(std::vector<fvhip_ctx*>& hs, const std::vector<const double*>& us,
	                         const std::vector<double*>& rs, bool dt, const std::vector<double*>& dts,
	                         bool overwrite, const GroupExchange& exg) {
		auto exchange = [&](const ArrayOf& arr_of, int width) {
			if(exg) { exg(arr_of, width); return; }
			for(size_t i = 0; i < hs.size(); i++) hs[i]->exchange_rccl(arr_of(i), width);
		};
		fvhip_ctx* h0 = hs[0];
		if(h0->fused()) {
			if(h0->halo()) {
				// ghost rows of u, then the gradients of the cells other ranks hold as ghosts
				exchange([&](size_t i) { return const_cast<double*>(us[i]); }, 4);
				for(size_t i = 0; i < hs.size(); i++) hs[i]->stage_border_gradients(us[i]);
				exchange([&](size_t i) { return hs[i]->d_grad; }, 8);
			}
			for(size_t i = 0; i < hs.size(); i++) hs[i]->stage_fused(us[i], rs[i], dt, dts[i], overwrite);
			return;
		}
		exchange([&](size_t i) { return const_cast<double*>(us[i]); }, 4);
		if(h0->recKind() != SR_FIRST) {
			for(size_t i = 0; i < hs.size(); i++) hs[i]->stage_gradients(us[i]);
			exchange([&](size_t i) { return hs[i]->d_grad; }, 8);
			if(h0->limited()) {
				for(fvhip_ctx* h : hs) h->stage_limiter();
				exchange([&](size_t i) { return hs[i]->d_phi; }, 4);
			}
			if(h0->cfg.reconstruction == FVHIP_REC_WENO) {
				for(fvhip_ctx* h : hs) h->stage_weno();
				exchange([&](size_t i) { return hs[i]->d_lgrad; }, 8);
			}
		}
		for(size_t i = 0; i < hs.size(); i++) hs[i]->stage_sweep(us[i], rs[i], dt, dts[i], overwrite);
	}

	/// face-ordered mesh view and block buffers for the Jacobian, built on first use
	void ensureJacobian() {
		if(nparts > 1) throw std::runtime_error("Jacobian assembly on partitioned meshes is not built yet");
		const int jf = cfg.conv_numflux_jac;
		if(jf == FVHIP_FLUX_VANLEER) throw std::runtime_error(" ! VanLeerFlux: Not implemented!");   // anumericalflux.cpp:253-257
		if(jf == FVHIP_FLUX_AUSMPLUS) throw std::runtime_error(" ! AUSMPlusFlux: Not implemented!"); // :556-560
		if(jf < 0 || jf > 6) throw std::invalid_argument("unknown Jacobian flux");
		for(int i = 0; i < cfg.nbc; i++)
			if(bc_type[i] == FVHIP_BC_SUBSONIC_INFLOW)   // InFlow::computeGhostStateAndJacobian, abc.cpp:178-185
				throw std::runtime_error("subsonic inflow BC has no Jacobian (Not implemented!)");
		if(jac_ready) return;
		auto& o = owned;
		J.ncell = L.ncell; J.nbface = L.nbface; J.ninface = L.ninface;
		J.if_LR = reinterpret_cast<const int2*>(upload(pack2(L.if_L, L.if_R), o));
		J.if_n = reinterpret_cast<const double2*>(upload(L.if_n, o));
		J.if_len = upload(L.if_len, o);
		J.bf_L = M.bf_L; J.bf_bc = M.bf_bc; J.bf_n = M.bf_n; J.bf_rcbp = M.bf_rcbp; J.rc = M.rc;
		J.bf_len = upload(L.bf_len, o);
		J.cell_rfaces = reinterpret_cast<const int4*>(upload(L.cell_rfaces, o));
		J.cell_nbr_fo = M.cell_nbr_fo;
		d_jb = dalloc(16*static_cast<size_t>(std::max(L.nbface,1)), o);
		jac_ready = true;
	}

	/// Spatial::assemble_jacobian into (diag internal order, lower/upper reference face order)
	void assemble(const double* u, double* diag, double* lower, double* upper) {
		ensureJacobian();
		timed("k_jac_faces", [&]{ launch_jac_faces(J, P, cfg.conv_numflux_jac, viscKind(), u, d_jb, lower, upper, stream); });
		timed("k_jac_diag", [&]{ launch_jac_diag(J, d_jb, lower, upper, diag, stream); });
		HC(hipGetLastError());
	}

	/// MatrixFreeSpatialJacobian::apply on device vectors (internal order)
	void matfree(const double* x, double* y) {
		if(nparts > 1) throw std::runtime_error("matrix-free operator on partitioned meshes is not built yet");
		if(!mf_u || !mf_r || !mf_mdt) throw std::runtime_error("matrix-free operator: state not set");
		const size_t N = static_cast<size_t>(L.ncell);
		if(!d_part) { d_part = dalloc(mf_partials(), owned); d_pm = dalloc(2, owned); }
		if(!d_mf_aux) { d_mf_aux = dalloc(4*N, owned); d_mf_y = dalloc(4*N, owned); }
		timed("k_mf_norm", [&]{ launch_mf_norm(4LL*L.ncell, x, mf_eps, d_part, d_pm, stream); });
		timed("k_mf_perturb", [&]{ launch_mf_perturb(4LL*L.ncell, mf_u, x, d_pm, d_mf_aux, stream); });
		residual(d_mf_aux, d_mf_y, false, nullptr, true);
		timed("k_mf_combine", [&]{ launch_mf_combine(L.ncell, mf_mdt, x, d_mf_y, mf_r, d_pm, y, stream); });
		HC(hipGetLastError());
	}
};

extern "C" {

const char* fvhip_last_error(void) { return g_err.c_str(); }
const char* fvhip_version(void) { return "fvhip 0.1 (gfx950)"; }
int fvhip_device_count(void) {
	int n = 0;
	if(hipGetDeviceCount(&n) != hipSuccess) return 0;
	return n;
}

static void checkConfig(const fvhip_flow_config* cfg)
{
	if(cfg->nbc > MAXBC) throw std::invalid_argument("too many boundary conditions");
	if(cfg->conv_numflux < 0 || cfg->conv_numflux > 6) throw std::invalid_argument("unknown flux"); // afactory.cpp:78-80
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
		M.fz_gnbr = reinterpret_cast<const int4*>(upload(L.fz_gnbr, o));
		M.fz_slot_lr = reinterpret_cast<const int2*>(upload(L.fz_slot_lr, o));
		M.fz_max_cells = L.fz_max_cells;
	}
	h->d_perm = upload(L.perm, o);
	h->nsend = static_cast<int>(L.send_cells.size());
	h->nborder = static_cast<int>(L.border_cells.size());
	if(h->nborder > 0) h->d_border = upload(L.border_cells, o);
	if(h->nsend > 0) {
		h->d_send = upload(L.send_cells, o);
		h->d_sendbuf = dalloc(8*static_cast<size_t>(h->nsend), o);
	}

	DevPhys& P = h->P;
	P.gas = gd::Gas{cfg->gamma, cfg->Minf, cfg->Tinf, cfg->Reinf, cfg->Pr, 110.5};
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
	h->h_stage.resize(16*N);
	return h.release();
}

int fvhip_create(const fvhip_mesh* mesh, const fvhip_flow_config* cfg, int device, fvhip_handle* out)
{
	return guard([&] {
		if(!mesh || !cfg || !out) throw std::invalid_argument("null argument");
		*out = createCtx(topoFromMesh(*mesh), cfg, device);
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

int fvhip_partition_rcb(const fvhip_mesh* mesh, int nparts, int* part)
{
	return guard([&] {
		const std::vector<int> p = partitionRCB(mesh->rc, mesh->nelem, nparts);
		std::memcpy(part, p.data(), p.size()*sizeof(int));
	});
}

int fvhip_partition_info(const fvhip_mesh* mesh, const int* part, int rank, int* counts, int* cell_global,
                         int* nbr_rank, int* ghost_start, int* send_start, int* send_global)
{
	return guard([&] {
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

int fvhip_comm_unique_id(void* id128)
{
	return guard([&] {
		ncclUniqueId id;
		NC(ncclGetUniqueId(&id));
		std::memcpy(id128, &id, sizeof(id));
	});
}

int fvhip_comm_init(fvhip_handle h, int nranks, int rank, const void* id128)
{
	return guard([&] {
		if(nranks != h->nparts || rank != h->rank)
			throw std::invalid_argument("communicator does not match the handle's partition");
		HC(hipSetDevice(h->device));
		ncclUniqueId id;
		std::memcpy(&id, id128, sizeof(id));
		NC(ncclCommInitRank(&h->comm, nranks, id, rank));
	});
}

struct fvhip_group_s { std::vector<fvhip_ctx*> hs; };

int fvhip_group_create(fvhip_handle* hs, int n, fvhip_group* out)
{
	return guard([&] {
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

int fvhip_group_destroy(fvhip_group g) { return guard([&] { for(fvhip_ctx* h : g->hs) h->in_group = false; delete g; }); }

int fvhip_group_compute_residual_device(fvhip_group g, const double* const* d_u, double* const* d_r,
                                        int gettimesteps, double* const* d_dtm, int flags)
{
	return guard([&] {
		const size_t n = g->hs.size();
		std::vector<fvhip_ctx*> byrank(n);
		for(fvhip_ctx* h : g->hs) byrank[h->rank] = h;
		// in-process exchange: pack everywhere, then copy each neighbour's packed rows into the ghost block
		auto exg = [&](const fvhip_ctx::ArrayOf& arr_of, int width) {
			for(size_t i = 0; i < n; i++) if(g->hs[i]->halo()) { HC(hipSetDevice(g->hs[i]->device)); g->hs[i]->pack(arr_of(i), width); }
			for(size_t i = 0; i < n; i++) HC(hipStreamSynchronize(g->hs[i]->stream));
			for(size_t i = 0; i < n; i++) {
				fvhip_ctx* h = g->hs[i];
				const Layout& L = h->L;
				for(size_t k = 0; k < L.nbr_rank.size(); k++) {
					fvhip_ctx* q = byrank[L.nbr_rank[k]];
					const Layout& Q = q->L;
					size_t kk = 0;
					while(kk < Q.nbr_rank.size() && Q.nbr_rank[kk] != h->rank) kk++;
					if(kk == Q.nbr_rank.size()) throw std::logic_error("halo lists are not symmetric");
					const int cnt = L.ghost_start[k+1] - L.ghost_start[k];
					if(cnt != Q.send_start[kk+1] - Q.send_start[kk]) throw std::logic_error("halo sizes differ");
					HC(hipMemcpyAsync(arr_of(i) + static_cast<size_t>(width)*(L.ncell + L.ghost_start[k]),
					                  q->d_sendbuf + static_cast<size_t>(width)*Q.send_start[kk],
					                  sizeof(double)*width*static_cast<size_t>(cnt), hipMemcpyDeviceToDevice, h->stream));
				}
			}
			for(size_t i = 0; i < n; i++) HC(hipStreamSynchronize(g->hs[i]->stream));
		};
		std::vector<const double*> us(d_u, d_u + n);
		std::vector<double*> rs(d_r, d_r + n), dts(n, nullptr);
		if(gettimesteps) dts.assign(d_dtm, d_dtm + n);
		fvhip_ctx::residual_seq(g->hs, us, rs, gettimesteps != 0, dts, (flags & FVHIP_RES_OVERWRITE) != 0, exg);
		for(size_t i = 0; i < n; i++) HC(hipStreamSynchronize(g->hs[i]->stream));
	});
}

int fvhip_destroy(fvhip_handle h) { return guard([&]{ delete h; }); }

int fvhip_compute_residual_device(fvhip_handle h, const double* d_u, double* d_r, int gettimesteps,
                                  double* d_dtm, int flags)
{
	return guard([&] {
		HC(hipSetDevice(h->device));
		h->use_staged = (flags & FVHIP_RES_STAGED) != 0;
		h->residual(d_u, d_r, gettimesteps != 0, d_dtm, (flags & FVHIP_RES_OVERWRITE) != 0);
		h->use_staged = false;
	});
}

static void toInternal(fvhip_ctx* h, const double* src, double* dst, int width) {
	const int N = h->L.ncell;
	for(int c = 0; c < N; c++)
		std::memcpy(dst + static_cast<size_t>(c)*width, src + static_cast<size_t>(h->L.perm[c])*width, width*sizeof(double));
}
static void fromInternal(fvhip_ctx* h, const double* src, double* dst, int width) {
	const int N = h->L.ncell;
	for(int c = 0; c < N; c++)
		std::memcpy(dst + static_cast<size_t>(h->L.perm[c])*width, src + static_cast<size_t>(c)*width, width*sizeof(double));
}

int fvhip_compute_residual(fvhip_handle h, const double* u, double* r, int gettimesteps, double* dtm)
{
	return guard([&] {
		HC(hipSetDevice(h->device));
		const size_t N = static_cast<size_t>(h->L.ncell);
		std::vector<double>& st = h->h_stage;
		toInternal(h, u, st.data(), 4);
		HC(hipMemcpyAsync(h->d_u, st.data(), 4*N*sizeof(double), hipMemcpyHostToDevice, h->stream));
		HC(hipStreamSynchronize(h->stream));
		toInternal(h, r, st.data(), 4);
		HC(hipMemcpyAsync(h->d_r, st.data(), 4*N*sizeof(double), hipMemcpyHostToDevice, h->stream));
		h->residual(h->d_u, h->d_r, gettimesteps != 0, h->d_dtm, false);
		HC(hipMemcpyAsync(st.data(), h->d_r, 4*N*sizeof(double), hipMemcpyDeviceToHost, h->stream));
		HC(hipStreamSynchronize(h->stream));
		fromInternal(h, st.data(), r, 4);
		if(gettimesteps) {
			HC(hipMemcpyAsync(st.data(), h->d_dtm, N*sizeof(double), hipMemcpyDeviceToHost, h->stream));
			HC(hipStreamSynchronize(h->stream));
			fromInternal(h, st.data(), dtm, 1);
		}
	});
}

int fvhip_get_gradients(fvhip_handle h, const double* u, double* grads)
{
	return guard([&] {
		HC(hipSetDevice(h->device));
		const size_t N = static_cast<size_t>(h->L.ncell);
		std::vector<double>& st = h->h_stage;
		toInternal(h, u, st.data(), 4);
		HC(hipMemcpyAsync(h->d_u, st.data(), 4*N*sizeof(double), hipMemcpyHostToDevice, h->stream));
		// ghost states from cell values, then the gradient scheme on CONSERVED variables
		exact::launch_prep(h->M, h->P, h->d_u, h->d_up, h->d_ubc, h->d_ug, false, h->stream);
		switch(h->cfg.gradientscheme) {
			case FVHIP_GRAD_LEASTSQUARES: exact::launch_grad_wls(h->M, h->d_u, h->d_ubc, h->d_grad, h->stream); break;
			case FVHIP_GRAD_GREENGAUSS: exact::launch_grad_gg(h->M, h->d_u, h->d_ubc, h->d_grad, h->stream); break;
			default: exact::launch_fill(h->d_grad, 0.0, 8LL*h->L.ncell, h->stream);
		}
		HC(hipGetLastError());
		HC(hipMemcpyAsync(st.data(), h->d_grad, 8*N*sizeof(double), hipMemcpyDeviceToHost, h->stream));
		HC(hipStreamSynchronize(h->stream));
		fromInternal(h, st.data(), grads, 8);
	});
}

int fvhip_assemble_jacobian(fvhip_handle h, const double* u, double* diag, double* lower, double* upper)
{
	return guard([&] {
		HC(hipSetDevice(h->device));
		const size_t N = static_cast<size_t>(h->L.ncell), Fi = static_cast<size_t>(h->L.ninface);
		std::vector<double>& st = h->h_stage;
		toInternal(h, u, st.data(), 4);
		HC(hipMemcpyAsync(h->d_u, st.data(), 4*N*sizeof(double), hipMemcpyHostToDevice, h->stream));
		HC(hipStreamSynchronize(h->stream));
		if(!h->d_jdiag) {
			h->d_jdiag = dalloc(16*N, h->owned);
			h->d_jlo = dalloc(16*std::max<size_t>(Fi,1), h->owned);
			h->d_jup = dalloc(16*std::max<size_t>(Fi,1), h->owned);
		}
		h->assemble(h->d_u, h->d_jdiag, h->d_jlo, h->d_jup);
		// ADD_VALUES into the caller's blocks (the reference's caller zeroes them, aodesolver.cpp:456)
		std::vector<double> dg(16*N), tmp(16*N), lo(16*Fi), up(16*Fi);
		HC(hipMemcpyAsync(dg.data(), h->d_jdiag, 16*N*sizeof(double), hipMemcpyDeviceToHost, h->stream));
		if(Fi) {
			HC(hipMemcpyAsync(lo.data(), h->d_jlo, 16*Fi*sizeof(double), hipMemcpyDeviceToHost, h->stream));
			HC(hipMemcpyAsync(up.data(), h->d_jup, 16*Fi*sizeof(double), hipMemcpyDeviceToHost, h->stream));
		}
		HC(hipStreamSynchronize(h->stream));
		fromInternal(h, dg.data(), tmp.data(), 16);
		for(size_t k = 0; k < 16*N; k++) diag[k] += tmp[k];
		for(size_t k = 0; k < 16*Fi; k++) { lower[k] += lo[k]; upper[k] += up[k]; }
	});
}

int fvhip_assemble_jacobian_device(fvhip_handle h, const double* d_u, double* d_diag, double* d_lower, double* d_upper)
{
	return guard([&] {
		HC(hipSetDevice(h->device));
		h->assemble(d_u, d_diag, d_lower, d_upper);
	});
}

int fvhip_add_pseudo_time_term_device(fvhip_handle h, double cfl, double* d_dtm, double* d_diag)
{
	return guard([&] {
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
		HC(hipSetDevice(h->device));
		h->ensureJacobian();
		h->timed("k_block_apply", [&]{ launch_block_apply(h->J, d_diag, d_lower, d_upper, d_x, d_y, h->stream); });
		HC(hipGetLastError());
	});
}

int fvhip_jacobian_pattern(fvhip_handle h, int* rowptr, int* colind)
{
	return guard([&] {
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

int fvhip_steady_forward_euler_device(fvhip_handle h, double* d_u, double cfl, double tol, int maxiter,
                                      int* steps, double* resratio, double* reshistory)
{
	return guard([&] {
		HC(hipSetDevice(h->device));
		if(h->nparts > 1) throw std::runtime_error("forward Euler driver: single-domain handles only");
		const int N = h->L.ncell;
		if(!h->d_rn) { h->d_rn_part = dalloc(resnorm_partials(), h->owned); h->d_rn = dalloc(1, h->owned); }
		double* part = h->d_rn_part;
		double* dn = h->d_rn;
		double resi = 1.0, initres = 1.0;
		int step = 0;
		while(resi/initres > tol && step < maxiter) {
			h->residual(d_u, h->d_r, true, h->d_dtm, true);       // r = 0 + (-r(u)), aodesolver.cpp:180-189
			launch_fe_update(N, h->d_r, h->d_dtm, h->M.area, cfl, d_u, h->stream);
			launch_resnorm(N, h->d_r, h->M.area, part, dn, h->stream);
			HC(hipGetLastError());
			HC(hipMemcpyAsync(&resi, dn, sizeof(double), hipMemcpyDeviceToHost, h->stream));
			HC(hipStreamSynchronize(h->stream));
			if(step == 0) initres = resi;
			if(reshistory) reshistory[step] = resi;
			step++;
			if(!std::isfinite(resi)) throw std::runtime_error("forward Euler diverged");   // Numerical_error
		}
		if(steps) *steps = step;
		if(resratio) *resratio = resi/initres;
	});
}

int fvhip_matfree_set_state(fvhip_handle h, const double* u, const double* r, const double* mdt)
{
	return guard([&] {
		HC(hipSetDevice(h->device));
		const size_t N = static_cast<size_t>(h->L.ncell);
		if(!h->d_mf_u) { h->d_mf_u = dalloc(4*N, h->owned); h->d_mf_r = dalloc(4*N, h->owned); h->d_mf_mdt = dalloc(N, h->owned); }
		std::vector<double> st(4*N);
		toInternal(h, u, st.data(), 4);
		HC(hipMemcpy(h->d_mf_u, st.data(), 4*N*sizeof(double), hipMemcpyHostToDevice));
		toInternal(h, r, st.data(), 4);
		HC(hipMemcpy(h->d_mf_r, st.data(), 4*N*sizeof(double), hipMemcpyHostToDevice));
		toInternal(h, mdt, st.data(), 1);
		HC(hipMemcpy(h->d_mf_mdt, st.data(), N*sizeof(double), hipMemcpyHostToDevice));
		h->mf_u = h->d_mf_u; h->mf_r = h->d_mf_r; h->mf_mdt = h->d_mf_mdt;
	});
}

int fvhip_matfree_apply(fvhip_handle h, const double* x, double* y)
{
	return guard([&] {
		HC(hipSetDevice(h->device));
		const size_t N = static_cast<size_t>(h->L.ncell);
		if(!h->d_mf_u) throw std::runtime_error("matrix-free operator: state not set");
		std::vector<double> st(4*N);
		toInternal(h, x, st.data(), 4);
		double *dx = h->d_u, *dy = h->d_r;   // scratch: the operator's state lives in d_mf_*
		HC(hipMemcpyAsync(dx, st.data(), 4*N*sizeof(double), hipMemcpyHostToDevice, h->stream));
		h->matfree(dx, dy);
		HC(hipMemcpyAsync(st.data(), dy, 4*N*sizeof(double), hipMemcpyDeviceToHost, h->stream));
		HC(hipStreamSynchronize(h->stream));
		fromInternal(h, st.data(), y, 4);
	});
}

int fvhip_matfree_set_state_device(fvhip_handle h, const double* d_u, const double* d_r, const double* d_mdt)
{
	return guard([&] { h->mf_u = d_u; h->mf_r = d_r; h->mf_mdt = d_mdt; });
}

int fvhip_matfree_apply_device(fvhip_handle h, const double* d_x, double* d_y)
{
	return guard([&] { HC(hipSetDevice(h->device)); h->matfree(d_x, d_y); });
}

int fvhip_matfree_set_eps(fvhip_handle h, double eps) { return guard([&] { h->mf_eps = eps; }); }

int fvhip_to_internal(fvhip_handle h, const double* host_ref, double* d_internal, int width)
{
	return guard([&] {
		HC(hipSetDevice(h->device));
		std::vector<double> st(static_cast<size_t>(h->L.ncell)*width);
		toInternal(h, host_ref, st.data(), width);
		HC(hipMemcpy(d_internal, st.data(), st.size()*sizeof(double), hipMemcpyHostToDevice));
	});
}
int fvhip_from_internal(fvhip_handle h, const double* d_internal, double* host_ref, int width)
{
	return guard([&] {
		HC(hipSetDevice(h->device));
		HC(hipStreamSynchronize(h->stream));
		std::vector<double> st(static_cast<size_t>(h->L.ncell)*width);
		HC(hipMemcpy(st.data(), d_internal, st.size()*sizeof(double), hipMemcpyDeviceToHost));
		fromInternal(h, st.data(), host_ref, width);
	});
}
int fvhip_get_permutation(fvhip_handle h, int* perm)
{
	return guard([&] { std::memcpy(perm, h->L.perm.data(), h->L.perm.size()*sizeof(int)); });
}
int fvhip_device_alloc(fvhip_handle h, unsigned long long bytes, void** ptr)
{
	return guard([&] { HC(hipSetDevice(h->device)); HC(hipMalloc(ptr, bytes)); });
}
int fvhip_device_free(fvhip_handle h, void* ptr)
{
	return guard([&] { HC(hipSetDevice(h->device)); HC(hipFree(ptr)); });
}
int fvhip_synchronize(fvhip_handle h)
{
	return guard([&] { HC(hipSetDevice(h->device)); HC(hipStreamSynchronize(h->stream)); });
}
void* fvhip_stream(fvhip_handle h) { return h ? static_cast<void*>(h->stream) : nullptr; }

int fvhip_profile(fvhip_handle h, int enable)
{
	return guard([&] {
		if(!enable && h->prof) h->collect();
		h->prof = enable != 0;
		if(enable) { h->collect(); h->acc.clear(); }
	});
}

int fvhip_kernel_times(fvhip_handle h, int maxk, char* names, int namelen, double* ms, int* counts)
{
	int n = 0;
	const int rc = guard([&] {
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

int fvhip_layout_stats(fvhip_handle h, long long* s)
{
	return guard([&] {
		s[0] = h->L.ncell; s[1] = h->L.naface; s[2] = static_cast<long long>(h->L.slot_L.size());
		s[3] = static_cast<long long>(h->L.patch_cell.size()) - 1; s[4] = h->L.max_slots; s[5] = h->L.nbface;
		s[6] = h->L.nghost; s[7] = static_cast<long long>(h->L.nbr_rank.size()); s[8] = h->nsend;
	});
}

int fvhip_local_flux(int flux_type, const double* gas5, int nf, const double* ul, const double* ur,
                     const double* n, double* flux)
{
	return guard([&] {
		gd::Gas G{gas5[0], gas5[1], gas5[2], gas5[3], gas5[4], 110.5};
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

int fvhip_local_flux_jacobian(int flux_type, const double* gas5, int nf, const double* ul,
                              const double* ur, const double* n, double* dfdl, double* dfdr)
{
	return guard([&] {
		if(flux_type == FVHIP_FLUX_VANLEER) throw std::runtime_error(" ! VanLeerFlux: Not implemented!");
		if(flux_type == FVHIP_FLUX_AUSMPLUS) throw std::runtime_error(" ! AUSMPlusFlux: Not implemented!");
		if(flux_type < 0 || flux_type > 6) throw std::invalid_argument("unknown flux");
		gd::Gas G{gas5[0], gas5[1], gas5[2], gas5[3], gas5[4], 110.5};
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
		if(kind == 0) m->raw = generateNacaOgrid(a, b, c, x, y);
		else if(kind == 1) m->raw = generateCylinderOgrid(a, b, x, y);
		else if(kind == 2) m->raw = generateFlatPlate(a, b, x, y, z);
		else throw std::invalid_argument("unknown mesh kind");
		m->mesh = buildMesh(m->raw);
		*out = m.release();
	});
}

int fvmesh_write_gmsh(fvmesh_handle m, const char* path) { return guard([&] { writeGmsh2(m->raw, path); }); }
int fvmesh_destroy(fvmesh_handle m) { return guard([&] { delete m; }); }

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
