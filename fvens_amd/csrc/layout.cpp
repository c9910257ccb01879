/** \file layout.cpp
 * \brief Builds the patch/slot device layout (see layout.hpp) and the per-cell geometric
 *   constants the reference precomputes in its constructors:
 *   - WLS normal-matrix inverses, agradientschemes.cpp:218-317 (face-order sums, Eigen 2x2 inverse)
 *   - Venkatakrishnan eps^2 = (K*clength)^3, limitedlinearreconstruction.cpp:178-205, 222
 */
#include <cstdlib>
#include "layout.hpp"
#include "partition.hpp"
#include <algorithm>
#include <numeric>
#include <stdexcept>
#include <string>
#include <cmath>

namespace fvhip {

namespace {

inline uint64_t hilbertD(uint32_t n, uint32_t x, uint32_t y)
{
	uint64_t d = 0;
	for(uint32_t s = n/2; s > 0; s /= 2) {
		const uint32_t rx = (x & s) > 0, ry = (y & s) > 0;
		d += static_cast<uint64_t>(s) * s * ((3 * rx) ^ ry);
		if(ry == 0) {
			if(rx == 1) { x = s-1 - x; y = s-1 - y; }
			const uint32_t t = x; x = y; y = t;
		}
	}
	return d;
}

/// Hilbert order of cell centres on a rank grid (adapts to graded meshes); perm[new] = old
std::vector<int> hilbertOrder(const double* rc, int N)
{
	std::vector<int> perm(N);
	std::iota(perm.begin(), perm.end(), 0);
	if(N <= 1) return perm;
	std::vector<uint32_t> ox(N), oy(N);
	std::vector<int> idx(N);
	std::iota(idx.begin(), idx.end(), 0);
	std::sort(idx.begin(), idx.end(), [&](int a, int b) { return rc[2*a] < rc[2*b] || (rc[2*a] == rc[2*b] && a < b); });
	for(int r = 0; r < N; r++) ox[idx[r]] = static_cast<uint32_t>(r);
	std::iota(idx.begin(), idx.end(), 0);
	std::sort(idx.begin(), idx.end(), [&](int a, int b) { return rc[2*a+1] < rc[2*b+1] || (rc[2*a+1] == rc[2*b+1] && a < b); });
	for(int r = 0; r < N; r++) oy[idx[r]] = static_cast<uint32_t>(r);
	uint32_t n = 1;
	while(n < static_cast<uint32_t>(N)) n <<= 1;
	std::vector<uint64_t> key(N);
	for(int i = 0; i < N; i++) key[i] = hilbertD(n, ox[i], oy[i]);
	std::sort(perm.begin(), perm.end(), [&](int a, int b) { return key[a] < key[b] || (key[a] == key[b] && a < b); });
	return perm;
}

}

Layout buildLayout(const fvhip_mesh& m, const fvhip_flow_config& cfg, bool renumber)
{
	return buildLayout(topoFromMesh(m), cfg, renumber);
}

/// faces per patch the layout aims at: SLOTS_MAX (the block size), or an experiment build's
/// FVHIP_PATCH_SLOTS (64..SLOTS_MAX: fewer faces per patch in blocks of SLOTS_MAX threads; measured slower on
/// every mesh, profiles/r04/patch_slots_ab.txt -- the block-matched variant is a build with FVHIP_SLOTS)
#ifndef FVHIP_PATCH_SLOTS
#define FVHIP_PATCH_SLOTS SLOTS_MAX
#endif
static int patchSlotCap()
{
	constexpr int v = FVHIP_PATCH_SLOTS;
	static_assert(v >= 64 && v <= SLOTS_MAX, "FVHIP_PATCH_SLOTS must lie in [64, FVHIP_SLOTS]");
	return v;
}

Layout buildLayout(const MeshTopo& T, const fvhip_flow_config& cfg, bool renumber)
{
	Layout Lo;
	const int N = T.nown, NT = T.ncell(), nb = T.nbface, F = T.naface;
	const int SC = patchSlotCap(), CC = std::min(CELLS_MAX, SC);
	Lo.ncell = N; Lo.nghost = T.nghost; Lo.nbface = nb; Lo.naface = F; Lo.ninface = F - nb;

	Lo.perm = renumber ? hilbertOrder(T.rc.data(), N) : std::vector<int>(N);
	if(!renumber) std::iota(Lo.perm.begin(), Lo.perm.end(), 0);
	Lo.iperm.assign(N, -1);
	for(int i = 0; i < N; i++) Lo.iperm[Lo.perm[i]] = i;

	auto nf = [&](int ref) { return T.nfael[ref]; };
	auto efc = [&](int ref, int j) { return T.cell_faces[4*static_cast<size_t>(ref)+j]; };
	auto esu = [&](int ref, int j) { return T.cell_esuel[4*static_cast<size_t>(ref)+j]; };
	auto Lref = [&](int f) { return T.L[f]; };
	auto Rref = [&](int f) { return T.R[f]; };
	// owned cells are renumbered; ghosts (>= N) and boundary codes (>= NT) keep their value
	auto toInt = [&](int refcell) { return refcell < N ? Lo.iperm[refcell] : refcell; };

	// --- patches, bounded slots and cells ---
	// renumbered meshes: each patch is grown breadth-first over interior faces from the first
	// unassigned cell in Hilbert order (and refilled from the next one when its region runs out), so
	// patches are compact in the mesh graph: on C4 17.6 % ring-1 cells and 8.2 % duplicated cut faces
	// against 35.2 % and 12.7 % for Hilbert ranges. The cells are then renumbered patch by patch
	// (BFS order inside a patch). Otherwise: greedy ranges of the given order.
	std::vector<int> mark(F, -1);
	Lo.patch_cell.push_back(0);
	if(renumber && N > 0) {
		std::vector<int> order;                      // new -> old, patch by patch
		order.reserve(N);
		std::vector<char> taken(static_cast<size_t>(N), 0);
		std::vector<int> queue, inq(static_cast<size_t>(N), -1);
		// partitioned meshes: cells within two faces of a ghost cell go into patches of their own
		// (built last), so that every other patch stages no ghost data -- its ring-1 cells and
		// their neighbours are all owned -- and can run while the halo is in flight
		std::vector<char> near(static_cast<size_t>(N), 0);
		if(T.nghost > 0) {
			std::vector<int> front;
			for(int c = 0; c < N; c++)
				for(int j = 0; j < nf(c); j++) {
					const int nb = esu(c, j);
					if(nb >= N && nb < NT) { near[c] = 1; front.push_back(c); break; }
				}
			for(const int c : std::vector<int>(front))
				for(int j = 0; j < nf(c); j++) {
					const int nb = esu(c, j);
					if(nb >= 0 && nb < N && !near[nb]) near[nb] = 1;
				}
		}
		int pid = 0;
		for(int pass = 0; pass < 2; pass++) {
			auto allowed = [&](int ref) { return (near[ref] != 0) == (pass == 1); };
			size_t seed = 0;
			for(;;) {
				while(seed < static_cast<size_t>(N) && (taken[Lo.perm[seed]] || !allowed(Lo.perm[seed]))) seed++;
				if(seed >= static_cast<size_t>(N)) break;
				queue.clear();
				size_t qi = 0;
				int cs = 0, cc = 0;
				for(;;) {
					if(qi == queue.size()) {
						// the patch's region is exhausted: continue from the next unassigned cell in
						// Hilbert order (a nearby hole or fresh cells), so every patch fills up
						if(cc > 0 && cs >= SC - 4) break;
						size_t sk = seed;
						while(sk < static_cast<size_t>(N) && (taken[Lo.perm[sk]] || inq[Lo.perm[sk]] == pid
						                                      || !allowed(Lo.perm[sk]))) sk++;
						if(sk >= static_cast<size_t>(N)) break;
						inq[Lo.perm[sk]] = pid;
						queue.push_back(Lo.perm[sk]);
					}
					const int ref = queue[qi++];
					int nnew = 0;
					for(int j = 0; j < nf(ref); j++) if(mark[efc(ref,j)] != pid) nnew++;
					if(cc > 0 && (cs + nnew > SC || cc + 1 > CC)) continue;   // left for later patches
					for(int j = 0; j < nf(ref); j++) mark[efc(ref,j)] = pid;
					cs += nnew; cc++;
					taken[ref] = 1;
					order.push_back(ref);
					for(int j = 0; j < nf(ref); j++) {
						const int nb = esu(ref, j);
						if(nb < 0 || nb >= N || taken[nb] || inq[nb] == pid || !allowed(nb)) continue;
						inq[nb] = pid;
						queue.push_back(nb);
					}
				}
				Lo.patch_cell.push_back(static_cast<int>(order.size()));
				pid++;
			}
		}
		Lo.perm = order;
		for(int i = 0; i < N; i++) Lo.iperm[Lo.perm[i]] = i;
	} else {
		int pid = 0, cs = 0, cc = 0;
		for(int c = 0; c < N; c++) {
			const int ref = Lo.perm[c];
			int nnew = 0;
			for(int j = 0; j < nf(ref); j++) if(mark[efc(ref,j)] != pid) nnew++;
			if(cc > 0 && (cs + nnew > SC || cc + 1 > CC)) {
				Lo.patch_cell.push_back(c);
				pid++; cs = 0; cc = 0; nnew = nf(ref);
			}
			for(int j = 0; j < nf(ref); j++) mark[efc(ref,j)] = pid;
			cs += nnew; cc++;
		}
		Lo.patch_cell.push_back(N);
	}
	// fused residual path: also cap the patch cells + ring-1 + ring-2 cells the patch stages in LDS
	// limited reconstructions (Barth-Jespersen / Venkatakrishnan) take the fused kernel on single-domain
	// meshes and on two-layer halos, whose layer-1 ghosts' limiter values are computed locally
	// (k_grad_ghost<LIM>); with the one-layer halo they would have to be exchanged as well
	const bool limitedRec = cfg.reconstruction == FVHIP_REC_BARTHJESPERSEN || cfg.reconstruction == FVHIP_REC_VENKATAKRISHNAN;
	const bool fused = fusedEligible(cfg) && (!limitedRec || T.nghost == 0 || T.halo_layers == 2);
	const int rowcap = fusedRowCap(cfg);
	Lo.fz_row_cap = rowcap;
	if(fused) {
		std::vector<int> ranges, mark2(NT, -1), r1;
		int stamp = 0;
		auto ring1 = [&](int c0, int c1) {
			stamp++;
			r1.clear();
			for(int c = c0; c < c1; c++) {
				const int ref = Lo.perm[c];
				for(int j = 0; j < nf(ref); j++) {
					const int nb = esu(ref, j);
					if(nb < 0 || nb >= NT) continue;          // boundary face
					const int ci = toInt(nb);
					if(ci >= c0 && ci < c1) continue;
					if(mark2[ci] != stamp) { mark2[ci] = stamp; r1.push_back(ci); }
				}
			}
			int n2 = 0;                                       // ring 2: through owned ring-1 cells
			for(const int ci : r1) {
				if(ci >= N) continue;
				const int ref = Lo.perm[ci];
				for(int j = 0; j < nf(ref); j++) {
					const int nb = esu(ref, j);
					if(nb < 0 || nb >= NT) continue;
					const int cj = toInt(nb);
					if((cj >= c0 && cj < c1) || mark2[cj] == stamp) continue;
					mark2[cj] = stamp; n2++;
				}
			}
			return static_cast<int>(r1.size()) + n2;
		};
		std::vector<std::pair<int,int>> stack;
		for(size_t k = 0; k + 1 < Lo.patch_cell.size(); k++) {
			stack.assign(1, {Lo.patch_cell[k], Lo.patch_cell[k+1]});
			std::vector<std::pair<int,int>> done;
			while(!stack.empty()) {
				const auto r = stack.back(); stack.pop_back();
				if(r.second - r.first > 1 && (r.second - r.first) + ring1(r.first, r.second) > rowcap) {
					const int mid = (r.first + r.second)/2;
					stack.push_back({mid, r.second}); stack.push_back({r.first, mid});
				} else done.push_back(r);
			}
			for(const auto& r : done) ranges.push_back(r.first);
		}
		ranges.push_back(N);
		Lo.patch_cell = ranges;
	}
	const int npatch = static_cast<int>(Lo.patch_cell.size()) - 1;

	// --- slots per patch ---
	std::vector<int> face_slot(F, -1);      // slot of face in the patch being built
	Lo.cell_slots.assign(static_cast<size_t>(N)*MAXF, -1);
	Lo.cell_face_local.assign(static_cast<size_t>(N)*MAXF, -1);
	Lo.cell_nbr_local.assign(static_cast<size_t>(N)*MAXF, -1);
	Lo.cell_nbr_fo.assign(static_cast<size_t>(N)*MAXF, -1);
	Lo.cell_nfael.assign(N, 0);
	Lo.patch_slot.push_back(0);
	std::vector<int> inner, cut, bnd;
	for(int p = 0; p < npatch; p++) {
		const int c0 = Lo.patch_cell[p], c1 = Lo.patch_cell[p+1];
		inner.clear(); cut.clear(); bnd.clear();
		for(int c = c0; c < c1; c++) {
			const int ref = Lo.perm[c];
			for(int j = 0; j < nf(ref); j++) {
				const int f = efc(ref,j);
				if(face_slot[f] == -2 - p) continue;     // already collected for this patch
				face_slot[f] = -2 - p;
				if(f < nb) { bnd.push_back(f); continue; }
				const int l = toInt(Lref(f)), r = toInt(Rref(f));
				if(l >= c0 && l < c1 && r >= c0 && r < c1) inner.push_back(f);
				else cut.push_back(f);
			}
		}
		const int s0 = static_cast<int>(Lo.slot_L.size());
		auto addSlot = [&](int f) {
			face_slot[f] = static_cast<int>(Lo.slot_L.size());
			Lo.slot_L.push_back(toInt(Lref(f)));
			Lo.slot_R.push_back(toInt(Rref(f)));
			Lo.slot_face.push_back(f);
			Lo.slot_n.push_back(T.facemetric[3*static_cast<size_t>(f)]);
			Lo.slot_n.push_back(T.facemetric[3*static_cast<size_t>(f)+1]);
			Lo.slot_len.push_back(T.facemetric[3*static_cast<size_t>(f)+2]);
			Lo.slot_gr.push_back(T.gr[2*static_cast<size_t>(f)]);
			Lo.slot_gr.push_back(T.gr[2*static_cast<size_t>(f)+1]);
		};
		for(int f : inner) addSlot(f);
		for(int f : cut) addSlot(f);
		for(int f : bnd) addSlot(f);
		const int ns = static_cast<int>(Lo.slot_L.size()) - s0;
		if(ns > SLOTS_MAX) throw std::logic_error("patch exceeds SLOTS_MAX");
		Lo.max_slots = std::max(Lo.max_slots, ns);
		Lo.patch_slot.push_back(static_cast<int>(Lo.slot_L.size()));
		// per-cell lists
		for(int c = c0; c < c1; c++) {
			const int ref = Lo.perm[c];
			const int k = nf(ref);
			Lo.cell_nfael[c] = k;
			int fs[MAXF];
			for(int j = 0; j < k; j++) {
				fs[j] = efc(ref,j);
				Lo.cell_face_local[static_cast<size_t>(c)*MAXF+j] = face_slot[fs[j]];
				Lo.cell_nbr_local[static_cast<size_t>(c)*MAXF+j] = toInt(esu(ref,j));
			}
			std::sort(fs, fs+k);     // local faces are in ascending global order
			for(int j = 0; j < k; j++) {
				Lo.cell_slots[static_cast<size_t>(c)*MAXF+j] = (face_slot[fs[j]] << 1) | (Lref(fs[j]) != ref ? 1 : 0);
				const int other = Lref(fs[j]) != ref ? Lref(fs[j]) : Rref(fs[j]);
				Lo.cell_nbr_fo[static_cast<size_t>(c)*MAXF+j] = toInt(other);
			}
		}
	}

	// --- cell geometry (internal order; ghosts after the owned cells) ---
	Lo.rc.resize(2*static_cast<size_t>(NT)); Lo.area.resize(N);
	for(int c = 0; c < N; c++) {
		const int ref = Lo.perm[c];
		Lo.rc[2*c] = T.rc[2*ref]; Lo.rc[2*c+1] = T.rc[2*ref+1]; Lo.area[c] = T.area[ref];
	}
	for(int c = N; c < NT; c++) { Lo.rc[2*c] = T.rc[2*c]; Lo.rc[2*c+1] = T.rc[2*c+1]; }

	// --- halo (internal ids) ---
	Lo.nbr_rank = T.nbr_rank;
	Lo.ghost_start = T.ghost_start;
	Lo.send_start = T.send_start;
	Lo.send_cells.resize(T.send_cells.size());
	for(size_t i = 0; i < T.send_cells.size(); i++) Lo.send_cells[i] = Lo.iperm[T.send_cells[i]];
	Lo.halo_layers = T.halo_layers;
	Lo.ghost_l1_end = T.ghost_l1_end;
	Lo.send_l1_end = T.send_l1_end;
	Lo.border_cells.clear();
	for(size_t k = 0; k + 1 < Lo.send_start.size(); k++) {
		const int e = k < Lo.send_l1_end.size() ? Lo.send_l1_end[k] : Lo.send_start[k+1];
		for(int i = Lo.send_start[k]; i < e; i++) Lo.border_cells.push_back(Lo.send_cells[i]);
	}
	std::sort(Lo.border_cells.begin(), Lo.border_cells.end());
	Lo.border_cells.erase(std::unique(Lo.border_cells.begin(), Lo.border_cells.end()), Lo.border_cells.end());
	Lo.cell_global.resize(NT);
	for(int c = 0; c < N; c++) Lo.cell_global[c] = T.cell_global[Lo.perm[c]];
	for(int c = N; c < NT; c++) Lo.cell_global[c] = T.cell_global[c];
	Lo.trace_conn.clear();
	for(const int row : T.ghost_row) Lo.trace_conn.push_back(row - N);

	// --- boundary faces ---
	Lo.bf_L.resize(nb); Lo.bf_bc.resize(nb); Lo.bf_n.resize(2*static_cast<size_t>(nb)); Lo.bf_rcbp.resize(2*static_cast<size_t>(nb));
	Lo.bf_tag.resize(nb); Lo.bf_gr.resize(2*static_cast<size_t>(nb));
	for(int f = 0; f < nb; f++) {
		Lo.bf_L[f] = Lo.iperm[Lref(f)];
		const int tag = T.btag[f];
		int bi = -1;
		for(int i = 0; i < cfg.nbc; i++) if(cfg.bc_tag[i] == tag) bi = i;
		if(bi < 0) throw std::runtime_error("no boundary condition for marker " + std::to_string(tag)); // bcs.at()
		Lo.bf_bc[f] = bi;
		Lo.bf_n[2*f] = T.facemetric[3*static_cast<size_t>(f)]; Lo.bf_n[2*f+1] = T.facemetric[3*static_cast<size_t>(f)+1];
		Lo.bf_rcbp[2*f] = T.rcbp[2*f]; Lo.bf_rcbp[2*f+1] = T.rcbp[2*f+1];
		Lo.bf_tag[f] = tag;
		Lo.bf_gr[2*f] = T.gr[2*static_cast<size_t>(f)]; Lo.bf_gr[2*f+1] = T.gr[2*static_cast<size_t>(f)+1];
	}
	// --- layer-1 ghosts of a two-layer halo: neighbour lists, extra boundary faces, WLS inverses ---
	Lo.gg_cells = T.g1_cells;               // ghosts keep their local ids
	Lo.gg_nbr.resize(T.g1_nbr.size());
	for(size_t k = 0; k < T.g1_nbr.size(); k++) Lo.gg_nbr[k] = T.g1_nbr[k] >= 0 ? toInt(T.g1_nbr[k]) : T.g1_nbr[k];
	Lo.xb_bc.resize(T.xb_btag.size());
	for(size_t x = 0; x < T.xb_btag.size(); x++) {
		int bi = -1;
		for(int i = 0; i < cfg.nbc; i++) if(cfg.bc_tag[i] == T.xb_btag[x]) bi = i;
		if(bi < 0) throw std::runtime_error("no boundary condition for marker " + std::to_string(T.xb_btag[x]));
		Lo.xb_bc[x] = bi;
	}
	Lo.xb_n = T.xb_n; Lo.xb_rcbp = T.xb_rcbp;
	Lo.gg_gp = T.g1_gr;
	if(cfg.reconstruction == FVHIP_REC_VENKATAKRISHNAN) {
		Lo.gg_eps2.resize(T.g1_clength.size());
		for(size_t i = 0; i < T.g1_clength.size(); i++) Lo.gg_eps2[i] = std::pow(cfg.limiter_param*T.g1_clength[i], 3);
	}
	if(cfg.gradientscheme == FVHIP_GRAD_LEASTSQUARES) {
		// the host WLS normal matrix below, cell by cell: faces in ascending global order, the ghost's
		// centre minus the other centre (the face loop's dr up to a sign that cancels in each term)
		Lo.gg_V.resize(4*Lo.gg_cells.size());
		for(size_t i = 0; i < Lo.gg_cells.size(); i++) {
			const int g = Lo.gg_cells[i];
			double v[4] = {0, 0, 0, 0};
			for(int j = 0; j < MAXF; j++) {
				const int nbk = Lo.gg_nbr[4*i+j];
				if(nbk == -1) break;
				const double* rn = nbk >= 0 ? &Lo.rc[2*static_cast<size_t>(nbk)] : &Lo.xb_rcbp[2*static_cast<size_t>(-2 - nbk)];
				double w2 = 0, dr[2];
				for(int d = 0; d < 2; d++) {
					w2 += (Lo.rc[2*static_cast<size_t>(g)+d]-rn[d])*(Lo.rc[2*static_cast<size_t>(g)+d]-rn[d]);
					dr[d] = Lo.rc[2*static_cast<size_t>(g)+d]-rn[d];
				}
				w2 = 1.0/(w2);
				for(int a = 0; a < 2; a++) for(int b = 0; b < 2; b++) v[2*a+b] += w2*dr[a]*dr[b];
			}
			const double det = v[0]*v[3] - v[2]*v[1];
			const double invdet = 1.0/det;
			double* o = &Lo.gg_V[4*i];
			o[0] = v[3]*invdet; o[2] = -v[2]*invdet; o[1] = -v[1]*invdet; o[3] = v[0]*invdet;
		}
	}
	// --- interior faces (reference order) ---
	Lo.if_L.resize(F-nb); Lo.if_R.resize(F-nb); Lo.if_slot.assign(F-nb, -1);
	Lo.if_n.resize(2*static_cast<size_t>(F-nb)); Lo.if_len.resize(F-nb); Lo.bf_len.resize(nb);
	for(int f = nb; f < F; f++) {
		Lo.if_L[f-nb] = toInt(Lref(f)); Lo.if_R[f-nb] = toInt(Rref(f));
		Lo.if_n[2*static_cast<size_t>(f-nb)] = T.facemetric[3*static_cast<size_t>(f)];
		Lo.if_n[2*static_cast<size_t>(f-nb)+1] = T.facemetric[3*static_cast<size_t>(f)+1];
		Lo.if_len[f-nb] = T.facemetric[3*static_cast<size_t>(f)+2];
	}
	for(int f = 0; f < nb; f++) Lo.bf_len[f] = T.facemetric[3*static_cast<size_t>(f)+2];
	for(size_t s = 0; s < Lo.slot_face.size(); s++)
		if(Lo.slot_face[s] >= nb) Lo.if_slot[Lo.slot_face[s]-nb] = static_cast<int>(s);
	// each cell's faces as reference face codes, same order as cell_slots
	Lo.cell_rfaces.assign(4*static_cast<size_t>(N), -1);
	for(size_t k = 0; k < Lo.cell_slots.size(); k++) {
		const int code = Lo.cell_slots[k];
		if(code >= 0) Lo.cell_rfaces[k] = (Lo.slot_face[code >> 1] << 1) | (code & 1);
	}

	// --- WLS normal matrices (agradientschemes.cpp:218-317), reference face order ---
	if(cfg.gradientscheme == FVHIP_GRAD_LEASTSQUARES) {
		std::vector<double> V(4*static_cast<size_t>(NT), 0.0);
		const double* rc = T.rc.data(); const double* rcbp = T.rcbp.data();
		for(int f = 0; f < nb; f++) {
			const int ie = Lref(f);
			double w2 = 0, dr[2];
			for(int d = 0; d < 2; d++) {
				w2 += (rc[2*ie+d]-rcbp[2*f+d])*(rc[2*ie+d]-rcbp[2*f+d]);
				dr[d] = rc[2*ie+d]-rcbp[2*f+d];
			}
			w2 = 1.0/(w2);
			for(int i = 0; i < 2; i++) for(int j = 0; j < 2; j++) V[4*ie+2*i+j] += w2*dr[i]*dr[j];
		}
		for(int f = nb; f < F; f++) {
			const int ie = Lref(f), je = Rref(f);
			double w2 = 0, dr[2];
			for(int d = 0; d < 2; d++) {
				w2 += (rc[2*ie+d]-rc[2*je+d])*(rc[2*ie+d]-rc[2*je+d]);
				dr[d] = rc[2*ie+d]-rc[2*je+d];
			}
			w2 = 1.0/(w2);
			for(int i = 0; i < 2; i++) for(int j = 0; j < 2; j++) {
				V[4*ie+2*i+j] += w2*dr[i]*dr[j];
				V[4*je+2*i+j] += w2*dr[i]*dr[j];
			}
		}
		Lo.wls_V.resize(4*static_cast<size_t>(N));
		for(int c = 0; c < N; c++) {
			const double* v = &V[4*static_cast<size_t>(Lo.perm[c])];
			const double det = v[0]*v[3] - v[2]*v[1];
			const double invdet = 1.0/det;
			double* o = &Lo.wls_V[4*static_cast<size_t>(c)];
			o[0] = v[3]*invdet; o[2] = -v[2]*invdet; o[1] = -v[1]*invdet; o[3] = v[0]*invdet;
		}
	}
	// --- Venkatakrishnan eps^2 ---
	if(cfg.reconstruction == FVHIP_REC_VENKATAKRISHNAN) {
		Lo.venk_eps2.resize(N);
		for(int c = 0; c < N; c++) Lo.venk_eps2[c] = std::pow(cfg.limiter_param*T.clength[Lo.perm[c]], 3);
	}
	if(fused) buildFused(Lo);
	if(Lo.nghost == 0 && pipelineEligible(cfg)) buildPipeline(Lo, PIPE_CHUNKS);
	return Lo;
}

bool pipelineEligible(const fvhip_flow_config& cfg)
{
	return cfg.order2 && cfg.gradientscheme == FVHIP_GRAD_LEASTSQUARES &&
	       (cfg.reconstruction == FVHIP_REC_VANALBADA || cfg.reconstruction == FVHIP_REC_NONE);
}

void buildPipeline(Layout& Lo, int chunks)
{
	const int N = Lo.ncell;
	const int npatch = static_cast<int>(Lo.patch_cell.size()) - 1;
	if(chunks < 1 || N == 0) { Lo.pipe_cell_start.clear(); return; }
	// chunk boundaries on 256-cell blocks of the gradient kernel
	const int nblk = (N + 255)/256;
	Lo.pipe_cell_start.assign(1, 0);
	for(int k = 1; k < chunks; k++) {
		const int b = static_cast<int>((static_cast<long long>(nblk)*k)/chunks)*256;
		if(b > Lo.pipe_cell_start.back() && b < N) Lo.pipe_cell_start.push_back(b);
	}
	Lo.pipe_cell_start.push_back(N);
	const int K = static_cast<int>(Lo.pipe_cell_start.size()) - 1;
	auto chunkOf = [&](int c) {
		return static_cast<int>(std::upper_bound(Lo.pipe_cell_start.begin(), Lo.pipe_cell_start.end(), c)
		                        - Lo.pipe_cell_start.begin()) - 1;
	};
	// a patch reads the primitive states and gradients of its cells and of the far side of its cut
	// faces (and the ghost states of its own boundary faces, written with its cells)
	std::vector<int> dep(npatch, 0);
	for(int p = 0; p < npatch; p++)
		for(int s = Lo.patch_slot[p]; s < Lo.patch_slot[p+1]; s++) {
			dep[p] = std::max(dep[p], chunkOf(Lo.slot_L[s]));
			if(Lo.slot_R[s] < N) dep[p] = std::max(dep[p], chunkOf(Lo.slot_R[s]));
		}
	Lo.pipe_group_start.assign(K+1, 0);
	for(int p = 0; p < npatch; p++) Lo.pipe_group_start[dep[p]+1]++;
	for(int k = 0; k < K; k++) Lo.pipe_group_start[k+1] += Lo.pipe_group_start[k];
	Lo.pipe_patch.assign(npatch, -1);
	std::vector<int> pos(Lo.pipe_group_start.begin(), Lo.pipe_group_start.end() - 1);
	for(int p = 0; p < npatch; p++) Lo.pipe_patch[pos[dep[p]]++] = p;
}

bool fusedEligible(const fvhip_flow_config& cfg)
{
	const bool limited = cfg.reconstruction == FVHIP_REC_BARTHJESPERSEN || cfg.reconstruction == FVHIP_REC_VENKATAKRISHNAN;
	// the fused kernel inlines the common BC types' ghost states (kernels.hip ghost_c); subsonic inflow
	// and isothermal walls take the staged path, whose kernels call the full ghost state out of line
	for(int i = 0; i < cfg.nbc; i++)
		if(cfg.bc_type[i] == FVHIP_BC_SUBSONIC_INFLOW || cfg.bc_type[i] == FVHIP_BC_ISOTHERMAL_WALL) return false;
	return cfg.order2 && cfg.gradientscheme == FVHIP_GRAD_LEASTSQUARES &&
	       (cfg.reconstruction == FVHIP_REC_VANALBADA || cfg.reconstruction == FVHIP_REC_NONE ||
	        (limited && !cfg.viscous_sim));
}

int fusedRowCap(const fvhip_flow_config& cfg)
{
	// inviscid unlimited: 14-double rows, five blocks per CU; viscous: 18-double rows (the temperature
	// terms), four blocks per CU -- 284 rows either way (31.8 / 40.9 KB); limited: 14-double rows, four
	const bool limited = cfg.reconstruction == FVHIP_REC_BARTHJESPERSEN || cfg.reconstruction == FVHIP_REC_VENKATAKRISHNAN;
	return !limited ? FUSED_LDS_CELLS_5W : FUSED_LDS_CELLS;
}

void buildFused(Layout& Lo)
{
	const int N = Lo.ncell + Lo.nghost;      // ghost cells may be ring-1 cells (their gradients are received)
	const int npatch = static_cast<int>(Lo.patch_cell.size()) - 1;
	Lo.fz_ext_start.assign(1, 0); Lo.fz_ext.clear(); Lo.fz_n1.assign(npatch, 0);
	Lo.fz_g_start.assign(1, 0);
	Lo.fz_gnbr.clear();
	Lo.fz_slot_lr.assign(2*Lo.slot_L.size(), -1);
	Lo.fz_slot_lr16.assign(Lo.slot_L.size(), 0xFFFFFFFFu);
	Lo.fz_gnbr16.clear();
	Lo.fz_gbf_start.assign(1, 0); Lo.fz_gbf.clear();
	Lo.fz_cslot16.assign(4*static_cast<size_t>(Lo.ncell), 0xFFFF);
	Lo.fz_max_cells = 0;
	Lo.fz_ring2 = 0;
	std::vector<int> lidx(N, -1);          // patch-local index of a cell while its patch is built
	std::vector<char> innerp(npatch, 0);
	for(int p = 0; p < npatch; p++) {
		const int c0 = Lo.patch_cell[p], c1 = Lo.patch_cell[p+1], nc = c1 - c0;
		const size_t e0 = Lo.fz_ext.size();
		for(int c = c0; c < c1; c++) lidx[c] = c - c0;
		int nl = nc;
		auto add = [&](int c) {
			if(c < 0 || c >= N || lidx[c] >= 0) return;
			lidx[c] = nl++; Lo.fz_ext.push_back(c);
		};
		// ring 1: the other side of the patch's cut faces
		for(int s = Lo.patch_slot[p]; s < Lo.patch_slot[p+1]; s++) { add(Lo.slot_L[s]); add(Lo.slot_R[s]); }
		const int ng = nl;
		// ring 2: the other neighbours of the owned ring-1 cells (their gradients read them)
		for(int i = nc; i < ng; i++) {
			const int c = Lo.fz_ext[e0 + (i - nc)];
			if(c >= Lo.ncell) continue;
			for(int j = 0; j < MAXF; j++) add(Lo.cell_nbr_fo[static_cast<size_t>(c)*MAXF+j]);
		}
		if(nl > Lo.fz_row_cap) throw std::logic_error("fused residual: patch exceeds its LDS budget");
		Lo.fz_n1[p] = ng - nc;
		Lo.fz_ring2 += nl - ng;
		Lo.fz_ext_start.push_back(static_cast<int>(Lo.fz_ext.size()));
		// neighbours of every cell whose gradient the patch computes, in ascending reference face order
		auto code = [&](int nb) {
			if(nb < 0) return -1;
			if(nb >= N) return -2 - (nb - N);
			if(lidx[nb] < 0) throw std::logic_error("fused residual: neighbour not staged");
			return lidx[nb];
		};
		for(int i = 0; i < ng; i++) {
			const int c = i < nc ? c0 + i : Lo.fz_ext[e0 + (i - nc)];
			for(int j = 0; j < MAXF; j++)     // ghost cells: gradient received, no neighbour list
				Lo.fz_gnbr.push_back(c < Lo.ncell ? code(Lo.cell_nbr_fo[static_cast<size_t>(c)*MAXF+j]) : -1);
		}
		Lo.fz_g_start.push_back(Lo.fz_g_start.back() + ng);
		for(int s = Lo.patch_slot[p]; s < Lo.patch_slot[p+1]; s++) {
			Lo.fz_slot_lr[2*static_cast<size_t>(s)] = code(Lo.slot_L[s]);
			Lo.fz_slot_lr[2*static_cast<size_t>(s)+1] = code(Lo.slot_R[s]);
		}
		// packed forms
		const size_t gb0 = Lo.fz_gbf.size();
		for(size_t k = Lo.fz_gnbr.size() - 4*static_cast<size_t>(ng); k < Lo.fz_gnbr.size(); k++) {
			const int v = Lo.fz_gnbr[k];
			if(v == -1) { Lo.fz_gnbr16.push_back(0xFFFF); continue; }
			if(v >= 0) { Lo.fz_gnbr16.push_back(static_cast<uint16_t>(v)); continue; }
			const size_t j = Lo.fz_gbf.size() - gb0;
			if(j >= 0x7FFF) throw std::logic_error("fused residual: too many boundary faces in one patch");
			Lo.fz_gbf.push_back(-2 - v);
			Lo.fz_gnbr16.push_back(static_cast<uint16_t>(0x8000 | j));
		}
		Lo.fz_gbf_start.push_back(static_cast<int>(Lo.fz_gbf.size()));
		for(int s = Lo.patch_slot[p]; s < Lo.patch_slot[p+1]; s++) {
			const int l = Lo.fz_slot_lr[2*static_cast<size_t>(s)], r = Lo.fz_slot_lr[2*static_cast<size_t>(s)+1];
			Lo.fz_slot_lr16[s] = static_cast<uint32_t>(l) | (static_cast<uint32_t>(r >= 0 ? r : 0xFFFF) << 16);
		}
		for(int c = c0; c < c1; c++)
			for(int j = 0; j < MAXF; j++) {
				const int e = Lo.cell_slots[static_cast<size_t>(c)*MAXF+j];
				if(e < 0) continue;
				const int ls = (e >> 1) - Lo.patch_slot[p];
				if(ls < 0 || ls >= SLOTS_MAX) throw std::logic_error("fused residual: cell face outside its patch");
				Lo.fz_cslot16[static_cast<size_t>(c)*MAXF+j] = static_cast<uint16_t>((ls << 1) | (e & 1));
			}
		Lo.fz_max_cells = std::max(Lo.fz_max_cells, nl);
		// interior patch: stages no ghost cell, so it needs no halo data and can run while the
		// exchange is in flight
		bool inner = true;
		for(size_t k = e0; k < Lo.fz_ext.size(); k++) if(Lo.fz_ext[k] >= Lo.ncell) inner = false;
		innerp[p] = inner ? 1 : 0;
		for(int c = c0; c < c1; c++) lidx[c] = -1;
		for(size_t k = e0; k < Lo.fz_ext.size(); k++) lidx[Lo.fz_ext[k]] = -1;
	}
	Lo.fz_order.clear();
	for(int p = 0; p < npatch; p++) if(innerp[p]) Lo.fz_order.push_back(p);
	Lo.fz_ninner = static_cast<int>(Lo.fz_order.size());
	for(int p = 0; p < npatch; p++) if(!innerp[p]) Lo.fz_order.push_back(p);
}

}
