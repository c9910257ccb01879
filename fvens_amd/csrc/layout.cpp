/** \file layout.cpp
 * \brief Builds the patch/slot device layout (see layout.hpp) and the per-cell geometric
 *   constants the reference precomputes in its constructors:
 *   - WLS normal-matrix inverses, agradientschemes.cpp:218-317 (face-order sums, Eigen 2x2 inverse)
 *   - Venkatakrishnan eps^2 = (K*clength)^3, limitedlinearreconstruction.cpp:178-205, 222
 */
#include "layout.hpp"
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
	if(m.nconnface != 0)
		throw std::runtime_error("buildLayout: connectivity faces need the partitioned path");
	if(m.maxnfael > MAXF) throw std::runtime_error("buildLayout: cells with more than 4 faces");
	Layout Lo;
	const int N = m.nelem, nb = m.nbface, F = m.naface;
	Lo.ncell = N; Lo.nbface = nb; Lo.naface = F; Lo.ninface = F - nb;

	Lo.perm = renumber ? hilbertOrder(m.rc, N) : std::vector<int>(N);
	if(!renumber) std::iota(Lo.perm.begin(), Lo.perm.end(), 0);
	Lo.iperm.assign(N, -1);
	for(int i = 0; i < N; i++) Lo.iperm[Lo.perm[i]] = i;

	auto nf = [&](int ref) { return m.nnode[ref]; };
	auto efc = [&](int ref, int j) { return m.elemface[static_cast<size_t>(ref)*m.maxnfael+j]; };
	auto esu = [&](int ref, int j) { return m.esuel[static_cast<size_t>(ref)*m.maxnfael+j]; };
	auto Lref = [&](int f) { return m.intfac[4*static_cast<size_t>(f)]; };
	auto Rref = [&](int f) { return m.intfac[4*static_cast<size_t>(f)+1]; };
	auto toInt = [&](int refcell) { return refcell < N ? Lo.iperm[refcell] : N + (refcell - N - m.nconnface); };

	// --- patches (greedy over internal cells, bounded slots and cells) ---
	std::vector<int> mark(F, -1);
	Lo.patch_cell.push_back(0);
	{
		int pid = 0, cs = 0, cc = 0;
		for(int c = 0; c < N; c++) {
			const int ref = Lo.perm[c];
			int nnew = 0;
			for(int j = 0; j < nf(ref); j++) if(mark[efc(ref,j)] != pid) nnew++;
			if(cc > 0 && (cs + nnew > SLOTS_MAX || cc + 1 > CELLS_MAX)) {
				Lo.patch_cell.push_back(c);
				pid++; cs = 0; cc = 0; nnew = nf(ref);
			}
			for(int j = 0; j < nf(ref); j++) mark[efc(ref,j)] = pid;
			cs += nnew; cc++;
		}
		Lo.patch_cell.push_back(N);
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
				const int l = Lo.iperm[Lref(f)], r = Lo.iperm[Rref(f)];
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
			Lo.slot_n.push_back(m.facemetric[3*static_cast<size_t>(f)]);
			Lo.slot_n.push_back(m.facemetric[3*static_cast<size_t>(f)+1]);
			Lo.slot_len.push_back(m.facemetric[3*static_cast<size_t>(f)+2]);
			Lo.slot_gr.push_back(m.gr[2*static_cast<size_t>(f)]);
			Lo.slot_gr.push_back(m.gr[2*static_cast<size_t>(f)+1]);
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
			std::sort(fs, fs+k);
			for(int j = 0; j < k; j++) {
				Lo.cell_slots[static_cast<size_t>(c)*MAXF+j] = (face_slot[fs[j]] << 1) | (Lref(fs[j]) != ref ? 1 : 0);
				const int other = Lref(fs[j]) != ref ? Lref(fs[j]) : Rref(fs[j]);
				Lo.cell_nbr_fo[static_cast<size_t>(c)*MAXF+j] = toInt(other);
			}
		}
	}

	// --- cell geometry (internal order) ---
	Lo.rc.resize(2*static_cast<size_t>(N)); Lo.area.resize(N);
	for(int c = 0; c < N; c++) {
		const int ref = Lo.perm[c];
		Lo.rc[2*c] = m.rc[2*ref]; Lo.rc[2*c+1] = m.rc[2*ref+1]; Lo.area[c] = m.area[ref];
	}

	// --- boundary faces ---
	Lo.bf_L.resize(nb); Lo.bf_bc.resize(nb); Lo.bf_n.resize(2*static_cast<size_t>(nb)); Lo.bf_rcbp.resize(2*static_cast<size_t>(nb));
	for(int f = 0; f < nb; f++) {
		Lo.bf_L[f] = Lo.iperm[Lref(f)];
		const int tag = m.btags[static_cast<size_t>(f)*m.nbtag];
		int bi = -1;
		for(int i = 0; i < cfg.nbc; i++) if(cfg.bc_tag[i] == tag) bi = i;
		if(bi < 0) throw std::runtime_error("no boundary condition for marker " + std::to_string(tag)); // bcs.at()
		Lo.bf_bc[f] = bi;
		Lo.bf_n[2*f] = m.facemetric[3*static_cast<size_t>(f)]; Lo.bf_n[2*f+1] = m.facemetric[3*static_cast<size_t>(f)+1];
		Lo.bf_rcbp[2*f] = m.rcbp[2*f]; Lo.bf_rcbp[2*f+1] = m.rcbp[2*f+1];
	}
	// --- interior faces (reference order) ---
	Lo.if_L.resize(F-nb); Lo.if_R.resize(F-nb); Lo.if_slot.assign(F-nb, -1);
	Lo.if_n.resize(2*static_cast<size_t>(F-nb)); Lo.if_len.resize(F-nb); Lo.bf_len.resize(nb);
	for(int f = nb; f < F; f++) {
		Lo.if_L[f-nb] = Lo.iperm[Lref(f)]; Lo.if_R[f-nb] = Lo.iperm[Rref(f)];
		Lo.if_n[2*static_cast<size_t>(f-nb)] = m.facemetric[3*static_cast<size_t>(f)];
		Lo.if_n[2*static_cast<size_t>(f-nb)+1] = m.facemetric[3*static_cast<size_t>(f)+1];
		Lo.if_len[f-nb] = m.facemetric[3*static_cast<size_t>(f)+2];
	}
	for(int f = 0; f < nb; f++) Lo.bf_len[f] = m.facemetric[3*static_cast<size_t>(f)+2];
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
		std::vector<double> V(4*static_cast<size_t>(N), 0.0);
		const double* rc = m.rc; const double* rcbp = m.rcbp;
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
		for(int c = 0; c < N; c++) {
			const int ref = Lo.perm[c];
			double cl = 0;
			for(int ifa = 0; ifa < m.nnode[ref]; ifa++) {
				const int a = m.inpoel[static_cast<size_t>(ref)*m.maxnnode+ifa];
				const int b = m.inpoel[static_cast<size_t>(ref)*m.maxnnode+(ifa+1)%m.nnode[ref]];
				double llen = 0;
				for(int d = 0; d < 2; d++) llen += std::pow(m.coords[2*a+d] - m.coords[2*b+d], 2);
				if(cl < llen) cl = llen;
			}
			cl = std::sqrt(cl);
			Lo.venk_eps2[c] = std::pow(cfg.limiter_param*cl, 3);
		}
	}
	return Lo;
}

}
