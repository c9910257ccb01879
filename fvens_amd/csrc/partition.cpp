/** \file partition.cpp
 * \brief RCB partitioning and per-rank local topologies (see partition.hpp).
 */
#include "partition.hpp"
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <numeric>
#include <queue>
#include <stdexcept>
#include <string>

namespace fvhip {

namespace {

/// longest edge of a cell (limitedlinearreconstruction.cpp:186-205)
double cellLength(const fvhip_mesh& m, int ref)
{
	double cl = 0;
	for(int ifa = 0; ifa < m.nnode[ref]; ifa++) {
		const int a = m.inpoel[static_cast<size_t>(ref)*m.maxnnode+ifa];
		const int b = m.inpoel[static_cast<size_t>(ref)*m.maxnnode+(ifa+1)%m.nnode[ref]];
		double llen = 0;
		for(int d = 0; d < 2; d++) llen += std::pow(m.coords[2*a+d] - m.coords[2*b+d], 2);
		if(cl < llen) cl = llen;
	}
	return std::sqrt(cl);
}

/// the hot path's cells are linear triangles and quads, whose node count is their face count (every
/// loop here takes nnode as the number of faces): reject anything else (quadratic gmsh elements,
/// nnode 6/8/9, which the reader accepts) before an esuel row or a 4-entry buffer is overrun
void checkLinearCells(const fvhip_mesh& m, const char* who)
{
	if(m.maxnfael > 4 || m.maxnfael < 3) throw std::runtime_error(std::string(who) + ": cells with more than 4 faces are not supported");
	for(int e = 0; e < m.nelem; e++)
		if(m.nnode[e] < 3 || m.nnode[e] > m.maxnfael)
			throw std::runtime_error(std::string(who) + ": cell " + std::to_string(e) + " has " + std::to_string(m.nnode[e]) +
			                         " nodes; only linear triangles and quadrangles are supported");
}

void rcbRecurse(const double* rc, int* idx, int n, int p0, int np, int* part)
{
	if(np == 1) { for(int i = 0; i < n; i++) part[idx[i]] = p0; return; }
	double lo[2] = {INFINITY, INFINITY}, hi[2] = {-INFINITY, -INFINITY};
	for(int i = 0; i < n; i++)
		for(int d = 0; d < 2; d++) {
			lo[d] = std::min(lo[d], rc[2*idx[i]+d]);
			hi[d] = std::max(hi[d], rc[2*idx[i]+d]);
		}
	const int ax = (hi[1]-lo[1] > hi[0]-lo[0]) ? 1 : 0;
	const int npl = np/2;
	const int nl = static_cast<int>((static_cast<long long>(n)*npl)/np);
	std::nth_element(idx, idx + nl, idx + n, [&](int a, int b) {
		return rc[2*a+ax] < rc[2*b+ax] || (rc[2*a+ax] == rc[2*b+ax] && a < b); });
	rcbRecurse(rc, idx, nl, p0, npl, part);
	rcbRecurse(rc, idx + nl, n - nl, p0 + npl, np - npl, part);
}

}

std::vector<std::vector<int>> findLinesReference(const fvhip_mesh& m, double threshold)
{
	checkLinearCells(m, "findLines");
	const int N = m.nelem;
	// computeWeights (meshordering.cpp:143-205): per cell, 1/|c_i - c_j| to every neighbour that is a
	// cell (vertex-average centres, ameshutils.hpp:48-60), divided by the smallest, in decreasing order
	// (ties keep face order: libstdc++ sorts these <= 4 entries by insertion, which is stable)
	std::vector<double> cc(2*static_cast<size_t>(N));
	for(int e = 0; e < N; e++) {
		double c[2] = {0, 0};
		for(int j = 0; j < m.nnode[e]; j++)
			for(int k = 0; k < 2; k++) c[k] += m.coords[2*static_cast<size_t>(m.inpoel[static_cast<size_t>(e)*m.maxnnode+j])+k];
		for(int k = 0; k < 2; k++) cc[2*static_cast<size_t>(e)+k] = c[k] / m.nnode[e];
	}
	std::vector<double> aniso(4*static_cast<size_t>(N), 0.0);
	std::vector<int> fidx(4*static_cast<size_t>(N), -1), nreal(N, 0);
	for(int e = 0; e < N; e++) {
		std::vector<std::pair<double,int>> w;
		double minw = 1e20;
		for(int j = 0; j < m.nnode[e]; j++) {
			const int je = m.esuel[static_cast<size_t>(e)*m.maxnfael+j];
			if(je < 0 || je >= N) continue;                  // ghost across a boundary or connectivity face
			double dist = 0;
			for(int k = 0; k < 2; k++) dist += std::pow(cc[2*static_cast<size_t>(e)+k] - cc[2*static_cast<size_t>(je)+k], 2);
			const double wt = 1.0/std::sqrt(dist);
			if(wt < minw) minw = wt;
			w.push_back({wt, j});
		}
		for(auto& x : w) x.first /= minw;
		std::stable_sort(w.begin(), w.end(), [](const std::pair<double,int>& a, const std::pair<double,int>& b) {
			return a.first > b.first; });
		nreal[e] = static_cast<int>(w.size());
		for(size_t j = 0; j < w.size(); j++) { aniso[4*static_cast<size_t>(e)+j] = w[j].first; fidx[4*static_cast<size_t>(e)+j] = w[j].second; }
	}
	// findLines (meshordering.cpp:207-264): from the cell of every physical boundary face in face order,
	// walk while the cell's largest anisotropy exceeds the threshold, always to the first (strongest)
	// neighbour not yet in a line whose anisotropy exceeds it; a one-cell walk is no line. A cell without
	// cell neighbours has no weights (the reference reads an unset entry there): it starts no line.
	std::vector<int> celline(N, -1);
	std::vector<std::vector<int>> lines;
	for(int f = 0; f < m.nbface; f++) {
		const int belem = m.intfac[4*static_cast<size_t>(f)];
		if(belem < 0 || belem >= N || celline[belem] >= 0) continue;
		std::vector<int> le;
		int cur = belem;
		for(;;) {
			if(nreal[cur] > 0 && aniso[4*static_cast<size_t>(cur)] > threshold) {
				le.push_back(cur);
				celline[cur] = static_cast<int>(lines.size());
			}
			else break;
			int next = -1;
			for(int j = 0; j < nreal[cur]; j++) {
				const int nb = m.esuel[static_cast<size_t>(cur)*m.maxnfael+fidx[4*static_cast<size_t>(cur)+j]];
				if(celline[nb] == -1 && aniso[4*static_cast<size_t>(cur)+j] > threshold) { next = nb; break; }
			}
			if(next < 0) break;
			cur = next;
		}
		if(le.size() > 1) lines.push_back(le);
		else if(le.size() == 1) celline[le[0]] = -1;
	}
	return lines;
}

std::vector<int> partitionRCB(const double* rc, int ncell, int nparts)
{
	if(nparts < 1) throw std::invalid_argument("partitionRCB: nparts < 1");
	std::vector<int> part(ncell, 0), idx(ncell);
	std::iota(idx.begin(), idx.end(), 0);
	if(ncell > 0) rcbRecurse(rc, idx.data(), ncell, 0, nparts, part.data());
	return part;
}

namespace {

/// one bisection of the cells `sub` (global ids) of the dual graph into `nl` and the rest: grown
/// breadth-first from a pseudo-peripheral cell (farthest from the farthest of the first cell, every
/// component in turn), then improved by passes of balanced boundary swaps (Kernighan-Lin gains)
void graphBisect(const fvhip_mesh& m, const std::vector<int>& sub, long long tw, const int* wt, std::vector<int>& side,
                 std::vector<int>& loc, std::vector<int>& dist)
{
	const int n = static_cast<int>(sub.size());
	auto w = [&](int a) { return wt ? wt[sub[a]] : 1; };   // weight of local cell a
	long long wmax = 1;
	for(int a = 0; a < n; a++) wmax = std::max<long long>(wmax, w(a));
	for(int i = 0; i < n; i++) loc[sub[i]] = i;
	auto nbrs = [&](int c, int* out) {          // neighbours of global cell c inside `sub` (local ids)
		int k = 0;
		for(int j = 0; j < m.nnode[c]; j++) {
			const int e = m.esuel[static_cast<size_t>(c)*m.maxnfael+j];
			if(e >= 0 && e < m.nelem && loc[e] >= 0) out[k++] = loc[e];
		}
		return k;
	};
	std::vector<int> queue;
	queue.reserve(n);
	auto bfs = [&](int root) {                  // distances from root inside its component; returns farthest
		queue.clear();
		dist[root] = 0; queue.push_back(root);
		int last = root;
		for(size_t q = 0; q < queue.size(); q++) {
			const int a = queue[q];
			last = a;
			int nb[4];
			const int k = nbrs(sub[a], nb);
			for(int j = 0; j < k; j++) if(dist[nb[j]] < 0) { dist[nb[j]] = dist[a] + 1; queue.push_back(nb[j]); }
		}
		return last;
	};
	// grow the first part breadth-first, component by component
	std::vector<int> order;
	order.reserve(n);
	std::vector<char> done(n, 0);
	for(int seed = 0; seed < n && static_cast<int>(order.size()) < n; seed++) {
		if(done[seed]) continue;
		int root = seed;
		for(int rep = 0; rep < 2; rep++) {       // pseudo-peripheral cell of this component
			const int far = bfs(root);
			for(const int a : queue) dist[a] = -1;
			root = far;
		}
		bfs(root);
		for(const int a : queue) { done[a] = 1; order.push_back(a); dist[a] = -1; }
	}
	// side 0 = the BFS prefix whose weight comes closest to the target tw
	for(int i = 0; i < n; i++) side[i] = 1;
	long long w0 = 0;
	for(int i = 0; i < n; i++) {
		const int a = order[i];
		if(w0 + w(a) > tw && (w0 + w(a) - tw) >= (tw - w0)) break;
		side[a] = 0; w0 += w(a);
	}
	// refinement: swap the best-gain boundary cells of the two sides while the swap cuts edges
	auto gain = [&](int a) {
		int nb[4];
		const int k = nbrs(sub[a], nb);
		int ext = 0, in = 0;
		for(int j = 0; j < k; j++) (side[nb[j]] != side[a] ? ext : in)++;
		return ext - in;
	};
	for(int pass = 0; pass < 12; pass++) {
		std::vector<std::pair<int,int>> cand[2];
		for(int a = 0; a < n; a++) {
			const int g = gain(a);
			if(g > -2) cand[side[a]].push_back({-g, a});
		}
		for(auto& c : cand) std::sort(c.begin(), c.end());
		size_t i0 = 0, i1 = 0;
		int moved = 0;
		while(i0 < cand[0].size() && i1 < cand[1].size()) {
			const int a = cand[0][i0].second, b = cand[1][i1].second;
			if(side[a] != 0) { i0++; continue; }
			if(side[b] != 1) { i1++; continue; }
			const int ga = gain(a), gb = gain(b);
			int nb[4], adj = 0;
			const int k = nbrs(sub[a], nb);
			for(int j = 0; j < k; j++) if(nb[j] == b) adj = 1;
			// a swap of unequal weights may move the balance by at most the largest weight
			const long long w0n = w0 - w(a) + w(b);
			const bool balanced = w0n == w0 || std::llabs(w0n - tw) <= std::max(std::llabs(w0 - tw), wmax);
			if(ga + gb - 2*adj <= 0 || !balanced) {
				// the stale-sorted lists ran out of improving pairs
				if(ga <= 0 && -cand[0][i0].first <= 0) break;
				if(ga < gb) i0++; else i1++;
				continue;
			}
			side[a] = 1; side[b] = 0;
			w0 = w0n;
			i0++; i1++; moved++;
		}
		if(!moved) break;
	}
	// connectivity: a side's small components (cut off by the swaps) join the other side, and the
	// balance is restored by moving the best-gain boundary cells back
	std::vector<int> comp(n);
	for(int round = 0; round < 4; round++) {
		std::fill(comp.begin(), comp.end(), -1);
		std::vector<int> csize, cside;
		for(int a0 = 0; a0 < n; a0++) {
			if(comp[a0] >= 0) continue;
			const int id = static_cast<int>(csize.size());
			queue.clear(); queue.push_back(a0); comp[a0] = id;
			for(size_t q = 0; q < queue.size(); q++) {
				int nb[4];
				const int k = nbrs(sub[queue[q]], nb);
				for(int j = 0; j < k; j++)
					if(comp[nb[j]] < 0 && side[nb[j]] == side[a0]) { comp[nb[j]] = id; queue.push_back(nb[j]); }
			}
			csize.push_back(static_cast<int>(queue.size())); cside.push_back(side[a0]);
		}
		int big[2] = {-1, -1};
		for(size_t c = 0; c < csize.size(); c++)
			if(big[cside[c]] < 0 || csize[c] > csize[big[cside[c]]]) big[cside[c]] = static_cast<int>(c);
		bool flipped = false;
		for(int a = 0; a < n; a++)
			if(comp[a] != big[side[a]]) { side[a] = 1 - side[a]; flipped = true; }
		if(!flipped) break;
		// restore the balance: move the best-gain cell off the heavier side while that brings side 0's
		// weight closer to the target (ties: the lowest local id). One max-heap of (gain, -id) per side
		// with lazy entries: a popped entry whose gain is stale goes back with the current one, a move
		// pushes its neighbours' new gains, and a cell too heavy to bring the weight closer now never will
		// be (|w0 - tw| only falls) -- the same sequence of moves as a full scan per move, in O(n log n)
		w0 = 0;
		for(int a = 0; a < n; a++) if(side[a] == 0) w0 += w(a);
		if(w0 != tw) {
			std::priority_queue<std::pair<int,int>> heap[2];
			for(int a = 0; a < n; a++) heap[side[a]].push({gain(a), -a});
			while(w0 != tw) {
				const int from = w0 > tw ? 0 : 1;
				int best = -1;
				while(!heap[from].empty()) {
					const auto top = heap[from].top();
					const int a = -top.second;
					heap[from].pop();
					if(side[a] != from) continue;
					const int g = gain(a);
					if(g != top.first) { heap[from].push({g, -a}); continue; }
					const long long w0n = from == 0 ? w0 - w(a) : w0 + w(a);
					if(std::llabs(w0n - tw) >= std::llabs(w0 - tw)) continue;
					best = a;
					break;
				}
				if(best < 0) break;
				side[best] = 1 - from;
				w0 += from == 0 ? -w(best) : w(best);
				heap[side[best]].push({gain(best), -best});
				int nb[4];
				const int k = nbrs(sub[best], nb);
				for(int j = 0; j < k; j++) heap[side[nb[j]]].push({gain(nb[j]), -nb[j]});
			}
		}
	}
	for(int i = 0; i < n; i++) loc[sub[i]] = -1;
}

void graphRecurse(const fvhip_mesh& m, std::vector<int>& sub, int p0, int np, const int* wt, int* part,
                  std::vector<int>& loc, std::vector<int>& dist)
{
	if(np == 1) { for(const int c : sub) part[c] = p0; return; }
	const int npl = np/2;
	const int n = static_cast<int>(sub.size());
	long long W = 0;
	for(const int c : sub) W += wt ? wt[c] : 1;
	std::vector<int> side(n);
	graphBisect(m, sub, (W*npl)/np, wt, side, loc, dist);
	std::vector<int> a, b;
	for(int i = 0; i < n; i++) (side[i] == 0 ? a : b).push_back(sub[i]);
	sub.clear(); sub.shrink_to_fit();
	graphRecurse(m, a, p0, npl, wt, part, loc, dist);
	graphRecurse(m, b, p0 + npl, np - npl, wt, part, loc, dist);
}

}

std::vector<int> partitionGraph(const fvhip_mesh& m, int nparts, const int* weight)
{
	if(nparts < 1) throw std::invalid_argument("partitionGraph: nparts < 1");
	if(m.nconnface != 0) throw std::invalid_argument("partitionGraph: expects the single-domain mesh");
	checkLinearCells(m, "partitionGraph");
	if(weight)
		for(int e = 0; e < m.nelem; e++)
			if(weight[e] < 1 || weight[e] > 4096) throw std::invalid_argument("partitionGraph: cell weights must lie in 1..4096");
	std::vector<int> part(m.nelem, 0), sub(m.nelem), loc(m.nelem, -1), dist(m.nelem, -1);
	std::iota(sub.begin(), sub.end(), 0);
	if(m.nelem > 0) graphRecurse(m, sub, 0, nparts, weight, part.data(), loc, dist);
	return part;
}

long long edgeCut(const fvhip_mesh& m, const int* part)
{
	long long cut = 0;
	for(int f = m.nbface; f < m.naface; f++) {
		const int l = m.intfac[4*static_cast<size_t>(f)], r = m.intfac[4*static_cast<size_t>(f)+1];
		if(r < m.nelem && part[l] != part[r]) cut++;
	}
	return cut;
}

MeshTopo topoFromMesh(const fvhip_mesh& m)
{
	if(m.nconnface != 0)
		throw std::runtime_error("mesh with connectivity faces: pass the global mesh and a partition instead");
	checkLinearCells(m, "fvhip_create");
	MeshTopo T;
	const int N = m.nelem, nb = m.nbface, F = m.naface;
	T.nown = N; T.nghost = 0; T.nbface = nb; T.naface = F;
	T.cell_global.resize(N); std::iota(T.cell_global.begin(), T.cell_global.end(), 0);
	T.nfael.resize(N);
	T.cell_faces.assign(4*static_cast<size_t>(N), -1);
	T.cell_esuel.assign(4*static_cast<size_t>(N), -1);
	T.clength.resize(N);
	for(int e = 0; e < N; e++) {
		T.nfael[e] = m.nnode[e];
		for(int j = 0; j < m.nnode[e]; j++) {
			T.cell_faces[4*static_cast<size_t>(e)+j] = m.elemface[static_cast<size_t>(e)*m.maxnfael+j];
			T.cell_esuel[4*static_cast<size_t>(e)+j] = m.esuel[static_cast<size_t>(e)*m.maxnfael+j];
		}
		T.clength[e] = cellLength(m, e);
	}
	T.rc.assign(m.rc, m.rc + 2*static_cast<size_t>(N));
	T.area.assign(m.area, m.area + N);
	T.face_global.resize(F); std::iota(T.face_global.begin(), T.face_global.end(), 0);
	T.L.resize(F); T.R.resize(F);
	for(int f = 0; f < F; f++) { T.L[f] = m.intfac[4*static_cast<size_t>(f)]; T.R[f] = m.intfac[4*static_cast<size_t>(f)+1]; }
	T.facemetric.assign(m.facemetric, m.facemetric + 3*static_cast<size_t>(F));
	T.gr.assign(m.gr, m.gr + 2*static_cast<size_t>(F));
	T.btag.resize(nb);
	for(int f = 0; f < nb; f++) T.btag[f] = m.btags[static_cast<size_t>(f)*m.nbtag];
	T.rcbp.assign(m.rcbp, m.rcbp + 2*static_cast<size_t>(nb));
	T.ghost_start.assign(1, 0);
	T.send_start.assign(1, 0);
	return T;
}

MeshTopo topoFromRankMesh(const fvhip_mesh& m)
{
	const int N = m.nelem, nb = m.nbface, F = m.naface, nc = m.nconnface;
	if(nc <= 0 || !m.connface) throw std::invalid_argument("per-rank mesh: connface missing");
	checkLinearCells(m, "per-rank mesh");
	const int cs = F - nc;                                  // gConnBFaceStart
	auto C = [&](int ic, int k) { return m.connface[5*static_cast<size_t>(ic)+k]; };
	std::vector<int> order(nc);
	std::iota(order.begin(), order.end(), 0);
	std::sort(order.begin(), order.end(), [&](int a, int b) {
		return C(a,2) < C(b,2) || (C(a,2) == C(b,2) && (C(a,4) < C(b,4) || (C(a,4) == C(b,4) && a < b))); });
	std::vector<int> gpos(nc);
	for(int i = 0; i < nc; i++) gpos[order[i]] = i;
	for(int ic = 0; ic < nc; ic++) {
		const int f = cs + ic;
		if(m.intfac[4*static_cast<size_t>(f)] != C(ic,0) || m.intfac[4*static_cast<size_t>(f)+1] != N + ic)
			throw std::invalid_argument("per-rank mesh: connectivity faces are not the last faces of intfac");
	}
	MeshTopo T;
	T.nown = N; T.nghost = nc; T.nbface = nb; T.naface = F;
	const int NT = N + nc;
	auto remap = [&](int code) {          // reference neighbour code -> local code
		if(code < 0) return code;
		if(code < N) return code;
		if(code < N + nc) return N + gpos[code - N];
		return code;                        // physical boundary: nelem+nconnface+iface = NT + iface
	};
	T.cell_global.resize(NT);
	std::iota(T.cell_global.begin(), T.cell_global.begin() + N, 0);
	T.ghost_row.resize(nc);
	for(int ic = 0; ic < nc; ic++) { T.cell_global[N + gpos[ic]] = C(ic,3); T.ghost_row[gpos[ic]] = N + ic; }
	T.nfael.resize(N);
	T.cell_faces.assign(4*static_cast<size_t>(N), -1);
	T.cell_esuel.assign(4*static_cast<size_t>(N), -1);
	T.clength.resize(N);
	for(int e = 0; e < N; e++) {
		T.nfael[e] = m.nnode[e];
		for(int j = 0; j < m.nnode[e]; j++) {
			T.cell_faces[4*static_cast<size_t>(e)+j] = m.elemface[static_cast<size_t>(e)*m.maxnfael+j];
			T.cell_esuel[4*static_cast<size_t>(e)+j] = remap(m.esuel[static_cast<size_t>(e)*m.maxnfael+j]);
		}
		T.clength[e] = cellLength(m, e);
	}
	T.rc.resize(2*static_cast<size_t>(NT));
	for(int c = 0; c < N; c++) { T.rc[2*c] = m.rc[2*c]; T.rc[2*c+1] = m.rc[2*c+1]; }
	for(int ic = 0; ic < nc; ic++)
		for(int d = 0; d < 2; d++) T.rc[2*static_cast<size_t>(N + gpos[ic])+d] = m.rc[2*static_cast<size_t>(N + ic)+d];
	T.area.assign(m.area, m.area + N);
	T.face_global.resize(F); std::iota(T.face_global.begin(), T.face_global.end(), 0);
	T.L.resize(F); T.R.resize(F);
	for(int f = 0; f < F; f++) {
		T.L[f] = m.intfac[4*static_cast<size_t>(f)];
		T.R[f] = remap(m.intfac[4*static_cast<size_t>(f)+1]);
	}
	T.facemetric.assign(m.facemetric, m.facemetric + 3*static_cast<size_t>(F));
	T.gr.assign(m.gr, m.gr + 2*static_cast<size_t>(F));
	T.btag.resize(nb);
	for(int f = 0; f < nb; f++) T.btag[f] = m.btags[static_cast<size_t>(f)*m.nbtag];
	T.rcbp.assign(m.rcbp, m.rcbp + 2*static_cast<size_t>(nb));
	// neighbour ranks and the exchange lists
	T.ghost_start.push_back(0);
	T.send_start.push_back(0);
	for(int i = 0; i < nc; i++) {
		const int q = C(order[i], 2);
		if(T.nbr_rank.empty() || T.nbr_rank.back() != q) {
			if(!T.nbr_rank.empty()) { T.ghost_start.push_back(i); T.send_start.push_back(i); }
			T.nbr_rank.push_back(q);
		}
		T.send_cells.push_back(C(order[i], 0));
	}
	T.ghost_start.push_back(nc);
	T.send_start.push_back(nc);
	return T;
}

MeshTopo extractPartition(const fvhip_mesh& m, const int* part, int rank, int layers)
{
	if(m.nconnface != 0) throw std::runtime_error("extractPartition: expects the single-domain mesh");
	checkLinearCells(m, "extractPartition");
	if(layers != 1 && layers != 2) throw std::invalid_argument("extractPartition: layers must be 1 or 2");
	const int N = m.nelem, nb = m.nbface, F = m.naface;
	auto Lg = [&](int f) { return m.intfac[4*static_cast<size_t>(f)]; };
	auto Rg = [&](int f) { return m.intfac[4*static_cast<size_t>(f)+1]; };
	auto esuel = [&](int e, int j) { return m.esuel[static_cast<size_t>(e)*m.maxnfael+j]; };
	MeshTopo T;
	T.halo_layers = layers;
	std::vector<int> loc(N, -1);
	for(int e = 0; e < N; e++) if(part[e] == rank) { loc[e] = T.nown++; T.cell_global.push_back(e); }
	if(T.nown == 0) throw std::runtime_error("extractPartition: rank owns no cells");

	// faces touching owned cells, ascending global index; layer-1 ghosts across interior faces
	std::vector<int> ghosts;
	for(int f = 0; f < F; f++) {
		const int l = Lg(f), r = Rg(f);
		const bool lo = part[l] == rank;
		if(f < nb) { if(lo) { T.face_global.push_back(f); T.nbface++; } continue; }
		const bool ro = part[r] == rank;
		if(!lo && !ro) continue;
		T.face_global.push_back(f);
		if(!lo) ghosts.push_back(l);
		if(!ro) ghosts.push_back(r);
	}
	T.naface = static_cast<int>(T.face_global.size());
	std::sort(ghosts.begin(), ghosts.end());
	ghosts.erase(std::unique(ghosts.begin(), ghosts.end()), ghosts.end());
	std::vector<char> layer(N, 0);                 // 1, 2: halo layer of a cell of this rank
	for(const int g : ghosts) layer[g] = 1;
	if(layers == 2) {
		const size_t n1 = ghosts.size();
		for(size_t i = 0; i < n1; i++)
			for(int j = 0; j < m.nnode[ghosts[i]]; j++) {
				const int e = esuel(ghosts[i], j);
				if(e < 0 || e >= N || part[e] == rank || layer[e]) continue;
				layer[e] = 2; ghosts.push_back(e);
			}
	}
	// grouped by owner rank, layer 1 before layer 2, ascending global id
	std::sort(ghosts.begin(), ghosts.end(), [&](int a, int b) {
		return part[a] < part[b] || (part[a] == part[b] && (layer[a] < layer[b] || (layer[a] == layer[b] && a < b))); });
	T.nghost = static_cast<int>(ghosts.size());
	// neighbour ranks: the owners of the ghosts. The relation is symmetric (a cell within two faces of
	// another rank's cell sees that rank's cell within two faces), so they are also the ranks this one
	// sends to
	for(int i = 0; i < T.nghost; i++) {
		const int g = ghosts[i];
		loc[g] = T.nown + i;
		T.cell_global.push_back(g);
		if(T.nbr_rank.empty() || T.nbr_rank.back() != part[g]) {
			if(!T.nbr_rank.empty()) T.ghost_start.push_back(i);
			else T.ghost_start.push_back(0);
			T.nbr_rank.push_back(part[g]);
		}
		if(layer[g] == 1) {
			if(T.ghost_l1_end.size() < T.nbr_rank.size()) T.ghost_l1_end.push_back(i + 1);
			else T.ghost_l1_end.back() = i + 1;
		} else if(T.ghost_l1_end.size() < T.nbr_rank.size()) T.ghost_l1_end.push_back(i);
	}
	if(T.nbr_rank.empty()) T.ghost_start.push_back(0);
	else T.ghost_start.push_back(T.nghost);
	const int NT = T.ncell();

	// faces
	std::vector<int> floc(F, -1);
	T.L.resize(T.naface); T.R.resize(T.naface);
	T.facemetric.resize(3*static_cast<size_t>(T.naface)); T.gr.resize(2*static_cast<size_t>(T.naface));
	for(int i = 0; i < T.naface; i++) {
		const int f = T.face_global[i];
		floc[f] = i;
		T.L[i] = loc[Lg(f)];
		T.R[i] = f < nb ? NT + i : loc[Rg(f)];
		for(int k = 0; k < 3; k++) T.facemetric[3*static_cast<size_t>(i)+k] = m.facemetric[3*static_cast<size_t>(f)+k];
		for(int k = 0; k < 2; k++) T.gr[2*static_cast<size_t>(i)+k] = m.gr[2*static_cast<size_t>(f)+k];
	}
	T.btag.resize(T.nbface); T.rcbp.resize(2*static_cast<size_t>(T.nbface));
	for(int i = 0; i < T.nbface; i++) {
		const int f = T.face_global[i];
		T.btag[i] = m.btags[static_cast<size_t>(f)*m.nbtag];
		T.rcbp[2*i] = m.rcbp[2*f]; T.rcbp[2*i+1] = m.rcbp[2*f+1];
	}

	// cells
	T.nfael.resize(T.nown);
	T.cell_faces.assign(4*static_cast<size_t>(T.nown), -1);
	T.cell_esuel.assign(4*static_cast<size_t>(T.nown), -1);
	T.area.resize(T.nown); T.clength.resize(T.nown);
	T.rc.resize(2*static_cast<size_t>(NT));
	for(int c = 0; c < NT; c++) {
		const int e = T.cell_global[c];
		T.rc[2*c] = m.rc[2*e]; T.rc[2*c+1] = m.rc[2*e+1];
	}
	for(int c = 0; c < T.nown; c++) {
		const int e = T.cell_global[c];
		T.area[c] = m.area[e];
		T.clength[c] = cellLength(m, e);
		T.nfael[c] = m.nnode[e];
		for(int j = 0; j < m.nnode[e]; j++) {
			const int f = m.elemface[static_cast<size_t>(e)*m.maxnfael+j];
			T.cell_faces[4*static_cast<size_t>(c)+j] = floc[f];
			const int nbr = esuel(e, j);
			T.cell_esuel[4*static_cast<size_t>(c)+j] = nbr >= N ? NT + floc[f] : loc[nbr];
		}
	}

	// layer-1 ghosts: neighbour lists in ascending global face order for their local gradients;
	// physical boundary faces that touch no owned cell become "extra" boundary faces
	if(layers == 2) {
		std::vector<int> xbloc;
		std::map<int,int> xbof;
		for(int i = 0; i < T.nghost; i++) {
			const int g = ghosts[i];
			if(layer[g] != 1) continue;
			T.g1_cells.push_back(T.nown + i);
			int fs[4];
			const int k = m.nnode[g];
			for(int j = 0; j < k; j++) fs[j] = m.elemface[static_cast<size_t>(g)*m.maxnfael+j];
			std::sort(fs, fs + k);
			for(int j = 0; j < 4; j++) {
				if(j >= k) { T.g1_nbr.push_back(-1); continue; }
				const int f = fs[j];
				if(f < nb) {
					auto it = xbof.find(f);
					int x;
					if(it != xbof.end()) x = it->second;
					else {
						x = static_cast<int>(T.xb_btag.size());
						xbof[f] = x;
						T.xb_btag.push_back(m.btags[static_cast<size_t>(f)*m.nbtag]);
						T.xb_n.push_back(m.facemetric[3*static_cast<size_t>(f)]);
						T.xb_n.push_back(m.facemetric[3*static_cast<size_t>(f)+1]);
						T.xb_rcbp.push_back(m.rcbp[2*static_cast<size_t>(f)]);
						T.xb_rcbp.push_back(m.rcbp[2*static_cast<size_t>(f)+1]);
					}
					T.g1_nbr.push_back(-2 - x);
					continue;
				}
				const int other = Lg(f) != g ? Lg(f) : Rg(f);
				if(loc[other] < 0) throw std::logic_error("extractPartition: layer-2 halo incomplete");
				T.g1_nbr.push_back(loc[other]);
			}
			for(int j = 0; j < 4; j++)
				for(int d = 0; d < 2; d++) T.g1_gr.push_back(j < k ? m.gr[2*static_cast<size_t>(fs[j])+d] : 0.0);
			T.g1_clength.push_back(cellLength(m, g));
		}
	}

	// send lists: per neighbour rank q, the owned cells q holds as ghosts, in q's order (layer, global
	// id); the layer of an owned cell for q is its face distance (1 or 2) to q's cells
	std::vector<std::vector<std::pair<int,int>>> sends(T.nbr_rank.size());
	std::vector<int> kof;
	{
		int maxr = 0;
		for(const int q : T.nbr_rank) maxr = std::max(maxr, q);
		kof.assign(maxr + 1, -1);
		for(size_t k = 0; k < T.nbr_rank.size(); k++) kof[T.nbr_rank[k]] = static_cast<int>(k);
	}
	std::vector<int> dq;                             // (rank, distance) seen from one owned cell
	for(int c = 0; c < T.nown; c++) {
		const int e = T.cell_global[c];
		dq.clear();
		for(int j = 0; j < m.nnode[e]; j++) {
			const int a = esuel(e, j);
			if(a < 0 || a >= N) continue;
			if(part[a] != rank) { dq.push_back(part[a]); dq.push_back(1); }
			if(layers < 2) continue;
			for(int jj = 0; jj < m.nnode[a]; jj++) {
				const int b = esuel(a, jj);
				if(b < 0 || b >= N || part[b] == rank) continue;
				dq.push_back(part[b]); dq.push_back(2);
			}
		}
		for(size_t i = 0; i < dq.size(); i += 2) {
			const int q = dq[i];
			int d = dq[i+1];
			bool first = true;
			for(size_t i2 = 0; i2 < dq.size(); i2 += 2) {
				if(dq[i2] != q) continue;
				if(dq[i2+1] < d || (dq[i2+1] == d && i2 < i)) { first = false; break; }
			}
			if(!first) continue;
			if(q >= static_cast<int>(kof.size()) || kof[q] < 0) throw std::logic_error("extractPartition: halo not symmetric");
			sends[kof[q]].push_back({d, e});
		}
	}
	T.send_start.push_back(0);
	for(size_t k = 0; k < T.nbr_rank.size(); k++) {
		std::sort(sends[k].begin(), sends[k].end());
		int n1 = 0;
		for(const auto& s : sends[k]) { T.send_cells.push_back(loc[s.second]); n1 += s.first == 1; }
		T.send_l1_end.push_back(T.send_start.back() + n1);
		T.send_start.push_back(static_cast<int>(T.send_cells.size()));
	}
	if(layers == 1) { T.ghost_l1_end.assign(T.ghost_start.begin() + 1, T.ghost_start.end()); }
	return T;
}

}
