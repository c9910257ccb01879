/** \file amg.cpp
 * \brief Host setup of the aggregation multigrid preconditioner (amg.hpp): aggregation of one level's
 *   graph along strong couplings, the coarse block pattern, the Galerkin contribution lists, member lists
 *   and the multicolour order of the coarse level. Everything is built in a fixed order (rows ascending),
 *   so the hierarchy and every device sum over it are the same on every run.
 */
#include "amg.hpp"

#include <algorithm>
#include <stdexcept>

namespace fvhip {

AmgLevelHost amgCoarsen(const AmgGraph& g, double threshold)
{
	const int n = g.n;
	if(n <= 0) throw std::invalid_argument("amgCoarsen: empty level");
	std::vector<double> wmax(static_cast<size_t>(n), 0.0);
	for(int i = 0; i < n; i++)
		for(int e = g.rowptr[i]; e < g.rowptr[i+1]; e++) wmax[i] = std::max(wmax[i], g.w[e]);
	auto strong = [&](int i, int e) {
		const int j = g.col[e];
		return g.w[e] >= threshold*wmax[i] && g.w[e] >= threshold*wmax[j];
	};
	// aggregation (Vanek, Mandel & Brezina): roots whose strong neighbours are all free take them (pass 1),
	// the remaining cells join the pass-1 aggregate of their strongest strong neighbour (pass 2), what is
	// left forms aggregates with its free strong neighbours (pass 3)
	std::vector<int> agg(static_cast<size_t>(n), -1);
	int na = 0;
	for(int i = 0; i < n; i++) {
		if(agg[i] >= 0) continue;
		bool any = false, free = true;
		for(int e = g.rowptr[i]; e < g.rowptr[i+1]; e++)
			if(strong(i, e)) { any = true; if(agg[g.col[e]] >= 0) { free = false; break; } }
		if(!any || !free) continue;
		agg[i] = na;
		for(int e = g.rowptr[i]; e < g.rowptr[i+1]; e++) if(strong(i, e)) agg[g.col[e]] = na;
		na++;
	}
	const std::vector<int> p1(agg);
	for(int i = 0; i < n; i++) {
		if(agg[i] >= 0) continue;
		int best = -1;
		double bw = -1.0;
		for(int e = g.rowptr[i]; e < g.rowptr[i+1]; e++)
			if(strong(i, e) && p1[g.col[e]] >= 0 && g.w[e] > bw) { bw = g.w[e]; best = p1[g.col[e]]; }
		if(best >= 0) agg[i] = best;
	}
	for(int i = 0; i < n; i++) {
		if(agg[i] >= 0) continue;
		agg[i] = na;
		for(int e = g.rowptr[i]; e < g.rowptr[i+1]; e++) if(strong(i, e) && agg[g.col[e]] < 0) agg[g.col[e]] = na;
		na++;
	}
	AmgLevelHost L;
	L.n = na;
	L.agg = agg;
	// members of each aggregate, ascending
	L.mstart.assign(static_cast<size_t>(na) + 1, 0);
	for(int i = 0; i < n; i++) L.mstart[agg[i] + 1]++;
	for(int a = 0; a < na; a++) L.mstart[a+1] += L.mstart[a];
	L.members.resize(static_cast<size_t>(n));
	{
		std::vector<int> pos(L.mstart.begin(), L.mstart.end() - 1);
		for(int i = 0; i < n; i++) L.members[pos[agg[i]]++] = i;
	}
	// coarse pattern: I and the aggregates of its members' neighbours, ascending
	L.rowptr.assign(static_cast<size_t>(na) + 1, 0);
	std::vector<int> tmp;
	for(int a = 0; a < na; a++) {
		tmp.assign(1, a);
		for(int m = L.mstart[a]; m < L.mstart[a+1]; m++) {
			const int i = L.members[m];
			for(int e = g.rowptr[i]; e < g.rowptr[i+1]; e++) tmp.push_back(agg[g.col[e]]);
		}
		std::sort(tmp.begin(), tmp.end());
		tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
		L.col.insert(L.col.end(), tmp.begin(), tmp.end());
		L.rowptr[a+1] = static_cast<int>(L.col.size());
	}
	const int nnz = L.rowptr[na];
	L.dpos.resize(static_cast<size_t>(na));
	auto find = [&](int a, int b) {
		const auto first = L.col.begin() + L.rowptr[a], last = L.col.begin() + L.rowptr[a+1];
		const auto it = std::lower_bound(first, last, b);
		if(it == last || *it != b) throw std::logic_error("amgCoarsen: pattern");
		return static_cast<int>(it - L.col.begin());
	};
	for(int a = 0; a < na; a++) L.dpos[a] = find(a, a);
	// Galerkin contributions (k, finer block) and the coarse couplings
	std::vector<std::pair<int,int>> pr;
	pr.reserve(static_cast<size_t>(n) + g.col.size());
	L.w.assign(static_cast<size_t>(nnz), 0.0);
	for(int i = 0; i < n; i++) {
		const int a = agg[i];
		pr.push_back({L.dpos[a], g.dblk[i]});
		for(int e = g.rowptr[i]; e < g.rowptr[i+1]; e++) {
			const int k = find(a, agg[g.col[e]]);
			pr.push_back({k, g.blk[e]});
			if(agg[g.col[e]] != a) L.w[k] += g.w[e];
		}
	}
	L.cstart.assign(static_cast<size_t>(nnz) + 1, 0);
	for(const auto& p : pr) L.cstart[p.first + 1]++;
	for(int k = 0; k < nnz; k++) L.cstart[k+1] += L.cstart[k];
	L.csrc.resize(pr.size());
	{
		std::vector<int> pos(L.cstart.begin(), L.cstart.end() - 1);
		for(const auto& p : pr) L.csrc[pos[p.first]++] = p.second;
	}
	for(int k = 0; k < nnz; k++) std::sort(L.csrc.begin() + L.cstart[k], L.csrc.begin() + L.cstart[k+1]);
	// greedy colouring in row order
	std::vector<int> colour(static_cast<size_t>(na), -1), mark;
	int ncol = 0;
	for(int a = 0; a < na; a++) {
		for(int k = L.rowptr[a]; k < L.rowptr[a+1]; k++) {
			const int b = L.col[k];
			if(b != a && colour[b] >= 0) {
				if(static_cast<int>(mark.size()) <= colour[b]) mark.resize(static_cast<size_t>(colour[b]) + 1, -1);
				mark[colour[b]] = a;
			}
		}
		int c = 0;
		while(c < static_cast<int>(mark.size()) && mark[c] == a) c++;
		colour[a] = c;
		ncol = std::max(ncol, c + 1);
	}
	L.cstart_colour.assign(static_cast<size_t>(ncol) + 1, 0);
	for(int a = 0; a < na; a++) L.cstart_colour[colour[a] + 1]++;
	for(int q = 0; q < ncol; q++) L.cstart_colour[q+1] += L.cstart_colour[q];
	L.cells.resize(static_cast<size_t>(na));
	{
		std::vector<int> pos(L.cstart_colour.begin(), L.cstart_colour.end() - 1);
		for(int a = 0; a < na; a++) L.cells[pos[colour[a]]++] = a;
	}
	return L;
}

AmgGraph amgGraphOf(const AmgLevelHost& L)
{
	AmgGraph g;
	g.n = L.n;
	g.rowptr.assign(static_cast<size_t>(L.n) + 1, 0);
	g.dblk = L.dpos;
	for(int a = 0; a < L.n; a++) {
		for(int k = L.rowptr[a]; k < L.rowptr[a+1]; k++) {
			if(L.col[k] == a) continue;
			g.col.push_back(L.col[k]);
			g.w.push_back(L.w[k]);
			g.blk.push_back(k);
		}
		g.rowptr[a+1] = static_cast<int>(g.col.size());
	}
	return g;
}

}
