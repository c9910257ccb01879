/** \file amg.hpp
 * \brief Aggregation multigrid preconditioner for the assembled first-order Jacobian (4x4 blocks): the
 *   device counterpart of the reference's GAMG option for the viscous NACA 0012 case
 *   (testcases/visc-naca0012/mgopts.solverc:1-35: -pc_type gamg -pc_gamg_type agg -pc_gamg_agg_nsmooths 0
 *   -pc_gamg_threshold 0.2 -pc_gamg_reuse_interpolation true -pc_mg_levels 3 -pc_mg_cycle_type v,
 *   Richardson + bjacobi/SOR smoothing with 2 iterations per level, Richardson + bjacobi/ILU coarse solve
 *   with 6 iterations).
 *
 * Setup (host, once per mesh, like -pc_gamg_reuse_interpolation): cells are aggregated along strong
 * couplings of the cell graph -- coupling of two cells = face length / centre distance, the term that
 * dominates the Jacobian blocks of thin cells (the same measure the line-implicit preconditioner uses);
 * strong when at least `threshold` times the strongest coupling of both cells -- so boundary-layer cells
 * aggregate along the wall normal (semi-coarsening). The prolongation is the tentative one (piecewise
 * constant over aggregates: -pc_gamg_agg_nsmooths 0), the coarse operators the Galerkin products
 * A_c = P^T A P, i.e. sums of fine blocks. Every coarse block's list of contributing fine blocks is built
 * on the host in ascending order, so the coarse operators are summed on the device in a fixed order:
 * deterministic, no atomics. Coarse levels are block-sparse rows (diagonal included) with a greedy
 * colouring for the multicolour block Gauss-Seidel smoother.
 *
 * Per Jacobian (each pseudo-time step): the Galerkin sums level by level and the coarse diagonal inverses.
 * Per application: one V-cycle (implicit.cpp LinOp::amgApply) -- on the finest level the one-level
 * preconditioner (line-implicit or block-Jacobi) as smoother, on the coarse levels forward / backward
 * colour Gauss-Seidel, on the coarsest `coarse_sweeps` of them.
 */
#ifndef FVHIP_AMG_HPP
#define FVHIP_AMG_HPP

#include <hip/hip_runtime.h>
#include <vector>

namespace fvhip {

/// one coarse level as built on the host
struct AmgLevelHost
{
	int n = 0;                               ///< block rows
	std::vector<int> rowptr, col, dpos;      ///< block CSR (columns ascending, diagonal included; dpos = its position)
	std::vector<int> cstart, csrc;           ///< per nonzero: contributing blocks of the finer level (ascending)
	std::vector<int> mstart, members;        ///< per row: the finer level's rows aggregated into it (ascending)
	std::vector<int> agg;                    ///< per row of the finer level: its aggregate (row of this level)
	std::vector<int> cstart_colour, cells;   ///< multicolour order: rows of colour q = cells[cstart_colour[q]..]
	std::vector<double> w;                   ///< coupling per nonzero (aggregation of the next level)
};

/// the finer level seen by the aggregation: rows, adjacency with couplings (symmetric), and the block index
/// of each nonzero of the finer operator (finest: diag c -> c, A[R][L] = lower fi -> n + fi, A[L][R] = upper
/// fi -> n + Fi + fi; coarse: the CSR position)
struct AmgGraph
{
	int n = 0;
	std::vector<int> rowptr, col;            ///< off-diagonal adjacency, columns ascending
	std::vector<double> w;                   ///< coupling per adjacency entry
	std::vector<int> blk;                    ///< block index of A[row][col] per adjacency entry
	std::vector<int> dblk;                   ///< block index of A[row][row]
};

/// aggregates graph g (threshold: strength relative to both cells' strongest coupling) and builds the
/// coarse level: pattern, Galerkin contribution lists, member lists, colouring, coarse couplings
AmgLevelHost amgCoarsen(const AmgGraph& g, double threshold);
/// the graph of a built coarse level (for the next aggregation)
AmgGraph amgGraphOf(const AmgLevelHost& L);

/// device arrays of one coarse level
struct AmgLevel
{
	int n = 0, nnz = 0;
	const int *rowptr = nullptr, *col = nullptr, *dpos = nullptr;
	const int *cstart = nullptr, *csrc = nullptr;
	const int *mstart = nullptr, *members = nullptr, *agg = nullptr;
	const int* cells = nullptr;              ///< colour order
	const int* d_cstart_colour = nullptr;    ///< the colour starts on the device (single-workgroup sweeps)
	std::vector<int> cstart_colour;          ///< host copy of the colour starts
	int nfine = 0;                           ///< rows of the finer level
	double *val = nullptr, *dinv = nullptr;  ///< [nnz][16], [n][16]
	double *x = nullptr, *b = nullptr, *r = nullptr;   ///< [n][4]
};

/// val[k] = sum of the listed finer-level blocks (finest: diag / lower / upper by the AmgGraph block index
/// with nfine rows and nif interior faces; else fval)
void launch_amg_galerkin_fine(const AmgLevel& L, int nfine, int nif, const double* diag, const double* lower,
                              const double* upper, hipStream_t s);
void launch_amg_galerkin(const AmgLevel& L, const double* fval, hipStream_t s);
/// dinv[i] = (diagonal block of row i)^-1
void launch_amg_invert(const AmgLevel& L, hipStream_t s);
/// b[I] = sum of r_fine over the members of aggregate I (ascending)
void launch_amg_restrict(const AmgLevel& L, const double* rfine, double* b, hipStream_t s);
/// x_fine[i] += x[agg[i]]
void launch_amg_prolong(const AmgLevel& L, const double* x, double* xfine, hipStream_t s);
/// r = b - A x on a coarse level
void launch_amg_residual(const AmgLevel& L, const double* x, const double* b, double* r, hipStream_t s);
/// one colour of a block Gauss-Seidel sweep on A x = b, in place: x_i = dinv_i (b_i - sum_{j != i} A_ij x_j)
void launch_amg_gs_colour(const AmgLevel& L, int q, const double* b, double* x, hipStream_t s);
/// levels of at most AMG_BLOCK_ROWS rows: `sweeps` whole Gauss-Seidel sweeps (colours forward on even sweeps,
/// backward on odd ones when `alternate`, else all in direction `fwd`) in one workgroup, a barrier between
/// colours -- the same row updates in the same order as per-colour launches, without a launch per colour;
/// zero: x = 0 first. The iterate is held in LDS (32 B a row: 64 KB at the limit)
constexpr int AMG_BLOCK_ROWS = 2048;
void launch_amg_gs_block(const AmgLevel& L, const double* b, double* x, int sweeps, bool fwd, bool alternate,
                         bool zero, hipStream_t s);

}
#endif
