/** \file krylov.hpp
 * \brief Device linear algebra of the implicit pseudo-time solver (krylov.hip): the point-block
 *   Jacobi preconditioner on the assembled 4x4 Jacobian blocks, deterministic multi-dot products
 *   and multi-AXPYs for restarted GMRES, and the nonlinear update of
 *   SteadyBackwardEulerSolver::solve (aodesolver.cpp:494-530, nonlinearrelaxation.cpp:24-38).
 *
 * They replace what the reference hands to PETSc (KSPSolve with GMRES and a block-Jacobi / SOR
 * preconditioner, aodesolver.cpp:483, casesolvers.cpp:166-201), so that Krylov vectors never leave
 * HBM. Every reduction uses a fixed partition and a fixed tree: results are
 * bitwise reproducible from run to run.
 */
#ifndef FVHIP_KRYLOV_HPP
#define FVHIP_KRYLOV_HPP

#include <hip/hip_runtime.h>
#include <cstddef>
#include "gasdyn.hpp"

namespace fvhip {

constexpr int KRY_MAXK = 128;     ///< largest GMRES restart length

/// FlowSimpleUpdate::getLocalRelaxationFactor (nonlinearrelaxation.cpp:24-38) with
/// IdealGasPhysics::getDeltaPressureFromConserved (aphysics_defs.hpp:67-80) as written there: its
/// momentum loop runs over i = 2 .. NDIM+1 (y-momentum and energy), and that is what is restated.
/// minfactor >= 1 means FullUpdate (nonlinearrelaxation.hpp:32-38): omega = 1.
FVHIP_HD double relaxation_factor(const gd::Gas& G, double minfactor, const double* du, const double* u)
{
	if(minfactor >= 1.0) return 1.0;
	const double p = gd::pressure_cons(G, u);
	double unew[4];
	for(int i = 0; i < 4; i++) unew[i] = u[i] + du[i];
	double dp = 0;
	for(int i = 2; i < 4; i++)
		dp -= ((u[i]+unew[i])*(u[0]+unew[0])/2.0*du[i] - (unew[i]*unew[i]+u[i]*u[i])/2.0*du[0]);
	dp = (G.g-1.0)*(du[3] - 1.0/(2*u[0]*unew[0])*dp);
	const double rdp = fabs(dp)/p;
	const double drho = fabs(du[0])/u[0];
	const double danger = rdp < drho ? drho : rdp;      // std::max(dp, drho)
	double omega = minfactor;
	if(danger < 1.0-minfactor) omega = 1.0-danger;
	return omega;
}

/// Lines of the line-implicit preconditioner (internal cell ids), sorted by length (longest first) and
/// dealt to groups of 64: lane j of group g walks line 64g + j, so one wave runs 64 recurrences side by
/// side. Everything per line cell is stored line-interleaved: row r = gstart[g] + k holds step k of the
/// group's 64 lines, slot r*64 + lane; a 4x4 block of row r is pair-interleaved, elements 2q, 2q+1 at
/// double2 index 512 r + 64 q + lane (one coalesced 16-byte load per element pair across the 64
/// lines). cell[slot] = the lane's k-th line cell or -1 once its line has ended; face[slot] (k > 0) =
/// interior face between its cells k-1 and k, fi<<1 | (cell k-1 is R); len[64 g + lane] = the lane's
/// line length (0: no line).
/// Device arrays written by the factorisation and read by the solve: D = dinvp_k (the inverted pivot
/// blocks), Lb = A[k][k-1], W = dinvp_k A[k][k+1]; G = forward-sweep scratch [rows][4][64].
struct LineSet {
	int nlines = 0, ngroups = 0;
	long long nrows = 0;             ///< rows over all groups (slots = 64 nrows)
	const int* gstart = nullptr;     ///< [ngroups+1]
	const int* cell = nullptr;       ///< [64 nrows]
	const int* face = nullptr;       ///< [64 nrows]
	const int* len = nullptr;        ///< [64 ngroups]
	int twisted_groups = 0;          ///< leading groups of 32 lines solved from both ends (lanes j, j+32)
	double *D = nullptr, *Lb = nullptr, *W = nullptr, *G = nullptr;
	double* zpart = nullptr;         ///< [ngroups] per-group sums of z.z (launch_line_solve with a norm)
	bool single = false;             ///< D, Lb, W held in fp32 (prec_single; float4 rows in the same buffers)
};
#ifndef FVHIP_LINE_MAX
#define FVHIP_LINE_MAX 256
#endif
constexpr int LINE_MAX_CELLS = FVHIP_LINE_MAX;   ///< longest line piece (ctx.hpp ensureLines)
#ifndef FVHIP_LINE_TWIST_MIN
#define FVHIP_LINE_TWIST_MIN 16
#endif
constexpr int LINE_TWIST_MIN = FVHIP_LINE_TWIST_MIN;   ///< shortest line solved from both ends
/// block-Thomas factorisation of every line (D, Lb, W of the line set) from the block operator
void launch_line_factor(const LineSet& Ls, const double* diag, const double* lower, const double* upper, hipStream_t s);
/// z = (block-tridiagonal line part of A)^-1 v; with zsq, also zsq[0] = z.z over the solved rows (each
/// lane sums the rows it writes, a fixed shuffle tree per group, a fixed-tree sum over the groups)
void launch_line_solve(const LineSet& Ls, const double* v, double* z, hipStream_t s, double* zsq = nullptr);
/// z += e over n cells
void launch_add_rows(int n, const double* e, double* z, hipStream_t s);
/// block ILU(0) in multicolour order, colour q's rows: dinv[c] = (A_cc - sum_{earlier-colour owned
/// neighbours k} A_ck dinv[k] A_kc)^-1 for the n listed cells (k_ilu_factor_colour)
void launch_ilu_factor_colour(int ncell, int nbface, const int4* rfaces, const int4* nbrs, const int* colour, int q,
                              const double* diag, const double* lower, const double* upper, double* dinv,
                              const int* cells, int n, hipStream_t s);
/// dinv[c] = diag[c]^-1 (Gauss-Jordan with row pivoting), c < ncell
void launch_bjac_invert(int ncell, const double* diag, double* dinv, hipStream_t s);
/// y[c] = dinv[c] x[c]
void launch_bjac_apply(int ncell, const double* dinv, const double* x, double* y, hipStream_t s);
void launch_bjac_apply(int ncell, const float* dinv, const double* x, double* y, hipStream_t s);
/// b = fp32(a), n a multiple of 4
void launch_to_single(long long n, const double* a, float* b, hipStream_t s);
/// z[c] += dinv[c] (b[c] - y[c]): one block-Jacobi sweep on A z = b, given y = A z
void launch_bjac_correct(int ncell, const double* dinv, const double* b, const double* y, double* z, hipStream_t s);

/// doubles of scratch `part` launch_mdot needs for up to k products
size_t kry_scratch(int k);
/// out[j] = V_j . w for j < k (V_j = V + j*ld) and, if self, out[k] = w . w; fixed-order sums
void launch_mdot(long long n, int k, const double* V, long long ld, const double* w, bool self,
                 double* part, double* out, hipStream_t s);
/// w -= sum_{j<k} h[j] V_j  (h: k doubles on the device; ascending j for every element)
void launch_maxpy(long long n, int k, const double* V, long long ld, const double* h, double* w, hipStream_t s);
/// w -= V h and out[0] = |w|^2 of the result (fixed partition and tree: reproducible); part: kry_scratch(1)
void launch_maxpy_norm(long long n, int k, const double* V, long long ld, const double* h, double* w, double* part,
                       double* out, hipStream_t s);
/// out = sum_{j<k} c[j] V_j  (c on the device)
void launch_lincomb(long long n, int k, const double* V, long long ld, const double* c, double* out, hipStream_t s);
/// y = a*x + b*y  (b == 0: y = a*x and y is not read)
void launch_axpby(long long n, double a, const double* x, double b, double* y, hipStream_t s);
/// pm[0] = sqrt(sq[0]), pm[1] = eps/pm[0]: the matrix-free step from a global sum of squares
/// (alinalg.cpp:159-167)
void launch_pertmag(const double* sq, double eps, double* pm, hipStream_t s);
/// out[0] = sum_e r[e][3]^2 area[e] (aodesolver.cpp:216-223, 516-526), fixed order
void launch_energy_sumsq(int ncell, const double* r, const double* area, double* part, double* out, hipStream_t s);
/// u[c] += omega(du[c], u[c]) du[c] (aodesolver.cpp:506-511)
void launch_relaxed_update(int ncell, const gd::Gas& G, double minfactor, const double* du, double* u,
                           hipStream_t s);

}
#endif
