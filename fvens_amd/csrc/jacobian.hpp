/** \file jacobian.hpp
 * \brief Launch interface of the Jacobian / operator kernels (jacobian.hip).
 */
#ifndef FVHIP_JACOBIAN_HPP
#define FVHIP_JACOBIAN_HPP

#include "kernels.hpp"

namespace fvhip {

/// Face-ordered view of the mesh for the Jacobian (reference face numbering, internal cells)
struct JacMesh
{
	int ncell, nbface, ninface;
	const int2* if_LR;          // [Fi] internal left/right cell of interior face nbface+fi
	const double2* if_n;        // [Fi]
	const double* if_len;       // [Fi]
	const int* bf_L;            // [nb]
	const int* bf_bc;           // [nb]
	const double2* bf_n;        // [nb]
	const double* bf_len;       // [nb]
	const double2* bf_rcbp;     // [nb]
	const double2* rc;          // [N]
	const int4* cell_rfaces;    // [N] (reference face << 1 | cell-is-right), ascending, -1 padded
	const int4* cell_nbr_fo;    // [N] neighbour across each of those faces
};

/// lower/upper [Fi][16] and boundary blocks bblk [nb][16] (row-major 4x4); jflux is the Jacobian
/// flux (LLF, AUSM, Roe, HLL, HLLC), visc 0 none / 1 Sutherland / 2 constant
void launch_jac_faces(const JacMesh& J, const DevPhys& P, int jflux, int visc, const double* u, double* bblk,
                      double* lower, double* upper, hipStream_t s);
/// diag[c] = -(sum of the cell's face blocks); with area != nullptr also the pseudo-time term of
/// launch_pseudo_time (dtm[c] <- area/(cfl dtm[c]), diag[c] += dtm[c] I), fused while the block is in registers
void launch_jac_diag(const JacMesh& J, const double* bblk, const double* lower, const double* upper,
                     double* diag, hipStream_t s, const double* area = nullptr, double cfl = 0.0, double* dtm = nullptr);
void launch_pseudo_time(int ncell, const double* area, double cfl, double* dtm, double* diag, hipStream_t s);
void launch_block_apply(const JacMesh& J, const double* diag, const double* lower, const double* upper,
                        const double* x, double* y, hipStream_t s);
/// t = v - A x (A with the ghost coupling: x needs its ghost rows), one pass
void launch_block_residual(const JacMesh& J, const double* diag, const double* lower, const double* upper,
                           const double* x, const double* v, double* t, hipStream_t s);
void launch_block_residual(const JacMesh& J, const float* diag, const float* lower, const float* upper,
                           const double* x, const double* v, double* t, hipStream_t s);
/// zout = D^-1 (v - (A - D) zin): one block-Jacobi sweep (dinv: inverted diagonal blocks)
void launch_bjac_sweep(const JacMesh& J, const double* dinv, const double* lower, const double* upper,
                       const double* v, const double* zin, double* zout, hipStream_t s);
/// the same with fp32 blocks (fp64 vectors and arithmetic)
void launch_bjac_sweep(const JacMesh& J, const float* dinv, const float* lower, const float* upper,
                       const double* v, const double* zin, double* zout, hipStream_t s);
/// one colour of a multicolour block Gauss-Seidel sweep, in place on z (cells: that colour's cells)
void launch_bgs_colour(const JacMesh& J, const double* dinv, const double* lower, const double* upper,
                       const double* v, double* z, const int* cells, int n, hipStream_t s);
void launch_bgs_colour(const JacMesh& J, const float* dinv, const float* lower, const float* upper,
                       const double* v, double* z, const int* cells, int n, hipStream_t s);
/// pm[0] = |x|, pm[1] = eps/|x|; part: mf_partials() doubles of scratch
void launch_mf_norm(long long n, const double* x, double eps, double* part, double* pm, hipStream_t s);
void launch_mf_perturb(long long n, const double* u, const double* x, const double* pm, double* aux, hipStream_t s);
void launch_mf_combine(int ncell, const double* mdt, const double* x, const double* yg, const double* res,
                       const double* pm, double* y, hipStream_t s);
int mf_partials();
void launch_local_jac(int flux, const gd::Gas& G, int nf, const double* ul, const double* ur, const double* n,
                      double* dfdl, double* dfdr, hipStream_t s);

}
#endif
