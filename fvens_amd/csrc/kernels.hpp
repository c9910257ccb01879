/** \file kernels.hpp
 * \brief Launch interface of the HIP kernels of the face sweep (kernels.hip).
 */
#ifndef FVHIP_KERNELS_HPP
#define FVHIP_KERNELS_HPP

#include <hip/hip_runtime.h>
#include "gasdyn.hpp"

namespace fvhip {

constexpr int MAXBC = 16;

/// Reconstruction kinds of the fused sweep
enum SweepRec { SR_FIRST = 0, SR_MUSCL = 1, SR_LINEAR = 2 };
/// Viscous kinds
enum SweepVisc { SV_NONE = 0, SV_SUTHERLAND = 1, SV_CONST = 2 };

struct DevMesh
{
	int ncell;                 // owned + ghost cells: a neighbour code >= ncell is a boundary face
	int nown;                  // owned cells (internal ids 0 .. nown-1)
	int nbface, npatch, nslot;
	const int* patch_cell;     // [npatch+1]
	const int* patch_slot;     // [npatch+1]
	const int2* slot_LR;       // [S]
	const double2* slot_n;     // [S]
	const double* slot_len;    // [S]
	const double2* slot_gr;    // [S]
	const int4* cell_slots;    // [N] (slot<<1 | isRight), -1 padded, ascending reference face
	const int4* cell_nbr;      // [N] esuel order neighbours (internal / ncell+bf)
	const int4* cell_face;     // [N] esuel order slots
	const int4* cell_nbr_fo;   // [N] neighbours in ascending reference face order
	const double2* rc;         // [N]
	const double* area;        // [N]
	const double4* wls_V;      // [N] row-major 2x2
	const double* venk_eps2;   // [N]
	const int* bf_L;           // [nb]
	const int* bf_bc;          // [nb]
	const double2* bf_n;       // [nb]
	const double2* bf_rcbp;    // [nb]
	// fused residual (layout.hpp fz_*)
	const int* fz_ext_start;   // [npatch+1]
	const int* fz_ext;         // ring-1 then ring-2 cells
	const int* fz_n1;          // [npatch] ring-1 count
	const int* fz_g_start;     // [npatch+1] first fz_gnbr row of each patch
	const int4* fz_gnbr;       // neighbour codes of the cells whose gradients a patch computes
	const unsigned* fz_slot_lr16;   // [S] patch-local L | R << 16 (R 0xFFFF: boundary face)
	const uint2* fz_gnbr16;    // per gradient row 4 x 16-bit neighbour codes (layout.hpp)
	const int* fz_gbf_start;   // [npatch+1]
	const int* fz_gbf;         // boundary faces of the 0x8000|j codes
	const uint2* fz_cslot16;   // [nown] 4 x 16-bit (patch-local slot << 1 | isRight)
	int fz_max_cells;
	// layer-1 ghosts of a two-layer halo (layout.hpp gg_*, xb_*)
	int gg_n;
	const int* gg_cells;
	const int4* gg_nbr;
	const double4* gg_V;
	const double2* gg_gp;      // [n1][4] face centres (limited reconstructions)
	const double* gg_eps2;     // [n1] Venkatakrishnan eps^2
	const int* xb_bc;
	const double2* xb_n;
	const double2* xb_rcbp;
};

struct DevPhys
{
	gd::Gas gas;
	double uinf[4];
	gd::BCDev bc[MAXBC];
	int nbc;
	double limiter_param;
};

struct SweepBuffers
{
	const double* u;      // [N][4] conserved
	const double* up;     // [N][4] primitive (order 2)
	const double* grad;   // [N][8] primitive gradients (viscous term)
	const double* rgrad;  // [N][8] gradients used for reconstruction (grad, or WENO-limited)
	const double* phi;    // [N][4] limiter values (BJ/Venkatakrishnan) or null
	const double* ubc;    // [nb][4] conserved ghost state of the cell value (order 2)
	const double* ug;     // [nb][4] primitive ghost state of the cell value (order 2)
	double* r;            // [N][4]
	double* dtm;          // [N]
	int overwrite;
	const int* plist;     // patches to sweep (pcount of them), or null: all patches
	int pcount;
	// matrix-free operator fused into the one-launch residual (k_residual_wls without time steps, single
	// domain; MatrixFreeSpatialJacobian::apply, alinalg.cpp:142-233): with mfx set, every state row the
	// kernel reads is u + pm[1] x (k_mf_perturb's arithmetic) and each cell writes, instead of its
	// residual yg, y = mdt x + (-yg + res)/pm[1] (k_mf_combine's) into r
	const double* mfx;    // [N][4] x, or null
	const double* mfpm;   // [2] (|x|, eps/|x|)
	const double* mfres;  // [N][4] -r(u) of the operator's state
	const double* mfmdt;  // [N] pseudo-time diagonal
};

// Host launchers (all asynchronous on stream). kernels.hip is compiled twice: namespace `exact`
// (-ffp-contract=off, IEEE division/sqrt: bitwise parity with the reference) and namespace `fast`
// (contracted FMAs and approximate division/sqrt: the reference's results to a stated tolerance).
#define FVHIP_SWEEP_LAUNCHERS \
void launch_prep(const DevMesh& M, const DevPhys& P, const double* u, double* up, double* ubc, double* ug, \
                 bool cells, hipStream_t s); \
void launch_grad_wls(const DevMesh& M, const double* up, const double* ug, double* grad, hipStream_t s); \
void launch_prep_grad_wls(const DevMesh& M, const DevPhys& P, const double* u, double* up, double* ubc, \
                          double* ug, double* grad, hipStream_t s, int c_begin = 0, int c_end = -1, \
                          int lim = 0, double* phi = nullptr); \
void launch_grad_wls_list(const DevMesh& M, const DevPhys& P, const double* u, const int* list, int n, \
                          double* grad, hipStream_t s); \
void launch_grad_ghost(const DevMesh& M, const DevPhys& P, const double* u, double* grad, hipStream_t s, \
                       int lim = 0, double* phi = nullptr); \
void launch_grad_gg(const DevMesh& M, const double* up, const double* ug, double* grad, hipStream_t s); \
void launch_limiter(const DevMesh& M, const DevPhys& P, int venk, const double* up, const double* ug, \
                    const double* grad, double* phi, hipStream_t s); \
void launch_weno(const DevMesh& M, const DevPhys& P, const double* grad, double* lgrad, hipStream_t s); \
/* returns the kernel name for profiling */ \
const char* launch_sweep(const DevMesh& M, const DevPhys& P, const SweepBuffers& B, int flux, int rec, \
                         int visc, bool dt, hipStream_t s); \
const char* launch_residual_wls(const DevMesh& M, const DevPhys& P, const SweepBuffers& B, int flux, int rec, \
                                int visc, int lim, bool dt, hipStream_t s); \
void launch_fill(double* p, double v, long long n, hipStream_t s); \
void launch_local_flux(int flux, const gd::Gas& G, int nf, const double* ul, const double* ur, \
                       const double* n, double* f, hipStream_t s); \
void launch_gather_cells(const int* perm, const double* src, double* dst, int n, int width, hipStream_t s); \
void launch_scatter_cells(const int* perm, const double* src, double* dst, int n, int width, hipStream_t s); \
void launch_divsqrt_probe(int n, const double* a, const double* b, double* out, hipStream_t s);

namespace exact { FVHIP_SWEEP_LAUNCHERS }
namespace fast { FVHIP_SWEEP_LAUNCHERS }

}
#endif
