/** \file jacobian.hip
 * \brief Analytic first-order Jacobian assembly, pseudo-time diagonal, block operator apply and the
 *   matrix-free finite-difference operator on MI355X.
 *
 * Replaces Spatial::assemble_jacobian (aspatial.cpp:242-340) with
 * FlowFV::compute_local_jacobian_interior/_boundary (flow_spatial.cpp:818-875),
 * SteadyBackwardEulerSolver::addPseudoTimeTerm (aodesolver.cpp:300-329) and
 * MatrixFreeSpatialJacobian::apply (alinalg.cpp:142-233).
 *
 * Storage is face-based, which is what the reference's assembly produces block by block:
 *   lower[fi], upper[fi] (interior face fi = f - nbface, reference order): A[R][L] += L, A[L][R] += U;
 *   diag[c] (internal cell order): 0 + sum over the cell's faces in ascending reference face index
 *   of -left (boundary), -L (cell is left), -U (cell is right) — the order of the reference's
 *   ADD_VALUES calls in a single-thread run, so diagonal blocks are bitwise reproducible.
 * One thread per face computes its blocks column by column (gasjac.hpp), so no atomics are used.
 */
#include "jacobian.hpp"
#include "gasjac.hpp"

namespace fvhip {

using namespace gd;

// -------------------------------------------------------------------------------------------------
// interior faces
// -------------------------------------------------------------------------------------------------
// waves per SIMD the face-Jacobian kernels are compiled for: 2 (256 registers) where that costs at most a
// 12-byte spill; Roe with the viscous terms and constant-viscosity HLLC would spill 92-380 bytes per
// lane, so they keep the allocator's choice (up to 256 VGPRs + AGPRs, one wave)
#ifndef FVHIP_JAC_WAVES
#define FVHIP_JAC_WAVES 2
#endif
// FVHIP_JAC_SPLIT = 1: the viscous face kernels compute the inviscid columns into the LDS block first and add
// the viscous terms to them afterwards (jac_face_split), so the inviscid and the viscous working sets are
// never live together and the kernel fits two waves per SIMD: the C5 (Roe + Sutherland) face kernel 3.60-3.63
// -> 2.88-2.89 ms, bitwise the same blocks (profiles/r05/jac_split_ab.txt)
#ifndef FVHIP_JAC_SPLIT
#define FVHIP_JAC_SPLIT 1
#endif
template <int FLUX, int VISC>
constexpr int jacWaves() {
	return (FVHIP_JAC_SPLIT && VISC) ? 2
	     : (FLUX == 4 /* Roe */ && VISC) || (FLUX == 6 /* HLLC */ && VISC == 1) ? 1 : FVHIP_JAC_WAVES;
}
// FVHIP_JAC_LDS_STORE = 1: where the face-Jacobian kernel runs at <= 2 waves per SIMD anyway (Roe, HLLC
// and the viscous instantiations: 190-256 VGPRs), the face blocks go through LDS and leave as coalesced
// 16-byte rows (a block's 256 faces own one contiguous 64 KB range of lower and of upper), instead of 32
// scattered 8-byte stores per thread (one cache line per lane per store). The light ones (LLF, HLL,
// AUSM without viscous terms: 3-5 waves) keep the direct stores: 64 KB of LDS per block would cap them
// at 2 waves.
#ifndef FVHIP_JAC_LDS_STORE
#define FVHIP_JAC_LDS_STORE 1
#endif
template <int FLUX, int VISC>
constexpr bool jacLds() {
	return FVHIP_JAC_LDS_STORE && !((FLUX == 0 && VISC != 1) || (FLUX == 2 && VISC == 0) || (FLUX == 5 && VISC == 0));
}
constexpr int JAC_LDS_STRIDE = 257;   // entry-major rows of 256 faces, padded: 257 = 1 mod 32 double banks

/// face fi's two blocks, column by column: out(i, k, lower entry, upper entry)
template <int FLUX, int VISC, typename Out>
__device__ __forceinline__ void jac_face(const JacMesh& J, const gd::Gas& G, const double* __restrict__ u, int fi,
                                         Out&& out)
{
	const int2 lr = J.if_LR[fi];
	const double2 nn = J.if_n[fi];
	const double n[2] = {nn.x, nn.y};
	const double len = J.if_len[fi];
	double ul[4], ur[4];
	{
		const double4* u4 = reinterpret_cast<const double4*>(u);
		const double4 a = u4[lr.x], b = u4[lr.y];
		ul[0] = a.x; ul[1] = a.y; ul[2] = a.z; ul[3] = a.w;
		ur[0] = b.x; ur[1] = b.y; ur[2] = b.z; ur[3] = b.w;
	}
	typename JacOf<FLUX>::T F;
	jac_prepare<FLUX>(G, ul, ur, n, F);
	ViscJ V;
	if(VISC) {
		const double2 a = J.rc[lr.x], b = J.rc[lr.y];
		const double cl[2] = {a.x, a.y}, cr[2] = {b.x, b.y};
		visc_jac_prepare(G, VISC == 2, ul, ur, cl, cr, V);
	}
#pragma unroll
	for(int k = 0; k < 4; k++) {
		double dl[4], dr[4];
		jac_col<FLUX>(G, F, n, k, dl, dr);
		if(VISC) visc_jac_col(G, V, ul, ur, n, k, dl, dr);
		for(int i = 0; i < 4; i++) out(i, k, dl[i]*len, dr[i]*len);
	}
}

/// jac_face for the viscous kernels in two phases over the LDS block sb (entry-major rows, stride
/// JAC_LDS_STRIDE, this thread's face in column t): the inviscid columns go in unscaled, then each column is
/// read back, the viscous terms are added to it in visc_jac_col's order and the face length applied --
/// the same operations on the same values as jac_face, so the same bits
template <int FLUX, int VISC>
__device__ __forceinline__ void jac_face_split(const JacMesh& J, const gd::Gas& G, const double* __restrict__ u, int fi,
                                               double* sb, int t)
{
	const int2 lr = J.if_LR[fi];
	const double2 nn = J.if_n[fi];
	const double n[2] = {nn.x, nn.y};
	double ul[4], ur[4];
	{
		const double4* u4 = reinterpret_cast<const double4*>(u);
		const double4 a = u4[lr.x], b = u4[lr.y];
		ul[0] = a.x; ul[1] = a.y; ul[2] = a.z; ul[3] = a.w;
		ur[0] = b.x; ur[1] = b.y; ur[2] = b.z; ur[3] = b.w;
	}
	{
		typename JacOf<FLUX>::T F;
		jac_prepare<FLUX>(G, ul, ur, n, F);
#pragma unroll
		for(int k = 0; k < 4; k++) {
			double dl[4], dr[4];
			jac_col<FLUX>(G, F, n, k, dl, dr);
			for(int i = 0; i < 4; i++) { sb[(i*4+k)*JAC_LDS_STRIDE + t] = dl[i]; sb[(16+i*4+k)*JAC_LDS_STRIDE + t] = dr[i]; }
		}
	}
	__builtin_amdgcn_sched_barrier(0);          // keep the viscous working set out of the inviscid phase
	const double len = J.if_len[fi];
	ViscJ V;
	{
		const double2 a = J.rc[lr.x], b = J.rc[lr.y];
		const double cl[2] = {a.x, a.y}, cr[2] = {b.x, b.y};
		visc_jac_prepare(G, VISC == 2, ul, ur, cl, cr, V);
	}
#pragma unroll
	for(int k = 0; k < 4; k++) {
		double dl[4], dr[4];
		for(int i = 0; i < 4; i++) { dl[i] = sb[(i*4+k)*JAC_LDS_STRIDE + t]; dr[i] = sb[(16+i*4+k)*JAC_LDS_STRIDE + t]; }
		visc_jac_col(G, V, ul, ur, n, k, dl, dr);
		for(int i = 0; i < 4; i++) { sb[(i*4+k)*JAC_LDS_STRIDE + t] = dl[i]*len; sb[(16+i*4+k)*JAC_LDS_STRIDE + t] = dr[i]*len; }
	}
}

template <int FLUX, int VISC>
__global__ __launch_bounds__(256, (jacWaves<FLUX, VISC>()))
void k_jac_interior(JacMesh J, gd::Gas G, const double* __restrict__ u,
                    double* __restrict__ lower, double* __restrict__ upper)
{
	const int t = static_cast<int>(threadIdx.x);
	const int f0 = blockIdx.x*256;
	const int fi = f0 + t;
	if constexpr(jacLds<FLUX, VISC>()) {
		// sb[side*16 + entry][face in block]: the columns land entry-major (consecutive threads,
		// consecutive words: no bank conflicts); then each thread writes double2s of the block's range
		__shared__ double sb[32*JAC_LDS_STRIDE];
		if(fi < J.ninface) {
			if constexpr(FVHIP_JAC_SPLIT && VISC != 0) jac_face_split<FLUX, VISC>(J, G, u, fi, sb, t);
			else
				jac_face<FLUX, VISC>(J, G, u, fi, [&](int i, int k, double lo, double up) {
					sb[(i*4+k)*JAC_LDS_STRIDE + t] = lo;
					sb[(16+i*4+k)*JAC_LDS_STRIDE + t] = up;
				});
		}
		__syncthreads();
		const int nf = min(256, J.ninface - f0);
		double2* Lo2 = reinterpret_cast<double2*>(lower + 16*static_cast<size_t>(f0));
		double2* Up2 = reinterpret_cast<double2*>(upper + 16*static_cast<size_t>(f0));
		for(int j = t; j < 8*nf; j += 256) {
			const int f = j >> 3, e = (j & 7)*2;
			Lo2[j] = make_double2(sb[e*JAC_LDS_STRIDE + f], sb[(e+1)*JAC_LDS_STRIDE + f]);
			Up2[j] = make_double2(sb[(16+e)*JAC_LDS_STRIDE + f], sb[(17+e)*JAC_LDS_STRIDE + f]);
		}
	} else {
		if(fi >= J.ninface) return;
		double* Lo = lower + 16*static_cast<size_t>(fi);
		double* Up = upper + 16*static_cast<size_t>(fi);
		jac_face<FLUX, VISC>(J, G, u, fi, [&](int i, int k, double lo, double up) { Lo[i*4+k] = lo; Up[i*4+k] = up; });
	}
}

// -------------------------------------------------------------------------------------------------
// physical boundary faces: left = len*(dfdl - dfdr * d(ghost)/d(u_L))
// -------------------------------------------------------------------------------------------------
template <int FLUX, int VISC>
__global__ __launch_bounds__(64)
void k_jac_boundary(JacMesh J, DevPhys P, const double* __restrict__ u, double* __restrict__ bblk)
{
	const int f = blockIdx.x*blockDim.x + threadIdx.x;
	if(f >= J.nbface) return;
	const int c = J.bf_L[f];
	const double2 nn = J.bf_n[f];
	const double n[2] = {nn.x, nn.y};
	const double len = J.bf_len[f];
	double ul[4];
	for(int i = 0; i < 4; i++) ul[i] = u[4*static_cast<size_t>(c)+i];
	double gs[4], dgs[16];
	ghost_jacobian(P.gas, P.bc[J.bf_bc[f]], P.uinf, ul, n, gs, dgs);
	typename JacOf<FLUX>::T F;
	jac_prepare<FLUX>(P.gas, ul, gs, n, F);
	ViscJ V;
	if(VISC) {
		const double2 a = J.rc[c], b = J.bf_rcbp[f];
		const double cl[2] = {a.x, a.y}, cr[2] = {b.x, b.y};
		visc_jac_prepare(P.gas, VISC == 2, ul, gs, cl, cr, V);
	}
	double left[16], right[16];
#pragma unroll
	for(int k = 0; k < 4; k++) {
		double dl[4], dr[4];
		jac_col<FLUX>(P.gas, F, n, k, dl, dr);
		if(VISC) visc_jac_col(P.gas, V, ul, gs, n, k, dl, dr);
		for(int i = 0; i < 4; i++) { left[i*4+k] = dl[i]; right[i*4+k] = dr[i]; }
	}
	double* out = bblk + 16*static_cast<size_t>(f);
#pragma unroll
	for(int i = 0; i < 4; i++)
#pragma unroll
		for(int j = 0; j < 4; j++) {
			double s = right[i*4+0]*dgs[0*4+j];
			for(int k = 1; k < 4; k++) s += right[i*4+k]*dgs[k*4+j];
			out[i*4+j] = len*(left[i*4+j] - s);
		}
}

// -------------------------------------------------------------------------------------------------
// diagonal blocks: per cell, ascending reference face order
// -------------------------------------------------------------------------------------------------
__device__ __attribute__((aligned(32))) const double kZeroBlock[16] = {};
__global__ __launch_bounds__(256)
void k_jac_diag(JacMesh J, const double* __restrict__ bblk, const double* __restrict__ lower,
                const double* __restrict__ upper, double* __restrict__ diag, const double* __restrict__ area,
                double cfl, double* __restrict__ dtm)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= J.ncell) return;
	const int4 fc = J.cell_rfaces[c];
	const int codes[4] = {fc.x, fc.y, fc.z, fc.w};
	double d[16];
#pragma unroll
	for(int k = 0; k < 16; k++) d[k] = 0;
	// all four blocks requested before any sum (0.547 -> 0.483 ms on C4 against a branch per face,
	// profiles/r03/ab/jacdiag_*); a missing face reads a zero block, whose terms d + (-1*0) = d + (-0) = d
	// change nothing (bitwise, signed zeros included)
	double4 v[4][4];
#pragma unroll
	for(int j = 0; j < 4; j++) {
		const int code = codes[j];
		const int f = code >> 1;
		const double* blk = code < 0 ? kZeroBlock
		                  : f < J.nbface ? bblk + 16*static_cast<size_t>(f)
		                  : ((code & 1) ? upper : lower) + 16*static_cast<size_t>(f - J.nbface);
		const double4* b4 = reinterpret_cast<const double4*>(blk);
#pragma unroll
		for(int q = 0; q < 4; q++) v[j][q] = b4[q];
	}
#pragma unroll
	for(int j = 0; j < 4; j++)
#pragma unroll
		for(int q = 0; q < 4; q++) {
			d[4*q+0] += -1.0*v[j][q].x; d[4*q+1] += -1.0*v[j][q].y; d[4*q+2] += -1.0*v[j][q].z; d[4*q+3] += -1.0*v[j][q].w;
		}
	if(area) {
		// the pseudo-time term of k_pseudo_time, same operations, while the block is in registers
		const double m = area[c] / (cfl*dtm[c]);
		dtm[c] = m;
#pragma unroll
		for(int i = 0; i < 4; i++)
#pragma unroll
			for(int k = 0; k < 4; k++) d[i*4+k] += m*(i == k ? 1.0 : 0.0);
	}
	double4* o = reinterpret_cast<double4*>(diag + 16*static_cast<size_t>(c));
#pragma unroll
	for(int q = 0; q < 4; q++) o[q] = make_double4(d[4*q], d[4*q+1], d[4*q+2], d[4*q+3]);
}

#ifndef FVHIP_BLOCK_ROWS
#define FVHIP_BLOCK_ROWS 1
#endif
/// k_jac_diag with four lanes per cell, lane i forming row i of the block: each face block is read as four
/// consecutive 32-byte rows by four consecutive lanes (one 128-byte segment per block instead of one per
/// lane and 16-byte piece), and the diagonal block is written the same way. Every entry takes the same
/// operations in the same order as k_jac_diag's (its terms over the faces in ascending order, then the
/// pseudo-time term), so the blocks are bitwise the same.
__global__ __launch_bounds__(256)
void k_jac_diag_rows(JacMesh J, const double* __restrict__ bblk, const double* __restrict__ lower,
                     const double* __restrict__ upper, double* __restrict__ diag, const double* __restrict__ area,
                     double cfl, double* __restrict__ dtm)
{
	const long long g = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	const int c = static_cast<int>(g >> 2), i = static_cast<int>(g & 3);
	if(c >= J.ncell) return;
	const int4 fc = J.cell_rfaces[c];
	const int codes[4] = {fc.x, fc.y, fc.z, fc.w};
	double4 v[4];
#pragma unroll
	for(int j = 0; j < 4; j++) {
		const int code = codes[j];
		const int f = code >> 1;
		const double* blk = code < 0 ? kZeroBlock
		                  : f < J.nbface ? bblk + 16*static_cast<size_t>(f)
		                  : ((code & 1) ? upper : lower) + 16*static_cast<size_t>(f - J.nbface);
		v[j] = reinterpret_cast<const double4*>(blk)[i];
	}
	double d[4] = {0, 0, 0, 0};
#pragma unroll
	for(int j = 0; j < 4; j++) {
		d[0] += -1.0*v[j].x; d[1] += -1.0*v[j].y; d[2] += -1.0*v[j].z; d[3] += -1.0*v[j].w;
	}
	if(area) {
		const double m = area[c] / (cfl*dtm[c]);
#pragma unroll
		for(int k = 0; k < 4; k++) d[k] += m*(i == k ? 1.0 : 0.0);
		if(i == 0) dtm[c] = m;            // after all four lanes of the cell (one wavefront) have read it
	}
	reinterpret_cast<double4*>(diag + 16*static_cast<size_t>(c))[i] = make_double4(d[0], d[1], d[2], d[3]);
}

// -------------------------------------------------------------------------------------------------
// pseudo-time term: dtm <- area/(cfl*dtm); diag += dtm*I (all 16 entries, as MatSetValuesBlocked)
// -------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256)
void k_pseudo_time(int ncell, const double* __restrict__ area, double cfl, double* __restrict__ dtm,
                   double* __restrict__ diag)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= ncell) return;
	const double m = area[c] / (cfl*dtm[c]);
	dtm[c] = m;
	double* d = diag + 16*static_cast<size_t>(c);
#pragma unroll
	for(int i = 0; i < 4; i++)
#pragma unroll
		for(int j = 0; j < 4; j++) d[i*4+j] += m*(i == j ? 1.0 : 0.0);
}

// -------------------------------------------------------------------------------------------------
// y = A x with the face-based blocks; per cell: diag first, then faces in ascending reference order
// -------------------------------------------------------------------------------------------------
/// s[i] = sum_k B[i][k] x[k] for a row-major 4x4 block, rows read as double4 (k ascending)
__device__ __forceinline__ void blk_row_dots(const double* __restrict__ B, const double4 x, double (&s)[4])
{
	const double4* b4 = reinterpret_cast<const double4*>(B);
#pragma unroll
	for(int i = 0; i < 4; i++) {
		const double4 r = b4[i];
		s[i] = r.x*x.x + r.y*x.y + r.z*x.z + r.w*x.w;
	}
}
/// the same for an fp32 block (entries widened to fp64, fp64 arithmetic)
__device__ __forceinline__ void blk_row_dots(const float* __restrict__ B, const double4 x, double (&s)[4])
{
	const float4* b4 = reinterpret_cast<const float4*>(B);
#pragma unroll
	for(int i = 0; i < 4; i++) {
		const float4 r = b4[i];
		s[i] = static_cast<double>(r.x)*x.x + static_cast<double>(r.y)*x.y + static_cast<double>(r.z)*x.z
		     + static_cast<double>(r.w)*x.w;
	}
}

__global__ __launch_bounds__(256)
void k_block_apply(JacMesh J, const double* __restrict__ diag, const double* __restrict__ lower,
                   const double* __restrict__ upper, const double* __restrict__ x, double* __restrict__ y)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= J.ncell) return;
	const double4* x4 = reinterpret_cast<const double4*>(x);
	double acc[4];
	blk_row_dots(diag + 16*static_cast<size_t>(c), x4[c], acc);
	const int4 fc = J.cell_rfaces[c];
	const int4 nb = J.cell_nbr_fo[c];
	const int codes[4] = {fc.x, fc.y, fc.z, fc.w};
	const int nbrs[4] = {nb.x, nb.y, nb.z, nb.w};
#pragma unroll
	for(int j = 0; j < 4; j++) {
		const int code = codes[j];
		if(code < 0) continue;
		const int f = code >> 1;
		if(f < J.nbface) continue;
		const double* B = ((code & 1) ? lower : upper) + 16*static_cast<size_t>(f - J.nbface);
		double s[4];
		blk_row_dots(B, x4[nbrs[j]], s);
#pragma unroll
		for(int i = 0; i < 4; i++) acc[i] += s[i];
	}
	reinterpret_cast<double4*>(y)[c] = make_double4(acc[0], acc[1], acc[2], acc[3]);
}

/// k_block_apply with four lanes per cell, lane i forming y[c][i]: the same row dot products in the same
/// order (diagonal block first, then the faces ascending), so bitwise the same y; each block is read as four
/// consecutive 32-byte rows by four consecutive lanes, and y is written as one 32-byte row per cell
__global__ __launch_bounds__(256)
void k_block_apply_rows(JacMesh J, const double* __restrict__ diag, const double* __restrict__ lower,
                        const double* __restrict__ upper, const double* __restrict__ x, double* __restrict__ y)
{
	const long long g = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	const int c = static_cast<int>(g >> 2), i = static_cast<int>(g & 3);
	if(c >= J.ncell) return;
	const double4* x4 = reinterpret_cast<const double4*>(x);
	const int4 fc = J.cell_rfaces[c];
	const int4 nb = J.cell_nbr_fo[c];
	const int codes[4] = {fc.x, fc.y, fc.z, fc.w};
	const int nbrs[4] = {nb.x, nb.y, nb.z, nb.w};
	double4 r = reinterpret_cast<const double4*>(diag + 16*static_cast<size_t>(c))[i];
	double4 xv = x4[c];
	double acc = r.x*xv.x + r.y*xv.y + r.z*xv.z + r.w*xv.w;
#pragma unroll
	for(int j = 0; j < 4; j++) {
		const int code = codes[j];
		if(code < 0) continue;
		const int f = code >> 1;
		if(f < J.nbface) continue;
		const double* B = ((code & 1) ? lower : upper) + 16*static_cast<size_t>(f - J.nbface);
		r = reinterpret_cast<const double4*>(B)[i];
		xv = x4[nbrs[j]];
		acc += r.x*xv.x + r.y*xv.y + r.z*xv.z + r.w*xv.w;
	}
	y[4*static_cast<size_t>(c) + i] = acc;
}

/// One block-Jacobi sweep fused into one pass: zout = D^-1 (v - sum_faces B zin[nbr]), the
/// off-diagonal half of k_block_apply followed by the diagonal solve (zin needs its ghost rows).
/// Same iterate as zin + D^-1 (v - A zin) up to rounding, without reading D or writing A zin.
template <typename T>
__global__ __launch_bounds__(256)
void k_bjac_sweep(JacMesh J, const T* __restrict__ dinv, const T* __restrict__ lower,
                  const T* __restrict__ upper, const double* __restrict__ v, const double* __restrict__ zin,
                  double* __restrict__ zout)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= J.ncell) return;
	const double4* z4 = reinterpret_cast<const double4*>(zin);
	const double4 vc = reinterpret_cast<const double4*>(v)[c];
	double acc[4] = {vc.x, vc.y, vc.z, vc.w};
	const int4 fc = J.cell_rfaces[c];
	const int4 nb = J.cell_nbr_fo[c];
	const int codes[4] = {fc.x, fc.y, fc.z, fc.w};
	const int nbrs[4] = {nb.x, nb.y, nb.z, nb.w};
#pragma unroll
	for(int j = 0; j < 4; j++) {
		const int code = codes[j];
		if(code < 0) continue;
		const int f = code >> 1;
		if(f < J.nbface) continue;
		const T* B = ((code & 1) ? lower : upper) + 16*static_cast<size_t>(f - J.nbface);
		double s[4];
		blk_row_dots(B, z4[nbrs[j]], s);
#pragma unroll
		for(int i = 0; i < 4; i++) acc[i] -= s[i];
	}
	double o[4];
	blk_row_dots(dinv + 16*static_cast<size_t>(c), make_double4(acc[0], acc[1], acc[2], acc[3]), o);
	reinterpret_cast<double4*>(zout)[c] = make_double4(o[0], o[1], o[2], o[3]);
}

/// row i of a row-major 4x4 block dotted with x, as blk_row_dots forms it (k ascending)
__device__ __forceinline__ double blk_row_dot(const double* __restrict__ B, int i, const double4 x)
{
	const double4 r = reinterpret_cast<const double4*>(B)[i];
	return r.x*x.x + r.y*x.y + r.z*x.z + r.w*x.w;
}
__device__ __forceinline__ double blk_row_dot(const float* __restrict__ B, int i, const double4 x)
{
	const float4 r = reinterpret_cast<const float4*>(B)[i];
	return static_cast<double>(r.x)*x.x + static_cast<double>(r.y)*x.y + static_cast<double>(r.z)*x.z
	     + static_cast<double>(r.w)*x.w;
}
/// t = v - A x in one pass (the multigrid's finest residuals): k_block_apply_rows' row sum, subtracted from v;
/// T = float: the blocks stored in fp32 (prec_single: the preconditioner's copy), the arithmetic in fp64
template <typename T>
__global__ __launch_bounds__(256)
void k_block_residual_rows(JacMesh J, const T* __restrict__ diag, const T* __restrict__ lower,
                           const T* __restrict__ upper, const double* __restrict__ x, const double* __restrict__ v,
                           double* __restrict__ t)
{
	const long long g = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	const int c = static_cast<int>(g >> 2), i = static_cast<int>(g & 3);
	if(c >= J.ncell) return;
	const double4* x4 = reinterpret_cast<const double4*>(x);
	const int4 fc = J.cell_rfaces[c];
	const int4 nb = J.cell_nbr_fo[c];
	const int codes[4] = {fc.x, fc.y, fc.z, fc.w};
	const int nbrs[4] = {nb.x, nb.y, nb.z, nb.w};
	double acc = blk_row_dot(diag + 16*static_cast<size_t>(c), i, x4[c]);
#pragma unroll
	for(int j = 0; j < 4; j++) {
		const int code = codes[j];
		if(code < 0) continue;
		const int f = code >> 1;
		if(f < J.nbface) continue;
		const T* B = ((code & 1) ? lower : upper) + 16*static_cast<size_t>(f - J.nbface);
		acc += blk_row_dot(B, i, x4[nbrs[j]]);
	}
	t[4*static_cast<size_t>(c) + i] = v[4*static_cast<size_t>(c) + i] - acc;
}

/// k_bjac_sweep with four lanes per cell, lane i forming row i (coalesced block rows, as k_block_apply_rows):
/// the same row sums in the same order, the four sums exchanged within the cell's lanes for the product
/// with D^-1, so bitwise k_bjac_sweep's z
template <typename T>
__global__ __launch_bounds__(256)
void k_bjac_sweep_rows(JacMesh J, const T* __restrict__ dinv, const T* __restrict__ lower,
                       const T* __restrict__ upper, const double* __restrict__ v, const double* __restrict__ zin,
                       double* __restrict__ zout)
{
	const long long g = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	const int c = static_cast<int>(g >> 2), i = static_cast<int>(g & 3);
	const bool live = c < J.ncell;
	const int cc = live ? c : J.ncell - 1;          // lanes past the end compute a copy and store nothing
	const double4* z4 = reinterpret_cast<const double4*>(zin);
	double acc = v[4*static_cast<size_t>(cc) + i];
	const int4 fc = J.cell_rfaces[cc];
	const int4 nb = J.cell_nbr_fo[cc];
	const int codes[4] = {fc.x, fc.y, fc.z, fc.w};
	const int nbrs[4] = {nb.x, nb.y, nb.z, nb.w};
#pragma unroll
	for(int j = 0; j < 4; j++) {
		const int code = codes[j];
		if(code < 0) continue;
		const int f = code >> 1;
		if(f < J.nbface) continue;
		const T* B = ((code & 1) ? lower : upper) + 16*static_cast<size_t>(f - J.nbface);
		acc -= blk_row_dot(B, i, z4[nbrs[j]]);
	}
	// the cell's four row sums to every lane of the cell (all 64 lanes of the wave take part)
	const double4 t = make_double4(__shfl(acc, 0, 4), __shfl(acc, 1, 4), __shfl(acc, 2, 4), __shfl(acc, 3, 4));
	const double o = blk_row_dot(dinv + 16*static_cast<size_t>(cc), i, t);
	if(live) zout[4*static_cast<size_t>(c) + i] = o;
}

/// One colour of a multicolour block Gauss-Seidel sweep, in place: z_c = D^-1 (v - sum_faces B z[nbr])
/// for the listed cells, which share no face, so every neighbour value read is either from an
/// earlier colour of this sweep or from the previous sweep (ghost rows: from the last exchange).
template <typename T>
__global__ __launch_bounds__(256)
void k_bgs_colour(JacMesh J, const T* __restrict__ dinv, const T* __restrict__ lower, const T* __restrict__ upper,
                  const double* __restrict__ v, double* z, const int* __restrict__ cells, int n)
{
	const int i = blockIdx.x*blockDim.x + threadIdx.x;
	if(i >= n) return;
	const int c = cells[i];
	const double4* z4 = reinterpret_cast<const double4*>(z);
	const double4 vc = reinterpret_cast<const double4*>(v)[c];
	double acc[4] = {vc.x, vc.y, vc.z, vc.w};
	const int4 fc = J.cell_rfaces[c];
	const int4 nb = J.cell_nbr_fo[c];
	const int codes[4] = {fc.x, fc.y, fc.z, fc.w};
	const int nbrs[4] = {nb.x, nb.y, nb.z, nb.w};
#pragma unroll
	for(int j = 0; j < 4; j++) {
		const int code = codes[j];
		if(code < 0) continue;
		const int f = code >> 1;
		if(f < J.nbface) continue;
		const T* B = ((code & 1) ? lower : upper) + 16*static_cast<size_t>(f - J.nbface);
		double s[4];
		blk_row_dots(B, z4[nbrs[j]], s);
#pragma unroll
		for(int k = 0; k < 4; k++) acc[k] -= s[k];
	}
	double o[4];
	blk_row_dots(dinv + 16*static_cast<size_t>(c), make_double4(acc[0], acc[1], acc[2], acc[3]), o);
	reinterpret_cast<double4*>(z)[c] = make_double4(o[0], o[1], o[2], o[3]);
}

/// k_bgs_colour with four lanes per cell (k_bjac_sweep_rows' arithmetic, in place): bitwise k_bgs_colour's z.
/// Every lane of the cell reads its neighbours' rows before any lane writes the cell (cells of a colour
/// share no face, so no neighbour is written by this launch)
template <typename T>
__global__ __launch_bounds__(256)
void k_bgs_colour_rows(JacMesh J, const T* __restrict__ dinv, const T* __restrict__ lower, const T* __restrict__ upper,
                       const double* __restrict__ v, double* z, const int* __restrict__ cells, int n)
{
	const long long g = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	const int k = static_cast<int>(g >> 2), i = static_cast<int>(g & 3);
	const bool live = k < n;
	const int c = cells[live ? k : n - 1];
	const double4* z4 = reinterpret_cast<const double4*>(z);
	double acc = v[4*static_cast<size_t>(c) + i];
	const int4 fc = J.cell_rfaces[c];
	const int4 nb = J.cell_nbr_fo[c];
	const int codes[4] = {fc.x, fc.y, fc.z, fc.w};
	const int nbrs[4] = {nb.x, nb.y, nb.z, nb.w};
#pragma unroll
	for(int j = 0; j < 4; j++) {
		const int code = codes[j];
		if(code < 0) continue;
		const int f = code >> 1;
		if(f < J.nbface) continue;
		const T* B = ((code & 1) ? lower : upper) + 16*static_cast<size_t>(f - J.nbface);
		acc -= blk_row_dot(B, i, z4[nbrs[j]]);
	}
	const double4 t = make_double4(__shfl(acc, 0, 4), __shfl(acc, 1, 4), __shfl(acc, 2, 4), __shfl(acc, 3, 4));
	const double o = blk_row_dot(dinv + 16*static_cast<size_t>(c), i, t);
	if(live) z[4*static_cast<size_t>(c) + i] = o;
}

// -------------------------------------------------------------------------------------------------
// matrix-free pieces
// -------------------------------------------------------------------------------------------------
constexpr int RED_BLOCKS = 1024;

/// deterministic two-stage sum of squares: fixed partition, fixed tree
__global__ __launch_bounds__(256)
void k_sumsq_partial(long long n, const double* __restrict__ x, double* __restrict__ part)
{
	__shared__ double s[256];
	double acc = 0;
	for(long long i = blockIdx.x*256LL + threadIdx.x; i < n; i += 256LL*gridDim.x) acc += x[i]*x[i];
	s[threadIdx.x] = acc;
	__syncthreads();
	for(int w = 128; w > 0; w >>= 1) {
		if(threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
		__syncthreads();
	}
	if(threadIdx.x == 0) part[blockIdx.x] = s[0];
}

/// pertmag = eps / sqrt(sum(part))
__global__ __launch_bounds__(256)
void k_pertmag(int np, const double* __restrict__ part, double eps, double* __restrict__ out)
{
	__shared__ double s[256];
	double acc = 0;
	for(int i = threadIdx.x; i < np; i += 256) acc += part[i];
	s[threadIdx.x] = acc;
	__syncthreads();
	for(int w = 128; w > 0; w >>= 1) {
		if(threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
		__syncthreads();
	}
	if(threadIdx.x == 0) { out[0] = sqrt(s[0]); out[1] = eps/out[0]; }
}

__global__ __launch_bounds__(256)
void k_mf_perturb(long long n, const double* __restrict__ u, const double* __restrict__ x,
                  const double* __restrict__ pm, double* __restrict__ aux)
{
	const long long i = blockIdx.x*256LL + threadIdx.x;
	if(i >= n) return;
	aux[i] = u[i] + pm[1]*x[i];
}

__global__ __launch_bounds__(256)
void k_mf_combine(int ncell, const double* __restrict__ mdt, const double* __restrict__ x,
                  const double* __restrict__ yg, const double* __restrict__ res,
                  const double* __restrict__ pm, double* __restrict__ y)
{
	const int c = blockIdx.x*256 + threadIdx.x;
	if(c >= ncell) return;
	const double pert = pm[1], d = mdt[c];
	// one 32-byte row per vector and cell; each entry mdt x + (-yg + res)/pert as before
	const double4 xv = reinterpret_cast<const double4*>(x)[c], gv = reinterpret_cast<const double4*>(yg)[c];
	const double4 rv = reinterpret_cast<const double4*>(res)[c];
	reinterpret_cast<double4*>(y)[c] = make_double4(d*xv.x + (-gv.x + rv.x)/pert, d*xv.y + (-gv.y + rv.y)/pert,
	                                                d*xv.z + (-gv.z + rv.z)/pert, d*xv.w + (-gv.w + rv.w)/pert);
}

// pointwise flux Jacobians (InviscidFlux::get_jacobian)
template <int FLUX>
__global__ __launch_bounds__(256)
void k_local_jac(gd::Gas G, int nf, const double* __restrict__ ul, const double* __restrict__ ur,
                 const double* __restrict__ nrm, double* __restrict__ dfdl, double* __restrict__ dfdr)
{
	const int f = blockIdx.x*blockDim.x + threadIdx.x;
	if(f >= nf) return;
	double a[4], b[4], n[2] = {nrm[2*f], nrm[2*f+1]};
	for(int i = 0; i < 4; i++) { a[i] = ul[4*f+i]; b[i] = ur[4*f+i]; }
	typename JacOf<FLUX>::T F;
	jac_prepare<FLUX>(G, a, b, n, F);
#pragma unroll
	for(int k = 0; k < 4; k++) {
		double dl[4], dr[4];
		jac_col<FLUX>(G, F, n, k, dl, dr);
		for(int i = 0; i < 4; i++) { dfdl[16*f+i*4+k] = dl[i]; dfdr[16*f+i*4+k] = dr[i]; }
	}
}

// -------------------------------------------------------------------------------------------------
// launchers
// -------------------------------------------------------------------------------------------------
static inline int nblk(long long n, int b) { return static_cast<int>((n + b - 1)/b); }

template <int FLUX, int VISC>
static void jac_launch(const JacMesh& J, const DevPhys& P, const double* u, double* bblk, double* lower,
                       double* upper, hipStream_t s)
{
	if(J.ninface > 0)
		hipLaunchKernelGGL((k_jac_interior<FLUX,VISC>), dim3(nblk(J.ninface,256)), dim3(256), 0, s, J, P.gas, u, lower, upper);
	if(J.nbface > 0)
		hipLaunchKernelGGL((k_jac_boundary<FLUX,VISC>), dim3(nblk(J.nbface,64)), dim3(64), 0, s, J, P, u, bblk);
}

template <int FLUX>
static void jac_launch_v(const JacMesh& J, const DevPhys& P, int visc, const double* u, double* bblk,
                         double* lower, double* upper, hipStream_t s)
{
	switch(visc) {
		case 0: jac_launch<FLUX,0>(J, P, u, bblk, lower, upper, s); break;
		case 1: jac_launch<FLUX,1>(J, P, u, bblk, lower, upper, s); break;
		default: jac_launch<FLUX,2>(J, P, u, bblk, lower, upper, s);
	}
}

void launch_jac_faces(const JacMesh& J, const DevPhys& P, int jflux, int visc, const double* u, double* bblk,
                      double* lower, double* upper, hipStream_t s)
{
	switch(jflux) {
		case 0: jac_launch_v<0>(J, P, visc, u, bblk, lower, upper, s); break;
		case 2: jac_launch_v<2>(J, P, visc, u, bblk, lower, upper, s); break;
		case 4: jac_launch_v<4>(J, P, visc, u, bblk, lower, upper, s); break;
		case 5: jac_launch_v<5>(J, P, visc, u, bblk, lower, upper, s); break;
		case 6: jac_launch_v<6>(J, P, visc, u, bblk, lower, upper, s); break;
		default: break;
	}
}

void launch_jac_diag(const JacMesh& J, const double* bblk, const double* lower, const double* upper,
                     double* diag, hipStream_t s, const double* area, double cfl, double* dtm)
{
	if(J.ncell <= 0) return;
	if(FVHIP_BLOCK_ROWS)
		hipLaunchKernelGGL(k_jac_diag_rows, dim3(nblk(4LL*J.ncell,256)), dim3(256), 0, s, J, bblk, lower, upper, diag, area, cfl, dtm);
	else
		hipLaunchKernelGGL(k_jac_diag, dim3(nblk(J.ncell,256)), dim3(256), 0, s, J, bblk, lower, upper, diag, area, cfl, dtm);
}

void launch_pseudo_time(int ncell, const double* area, double cfl, double* dtm, double* diag, hipStream_t s)
{
	hipLaunchKernelGGL(k_pseudo_time, dim3(nblk(ncell,256)), dim3(256), 0, s, ncell, area, cfl, dtm, diag);
}

void launch_block_apply(const JacMesh& J, const double* diag, const double* lower, const double* upper,
                        const double* x, double* y, hipStream_t s)
{
	if(J.ncell <= 0) return;
	if(FVHIP_BLOCK_ROWS)
		hipLaunchKernelGGL(k_block_apply_rows, dim3(nblk(4LL*J.ncell,256)), dim3(256), 0, s, J, diag, lower, upper, x, y);
	else
		hipLaunchKernelGGL(k_block_apply, dim3(nblk(J.ncell,256)), dim3(256), 0, s, J, diag, lower, upper, x, y);
}

void launch_block_residual(const JacMesh& J, const double* diag, const double* lower, const double* upper,
                           const double* x, const double* v, double* t, hipStream_t s)
{
	if(J.ncell <= 0) return;
	hipLaunchKernelGGL(k_block_residual_rows<double>, dim3(nblk(4LL*J.ncell,256)), dim3(256), 0, s, J, diag, lower, upper, x, v, t);
}

void launch_block_residual(const JacMesh& J, const float* diag, const float* lower, const float* upper,
                           const double* x, const double* v, double* t, hipStream_t s)
{
	if(J.ncell <= 0) return;
	hipLaunchKernelGGL(k_block_residual_rows<float>, dim3(nblk(4LL*J.ncell,256)), dim3(256), 0, s, J, diag, lower, upper, x, v, t);
}

void launch_bjac_sweep(const JacMesh& J, const double* dinv, const double* lower, const double* upper,
                       const double* v, const double* zin, double* zout, hipStream_t s)
{
	if(J.ncell <= 0) return;
	if(FVHIP_BLOCK_ROWS)
		hipLaunchKernelGGL(k_bjac_sweep_rows<double>, dim3(nblk(4LL*J.ncell,256)), dim3(256), 0, s, J, dinv, lower, upper, v, zin, zout);
	else
		hipLaunchKernelGGL(k_bjac_sweep<double>, dim3(nblk(J.ncell,256)), dim3(256), 0, s, J, dinv, lower, upper, v, zin, zout);
}
void launch_bjac_sweep(const JacMesh& J, const float* dinv, const float* lower, const float* upper,
                       const double* v, const double* zin, double* zout, hipStream_t s)
{
	if(J.ncell <= 0) return;
	if(FVHIP_BLOCK_ROWS)
		hipLaunchKernelGGL(k_bjac_sweep_rows<float>, dim3(nblk(4LL*J.ncell,256)), dim3(256), 0, s, J, dinv, lower, upper, v, zin, zout);
	else
		hipLaunchKernelGGL(k_bjac_sweep<float>, dim3(nblk(J.ncell,256)), dim3(256), 0, s, J, dinv, lower, upper, v, zin, zout);
}

template <typename T>
void launch_bgs_colour_t(const JacMesh& J, const T* dinv, const T* lower, const T* upper, const double* v,
                         double* z, const int* cells, int n, hipStream_t s)
{
	if(n <= 0) return;
	if(FVHIP_BLOCK_ROWS)
		hipLaunchKernelGGL(k_bgs_colour_rows<T>, dim3(nblk(4LL*n,256)), dim3(256), 0, s, J, dinv, lower, upper, v, z, cells, n);
	else
		hipLaunchKernelGGL(k_bgs_colour<T>, dim3(nblk(n,256)), dim3(256), 0, s, J, dinv, lower, upper, v, z, cells, n);
}
void launch_bgs_colour(const JacMesh& J, const double* dinv, const double* lower, const double* upper,
                       const double* v, double* z, const int* cells, int n, hipStream_t s)
{ launch_bgs_colour_t(J, dinv, lower, upper, v, z, cells, n, s); }
void launch_bgs_colour(const JacMesh& J, const float* dinv, const float* lower, const float* upper,
                       const double* v, double* z, const int* cells, int n, hipStream_t s)
{ launch_bgs_colour_t(J, dinv, lower, upper, v, z, cells, n, s); }

void launch_mf_norm(long long n, const double* x, double eps, double* part, double* pm, hipStream_t s)
{
	hipLaunchKernelGGL(k_sumsq_partial, dim3(RED_BLOCKS), dim3(256), 0, s, n, x, part);
	hipLaunchKernelGGL(k_pertmag, dim3(1), dim3(256), 0, s, RED_BLOCKS, part, eps, pm);
}

void launch_mf_perturb(long long n, const double* u, const double* x, const double* pm, double* aux, hipStream_t s)
{
	hipLaunchKernelGGL(k_mf_perturb, dim3(nblk(n,256)), dim3(256), 0, s, n, u, x, pm, aux);
}

void launch_mf_combine(int ncell, const double* mdt, const double* x, const double* yg, const double* res,
                       const double* pm, double* y, hipStream_t s)
{
	hipLaunchKernelGGL(k_mf_combine, dim3(nblk(ncell,256)), dim3(256), 0, s, ncell, mdt, x, yg, res, pm, y);
}

int mf_partials() { return RED_BLOCKS; }

void launch_local_jac(int flux, const gd::Gas& G, int nf, const double* ul, const double* ur, const double* n,
                      double* dfdl, double* dfdr, hipStream_t s)
{
	const dim3 g(nblk(nf,256)), b(256);
	switch(flux) {
		case 0: hipLaunchKernelGGL(k_local_jac<0>, g, b, 0, s, G, nf, ul, ur, n, dfdl, dfdr); break;
		case 2: hipLaunchKernelGGL(k_local_jac<2>, g, b, 0, s, G, nf, ul, ur, n, dfdl, dfdr); break;
		case 4: hipLaunchKernelGGL(k_local_jac<4>, g, b, 0, s, G, nf, ul, ur, n, dfdl, dfdr); break;
		case 5: hipLaunchKernelGGL(k_local_jac<5>, g, b, 0, s, G, nf, ul, ur, n, dfdl, dfdr); break;
		case 6: hipLaunchKernelGGL(k_local_jac<6>, g, b, 0, s, G, nf, ul, ur, n, dfdl, dfdr); break;
		default: break;
	}
}

}
