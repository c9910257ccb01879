/** \file krylov.hip
 * \brief Device linear algebra of the implicit pseudo-time solver (declarations and sources in
 *   krylov.hpp). One thread per cell for the 4x4 block kernels (128 B of blocks and 64 B of
 *   vectors per cell, HBM-bound); the multi-dot reads w once per group of KRY_GROUP basis vectors
 *   and reduces with a fixed grid and a fixed tree, so every GMRES coefficient is reproducible.
 */
#include "krylov.hpp"
#include "blk4.hpp"

namespace fvhip {

constexpr int KRY_BLOCKS = 512;   ///< partial sums of the energy norm (= ode.hip's ODE_RED_BLOCKS)
constexpr int KRY_DOT_BLOCKS = 2048;   ///< partial sums per GMRES dot product (8 blocks per CU: enough loads in flight)
constexpr int KRY_GROUP = 8;      ///< dot products per block row of the multi-dot (w read once per 8 basis vectors)

static inline int nblk(long long n, int b) { return static_cast<int>((n + b - 1)/b); }

/// fixed-tree sum over the block of NV values per thread; thread 0 writes out[q*stride]
template <int NV>
__device__ __forceinline__ void block_sum(double (&acc)[NV], double* out, int stride)
{
	__shared__ double s[NV][256];
	const int t = static_cast<int>(threadIdx.x);
	#pragma unroll
	for(int q = 0; q < NV; q++) s[q][t] = acc[q];
	__syncthreads();
	for(int w = 128; w > 0; w >>= 1) {
		if(t < w) {
			#pragma unroll
			for(int q = 0; q < NV; q++) s[q][t] += s[q][t + w];
		}
		__syncthreads();
	}
	if(t == 0) {
		#pragma unroll
		for(int q = 0; q < NV; q++) out[q*stride] = s[q][0];
	}
}

__global__ __launch_bounds__(256)
void k_bjac_invert(int n, const double* __restrict__ diag, double* __restrict__ dinv)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= n) return;
	double a[4][4], b[4][4];
	ld16(diag + 16*static_cast<size_t>(c), a);
	inv4(a, b);
	st16(dinv + 16*static_cast<size_t>(c), b);
}

/// Block ILU(0) of the operator in multicolour order (prec_ilu), the factorisation of colour q: for each
/// listed cell i
///     Dt_i = A_ii - sum_{k ~ i, colour(k) < q} A_ik Dt_k^-1 A_ki,     dinv_i = Dt_i^-1
/// over the owned neighbours across interior faces (ghost couplings are dropped: block-Jacobi across
/// ranks, as PETSc's bjacobi + ilu). The product of row i's lower factor with a neighbour's upper
/// factor lands only on the diagonal unless three cells pairwise share faces, so this D-ILU form is
/// ILU(0) itself on meshes without such triples (fvhip_colouring reports their count). Face blocks:
/// lower[fi] = A[R][L], upper[fi] = A[L][R]; rfaces code = face << 1 | cell-is-R.
__global__ __launch_bounds__(256)
void k_ilu_factor_colour(int ncell, int nbface, const int4* __restrict__ rfaces, const int4* __restrict__ nbrs,
                         const int* __restrict__ colour, int q, const double* __restrict__ diag,
                         const double* __restrict__ lower, const double* __restrict__ upper, double* dinv,
                         const int* __restrict__ cells, int n)
{
	const int t = blockIdx.x*blockDim.x + threadIdx.x;
	if(t >= n) return;
	const int c = cells[t];
	double a[4][4];
	ld16(diag + 16*static_cast<size_t>(c), a);
	const int4 fc = rfaces[c], nb = nbrs[c];
	const int codes[4] = {fc.x, fc.y, fc.z, fc.w};
	const int ks[4] = {nb.x, nb.y, nb.z, nb.w};
	for(int j = 0; j < 4; j++) {
		const int code = codes[j], k = ks[j];
		if(code < 0 || (code >> 1) < nbface || k < 0 || k >= ncell || colour[k] >= q) continue;
		const size_t fi = static_cast<size_t>((code >> 1) - nbface);
		double aik[4][4], aki[4][4], dk[4][4], tk[4][4], p[4][4];
		ld16(((code & 1) ? lower : upper) + 16*fi, aik);
		ld16(((code & 1) ? upper : lower) + 16*fi, aki);
		ld16(dinv + 16*static_cast<size_t>(k), dk);
		mm4(dk, aki, tk);
		mm4(aik, tk, p);
		#pragma unroll
		for(int r = 0; r < 4; r++)
			#pragma unroll
			for(int s = 0; s < 4; s++) a[r][s] -= p[r][s];
	}
	double b[4][4];
	inv4(a, b);
	st16(dinv + 16*static_cast<size_t>(c), b);
}

/// y = B x for a row-major fp32 4x4 block, entries widened to fp64
__device__ __forceinline__ void blk_mv(const float* __restrict__ B, const double4 x, double* y)
{
	const float4* b4 = reinterpret_cast<const float4*>(B);
	#pragma unroll
	for(int i = 0; i < 4; i++) {
		const float4 r = b4[i];
		y[i] = static_cast<double>(r.x)*x.x + static_cast<double>(r.y)*x.y + static_cast<double>(r.z)*x.z
		     + static_cast<double>(r.w)*x.w;
	}
}

template <typename T>
__global__ __launch_bounds__(256)
void k_bjac_apply(int n, const T* __restrict__ dinv, const double* __restrict__ x, double* __restrict__ y)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= n) return;
	double o[4];
	blk_mv(dinv + 16*static_cast<size_t>(c), reinterpret_cast<const double4*>(x)[c], o);
	reinterpret_cast<double4*>(y)[c] = make_double4(o[0], o[1], o[2], o[3]);
}

#ifndef FVHIP_BLOCK_ROWS
#define FVHIP_BLOCK_ROWS 1
#endif
/// k_bjac_apply with four lanes per cell, lane i forming y[c][i] = row i of D^-1 . x[c] (the same dot, in the
/// same order: bitwise k_bjac_apply's y), the block read as four consecutive rows by the cell's four lanes
template <typename T>
__global__ __launch_bounds__(256)
void k_bjac_apply_rows(int n, const T* __restrict__ dinv, const double* __restrict__ x, double* __restrict__ y)
{
	const long long g = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	const int c = static_cast<int>(g >> 2), i = static_cast<int>(g & 3);
	if(c >= n) return;
	const double4 xv = reinterpret_cast<const double4*>(x)[c];
	double o;
	if constexpr(sizeof(T) == sizeof(double)) {
		const double4 r = reinterpret_cast<const double4*>(dinv + 16*static_cast<size_t>(c))[i];
		o = r.x*xv.x + r.y*xv.y + r.z*xv.z + r.w*xv.w;
	} else {
		const float4 r = reinterpret_cast<const float4*>(dinv + 16*static_cast<size_t>(c))[i];
		o = static_cast<double>(r.x)*xv.x + static_cast<double>(r.y)*xv.y + static_cast<double>(r.z)*xv.z
		  + static_cast<double>(r.w)*xv.w;
	}
	y[4*static_cast<size_t>(c) + i] = o;
}

__global__ __launch_bounds__(256)
void k_to_single(long long n, const double* __restrict__ a, float* __restrict__ b)
{
	const long long i = blockIdx.x*256LL + threadIdx.x;
	if(i >= n/4) return;
	const double4 v = reinterpret_cast<const double4*>(a)[i];
	reinterpret_cast<float4*>(b)[i] = make_float4(static_cast<float>(v.x), static_cast<float>(v.y),
	                                              static_cast<float>(v.z), static_cast<float>(v.w));
}

__global__ __launch_bounds__(256)
void k_bjac_correct(int n, const double* __restrict__ dinv, const double* __restrict__ b,
                    const double* __restrict__ y, double* __restrict__ z)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= n) return;
	const double4 bb = reinterpret_cast<const double4*>(b)[c], yy = reinterpret_cast<const double4*>(y)[c];
	double o[4];
	blk_mv(dinv + 16*static_cast<size_t>(c), make_double4(bb.x-yy.x, bb.y-yy.y, bb.z-yy.z, bb.w-yy.w), o);
	double4 zz = reinterpret_cast<double4*>(z)[c];
	zz.x += o[0]; zz.y += o[1]; zz.z += o[2]; zz.w += o[3];
	reinterpret_cast<double4*>(z)[c] = zz;
}

// -------------------------------------------------------------------------------------------------
// reductions and vector updates
// -------------------------------------------------------------------------------------------------
/// block row y of the grid: products j0 = KRY_GROUP*y .. j0+KRY_GROUP-1 (j == k is w . w)
__global__ __launch_bounds__(256)
void k_mdot_partial(long long n, int k, int kt, const double* __restrict__ V, long long ld,
                    const double* __restrict__ w, double* __restrict__ part)
{
	const int j0 = KRY_GROUP*static_cast<int>(blockIdx.y);
	const double* vp[KRY_GROUP];
	#pragma unroll
	for(int q = 0; q < KRY_GROUP; q++) vp[q] = (j0 + q < k) ? V + static_cast<long long>(j0 + q)*ld : w;
	double acc[KRY_GROUP];
	#pragma unroll
	for(int q = 0; q < KRY_GROUP; q++) acc[q] = 0.0;
	// 16-byte loads (n is a multiple of 4: four unknowns per cell); the same fixed order every call
	const long long n2 = n >> 1;
	const double2* w2 = reinterpret_cast<const double2*>(w);
	for(long long i = blockIdx.x*256LL + threadIdx.x; i < n2; i += 256LL*gridDim.x) {
		const double2 wi = w2[i];
		#pragma unroll
		for(int q = 0; q < KRY_GROUP; q++)
			if(j0 + q < kt) {
				const double2 vi = reinterpret_cast<const double2*>(vp[q])[i];
				acc[q] += vi.x*wi.x;
				acc[q] += vi.y*wi.y;
			}
	}
	block_sum<KRY_GROUP>(acc, part + static_cast<size_t>(j0)*KRY_DOT_BLOCKS + blockIdx.x, KRY_DOT_BLOCKS);
}

/// out[b] = sum of the np partials of product b (one block per product)
__global__ __launch_bounds__(256)
void k_sum_partials(int np, const double* __restrict__ part, double* __restrict__ out)
{
	const double* p = part + static_cast<size_t>(blockIdx.x)*np;
	double acc[1] = {0.0};
	for(int i = threadIdx.x; i < np; i += 256) acc[0] += p[i];
	block_sum<1>(acc, out + blockIdx.x, 1);
}

/// s += c[j] * X[j*ld + i] over j = 0 .. k-1 in order (X read as T rows: double or double2)
template <typename T, typename F>
__device__ __forceinline__ void basis_sum(int k, const double* __restrict__ c, const double* __restrict__ V, long long ld,
                                          long long i, F&& add)
{
	for(int j = 0; j < k; j++) add(c[j], reinterpret_cast<const T*>(V + j*ld)[i]);
}

__global__ __launch_bounds__(256)
void k_maxpy(long long n, int k, const double* __restrict__ V, long long ld, const double* __restrict__ h,
             double* __restrict__ w)
{
	const long long i = blockIdx.x*256LL + threadIdx.x;
	if(i >= n) return;
	double s = 0.0;
	basis_sum<double>(k, h, V, ld, i, [&](double c, double v) { s += c*v; });
	w[i] -= s;
}

/// w -= V h over k basis vectors (k_maxpy's sum, in its order: the same w bit for bit) and |w|^2 of the result,
/// over the multi-dot's fixed partition and tree: the Arnoldi step's new norm without another pass over w
__global__ __launch_bounds__(256)
void k_maxpy_norm(long long n, int k, const double* __restrict__ V, long long ld, const double* __restrict__ h,
                  double* __restrict__ w, double* __restrict__ part)
{
	double acc[1] = {0.0};
	const long long n2 = n >> 1;
	double2* w2 = reinterpret_cast<double2*>(w);
	for(long long i = blockIdx.x*256LL + threadIdx.x; i < n2; i += 256LL*gridDim.x) {
		double sx = 0.0, sy = 0.0;
		basis_sum<double2>(k, h, V, ld, i, [&](double c, double2 v) { sx += c*v.x; sy += c*v.y; });
		double2 wi = w2[i];
		wi.x -= sx; wi.y -= sy;
		w2[i] = wi;
		acc[0] += wi.x*wi.x;
		acc[0] += wi.y*wi.y;
	}
	block_sum<1>(acc, part + blockIdx.x, 1);
}

__global__ __launch_bounds__(256)
void k_lincomb(long long n, int k, const double* __restrict__ V, long long ld, const double* __restrict__ c,
               double* __restrict__ out)
{
	const long long i = blockIdx.x*256LL + threadIdx.x;
	if(i >= n) return;
	double s = 0.0;
	basis_sum<double>(k, c, V, ld, i, [&](double cj, double v) { s += cj*v; });
	out[i] = s;
}

__global__ __launch_bounds__(256)
void k_axpby(long long n, double a, const double* __restrict__ x, double b, double* __restrict__ y)
{
	const long long i = blockIdx.x*256LL + threadIdx.x;
	if(i >= n) return;
	y[i] = b == 0.0 ? a*x[i] : a*x[i] + b*y[i];
}

__global__ void k_pertmag(const double* __restrict__ sq, double eps, double* __restrict__ pm)
{
	if(threadIdx.x == 0 && blockIdx.x == 0) {
		const double xnorm = sqrt(sq[0]);
		pm[0] = xnorm;
		pm[1] = eps/xnorm;
	}
}

__global__ __launch_bounds__(256)
void k_energy_partial(int n, const double* __restrict__ r, const double* __restrict__ area, double* __restrict__ part)
{
	double acc[1] = {0.0};
	for(int e = blockIdx.x*256 + threadIdx.x; e < n; e += 256*gridDim.x)
		acc[0] += r[4*static_cast<size_t>(e)+3]*r[4*static_cast<size_t>(e)+3]*area[e];
	block_sum<1>(acc, part + blockIdx.x, 1);
}

__global__ __launch_bounds__(256)
void k_relaxed_update(int n, gd::Gas G, double minfactor, const double* __restrict__ du, double* __restrict__ u)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= n) return;
	const double4 a = reinterpret_cast<const double4*>(u)[c];
	const double4 d = reinterpret_cast<const double4*>(du)[c];
	const double uu[4] = {a.x, a.y, a.z, a.w}, dd[4] = {d.x, d.y, d.z, d.w};
	const double om = relaxation_factor(G, minfactor, dd, uu);
	reinterpret_cast<double4*>(u)[c] = make_double4(uu[0] + om*dd[0], uu[1] + om*dd[1], uu[2] + om*dd[2],
	                                                uu[3] + om*dd[3]);
}

// -------------------------------------------------------------------------------------------------
// launchers
// -------------------------------------------------------------------------------------------------
// -------------------------------------------------------------------------------------------------
// line-implicit preconditioner: block-tridiagonal solves along lines of strongly coupled cells
// -------------------------------------------------------------------------------------------------
/// the coupling blocks between line cells k-1 = p and k = c through interior face code fc = fi<<1 | o:
/// o = 0: p is the face's L, so A[c][p] = lower[fi] (A[R][L]) and A[p][c] = upper[fi]; o = 1: swapped
__device__ __forceinline__ const double* blk_cp(int fc, const double* lower, const double* upper) {
	return ((fc & 1) ? upper : lower) + 16*static_cast<size_t>(fc >> 1);
}
__device__ __forceinline__ const double* blk_pc(int fc, const double* lower, const double* upper) {
	return ((fc & 1) ? lower : upper) + 16*static_cast<size_t>(fc >> 1);
}

/// Row r of a pair-interleaved 4x4 block array (LineSet): elements 2q, 2q+1 of lane j's block at
/// double2 index 512 r + 64 q + j -- one 16-byte load per lane per element pair, 1 KB contiguous per
/// wave instruction, 8 instructions per block instead of 16 8-byte loads (C4 line-implicit step
/// 9.41 -> 9.12 ms, same-box A/B, profiles/r03/ab/abl_*)
__device__ __forceinline__ void ldP16(const double* __restrict__ X, long long r, int j, double (&a)[4][4])
{
	const double2* p = reinterpret_cast<const double2*>(X) + 512*r + j;
	#pragma unroll
	for(int q = 0; q < 8; q++) { const double2 t = p[64*q]; a[q >> 1][(q & 1)*2] = t.x; a[q >> 1][(q & 1)*2 + 1] = t.y; }
}
__device__ __forceinline__ void stP16(double* __restrict__ X, long long r, int j, const double (&a)[4][4])
{
	double2* p = reinterpret_cast<double2*>(X) + 512*r + j;
	#pragma unroll
	for(int q = 0; q < 8; q++) p[64*q] = make_double2(a[q >> 1][(q & 1)*2], a[q >> 1][(q & 1)*2 + 1]);
}
/// fp32 storage of the same rows (prec_single): row q of lane j's block as one float4 at index
/// 256 r + 64 q + j -- 4 KB per row, 4 coalesced 16-byte loads per block; the recurrence itself runs in fp64
__device__ __forceinline__ void ldP16(const float* __restrict__ X, long long r, int j, double (&a)[4][4])
{
	const float4* p = reinterpret_cast<const float4*>(X) + 256*r + j;
	#pragma unroll
	for(int q = 0; q < 4; q++) { const float4 t = p[64*q]; a[q][0] = t.x; a[q][1] = t.y; a[q][2] = t.z; a[q][3] = t.w; }
}
__device__ __forceinline__ void stP16(float* __restrict__ X, long long r, int j, const double (&a)[4][4])
{
	float4* p = reinterpret_cast<float4*>(X) + 256*r + j;
	#pragma unroll
	for(int q = 0; q < 4; q++)
		p[64*q] = make_float4(static_cast<float>(a[q][0]), static_cast<float>(a[q][1]), static_cast<float>(a[q][2]),
		                      static_cast<float>(a[q][3]));
}

/// block-Thomas factorisation, lane j of workgroup g on line 64g + j (LineSet): per line cell k
///   W_{k-1} = dinvp_{k-1} A[k-1][k],  dinvp_k = (D_k - A[k][k-1] W_{k-1})^-1
/// and D, Lb, W stored pair-interleaved for the solve. The next cell's blocks are requested before the
/// current cell's arithmetic (their addresses do not depend on it) and the cell/face codes two cells
/// ahead, so the recurrence does not wait a memory round trip per cell.
/// Twisted groups (g < twisted_groups; ctx.hpp ensureLines): lane j walks the top half of line j and
/// lane j+32 the bottom half backwards, each list ending in the twist cell t. A half stops at t with the
/// Schur term S = A[t][last] W_last of its side instead of a pivot; the two lanes swap S and lane j
/// stores the twist pivot (A_tt - S_top - S_bottom)^-1 in its row of t. That is the same block
/// elimination of the same block-tridiagonal matrix, ordered from both ends: the chain per lane halves.
template <typename T>
__global__ __launch_bounds__(64)
void k_line_factor(const int* __restrict__ gstart, const int* __restrict__ lcell, const int* __restrict__ lface,
                   const int* __restrict__ llen, int twisted_groups,
                   const double* __restrict__ diag, const double* __restrict__ lower, const double* __restrict__ upper,
                   T* __restrict__ D, T* __restrict__ Lb, T* __restrict__ W)
{
	const int g = blockIdx.x, j = threadIdx.x;
	const long long r0 = gstart[g];
	const int len = llen[64*g + j];
	const bool tw = g < twisted_groups;
	double a[4][4], Lk[4][4], Uk[4][4], prev[4][4], S[4][4];
	if(len > 0) {
	int c = lcell[64*r0 + j];
	int c1 = len > 1 ? lcell[64*(r0+1) + j] : -1, f1 = len > 1 ? lface[64*(r0+1) + j] : -1;
	ld16(diag + 16*static_cast<size_t>(c), a);
	for(int k = 0; k < len; k++) {
		// requests for cell k+1 (blocks) and k+2 (codes)
		const int cn = c1, fn = f1;
		c1 = -1; f1 = -1;
		if(cn >= 0 && k + 2 < len) { c1 = lcell[64*(r0+k+2) + j]; f1 = lface[64*(r0+k+2) + j]; }
		double an[4][4], Ln[4][4], Un[4][4];
		if(cn >= 0) {
			ld16(diag + 16*static_cast<size_t>(cn), an);
			ld16(blk_cp(fn, lower, upper), Ln);
			ld16(blk_pc(fn, lower, upper), Un);
		}
		if(k > 0) {
			double t[4][4];
			#pragma unroll
			for(int r = 0; r < 4; r++)
				#pragma unroll
				for(int q = 0; q < 4; q++) t[r][q] = prev[r][0]*Uk[0][q] + prev[r][1]*Uk[1][q] + prev[r][2]*Uk[2][q] + prev[r][3]*Uk[3][q];
			stP16(W, r0 + k - 1, j, t);
			stP16(Lb, r0 + k, j, Lk);
			if(tw && k == len - 1) {                   // the twist: this side's Schur term, no pivot
				#pragma unroll
				for(int r = 0; r < 4; r++)
					#pragma unroll
					for(int q = 0; q < 4; q++) S[r][q] = Lk[r][0]*t[0][q] + Lk[r][1]*t[1][q] + Lk[r][2]*t[2][q] + Lk[r][3]*t[3][q];
				break;
			}
			#pragma unroll
			for(int r = 0; r < 4; r++)
				#pragma unroll
				for(int q = 0; q < 4; q++) a[r][q] -= Lk[r][0]*t[0][q] + Lk[r][1]*t[1][q] + Lk[r][2]*t[2][q] + Lk[r][3]*t[3][q];
		}
		inv4(a, prev);
		stP16(D, r0 + k, j, prev);
		if(cn < 0) break;
		#pragma unroll
		for(int r = 0; r < 4; r++)
			#pragma unroll
			for(int q = 0; q < 4; q++) { a[r][q] = an[r][q]; Lk[r][q] = Ln[r][q]; Uk[r][q] = Un[r][q]; }
	}
	}
	if(!tw) return;
	// twist pivot: lane j (top half) combines both sides' Schur terms, a = A_tt on both lanes
	double So[4][4];
	#pragma unroll
	for(int r = 0; r < 4; r++)
		#pragma unroll
		for(int q = 0; q < 4; q++) So[r][q] = __shfl_xor(S[r][q], 32);
	if(j < 32 && len > 0) {
		#pragma unroll
		for(int r = 0; r < 4; r++)
			#pragma unroll
			for(int q = 0; q < 4; q++) a[r][q] = (a[r][q] - S[r][q]) - So[r][q];
		inv4(a, prev);
		stP16(D, r0 + len - 1, j, prev);
	}
}

/// z = (block-tridiagonal line part)^-1 v, lanes as in k_line_factor, lane j's line llen[64g + j] cells
/// long: forward g_k = dinvp_k (v_k - A[k][k-1] g_{k-1}) into the pair-interleaved scratch G, backward
/// z_k = g_k - W_k z_{k+1}; the next cell's rows (and its v row) are requested before the current
/// cell's arithmetic. (A deeper register ring of rows in flight -- 3 or 4 cells ahead -- exceeds the 256
/// architected VGPRs and turns into accumulator-register copies that wait on the loads: measured
/// slower, profiles/r03/ab/abl_*.)
/// Twisted groups: each half's forward sweep ends at the twist cell t with s = A[t][last] g_last; the
/// lanes swap s, lane j forms z_t = pivot_t (v_t - s_top - s_bottom) and hands it to lane j+32, and both
/// sweep back from z_t.
/// one lane's line of k_line_solve; returns the sum of squares of the z rows this lane wrote
template <typename T>
__device__ __forceinline__ double line_solve_lane(int g, int j, const int* __restrict__ gstart, const int* __restrict__ lcell,
                                                  const int* __restrict__ llen, int twisted_groups,
                                                  const T* __restrict__ D, const T* __restrict__ Lb,
                                                  const T* __restrict__ W, double* __restrict__ G,
                                                  const double* __restrict__ v, double* __restrict__ z)
{
	double zz = 0.0;
	const long long r0 = gstart[g];
	const int n = llen[64*g + j];
	const bool tw = g < twisted_groups;
	if(n == 0 && !tw) return zz;
	const int* cl = lcell + 64*r0 + j;
	const double4* v4 = reinterpret_cast<const double4*>(v);
	double4* z4 = reinterpret_cast<double4*>(z);
	double2* G2 = reinterpret_cast<double2*>(G) + 128*r0 + j;     // row k: G2[128k], G2[128k + 64]
	double Dk[4][4], Lk[4][4];
	double4 gp = make_double4(0, 0, 0, 0), vk = make_double4(0, 0, 0, 0), s = make_double4(0, 0, 0, 0);
	// the cells of rows k+1 and k+2 are known before row k's arithmetic: the v row of k+1 is requested
	// without first waiting for its cell index (one memory round trip per cell instead of two)
	int c1 = n > 1 ? cl[64] : 0, c2 = n > 2 ? cl[128] : 0;
	if(n > 0) { vk = v4[cl[0]]; ldP16(D, r0, j, Dk); }
	for(int k = 0; k < n; k++) {
		double Dn[4][4], Ln[4][4];
		double4 vn = make_double4(0, 0, 0, 0);
		if(k + 1 < n) {
			vn = v4[c1];
			ldP16(D, r0 + k + 1, j, Dn);
			ldP16(Lb, r0 + k + 1, j, Ln);
			c1 = c2;
			c2 = k + 3 < n ? cl[64*(k+3)] : 0;
		}
		if(tw && k == n - 1) {                         // the twist: this side's term A[t][last] g_last
			s = make_double4(Lk[0][0]*gp.x + Lk[0][1]*gp.y + Lk[0][2]*gp.z + Lk[0][3]*gp.w,
			                 Lk[1][0]*gp.x + Lk[1][1]*gp.y + Lk[1][2]*gp.z + Lk[1][3]*gp.w,
			                 Lk[2][0]*gp.x + Lk[2][1]*gp.y + Lk[2][2]*gp.z + Lk[2][3]*gp.w,
			                 Lk[3][0]*gp.x + Lk[3][1]*gp.y + Lk[3][2]*gp.z + Lk[3][3]*gp.w);
			break;
		}
		double r[4] = {vk.x, vk.y, vk.z, vk.w};
		if(k > 0) {
			#pragma unroll
			for(int i = 0; i < 4; i++) r[i] -= Lk[i][0]*gp.x + Lk[i][1]*gp.y + Lk[i][2]*gp.z + Lk[i][3]*gp.w;
		}
		double y[4];
		#pragma unroll
		for(int i = 0; i < 4; i++) y[i] = Dk[i][0]*r[0] + Dk[i][1]*r[1] + Dk[i][2]*r[2] + Dk[i][3]*r[3];
		gp = make_double4(y[0], y[1], y[2], y[3]);
		if(k + 1 == n) break;
		G2[128*k] = make_double2(y[0], y[1]); G2[128*k + 64] = make_double2(y[2], y[3]);
		#pragma unroll
		for(int i = 0; i < 4; i++)
			#pragma unroll
			for(int q = 0; q < 4; q++) { Dk[i][q] = Dn[i][q]; Lk[i][q] = Ln[i][q]; }
		vk = vn;
	}
	// backward from the line's last cell: z_{n-1} = g_{n-1}; twisted: from the twist cell's z_t
	double4 x = gp;
	if(tw) {
		const double4 so = make_double4(__shfl_xor(s.x, 32), __shfl_xor(s.y, 32), __shfl_xor(s.z, 32), __shfl_xor(s.w, 32));
		if(j < 32 && n > 0) {
			double Dt[4][4];
			ldP16(D, r0 + n - 1, j, Dt);                 // lane j's row of t holds the twist pivot
			const double r[4] = {(vk.x - s.x) - so.x, (vk.y - s.y) - so.y, (vk.z - s.z) - so.z, (vk.w - s.w) - so.w};
			double y[4];
			#pragma unroll
			for(int i = 0; i < 4; i++) y[i] = Dt[i][0]*r[0] + Dt[i][1]*r[1] + Dt[i][2]*r[2] + Dt[i][3]*r[3];
			x = make_double4(y[0], y[1], y[2], y[3]);
			z4[cl[64*(n-1)]] = x;
			zz += x.x*x.x; zz += x.y*x.y; zz += x.z*x.z; zz += x.w*x.w;
		}
		const double4 xo = make_double4(__shfl_xor(x.x, 32), __shfl_xor(x.y, 32), __shfl_xor(x.z, 32), __shfl_xor(x.w, 32));
		if(j >= 32) x = xo;                            // z_t from lane j
		if(n == 0) return zz;
	}
	else {
		z4[cl[64*(n-1)]] = x;
		zz += x.x*x.x; zz += x.y*x.y; zz += x.z*x.z; zz += x.w*x.w;
	}
	if(n == 1) return zz;
	double Wk[4][4];
	ldP16(W, r0 + n - 2, j, Wk);
	double2 ga = G2[128*(n-2)], gb = G2[128*(n-2) + 64];
	int ck = cl[64*(n-2)];
	for(int k = n - 2; k >= 0; k--) {
		double Wn[4][4];
		double2 na = make_double2(0, 0), nb = make_double2(0, 0);
		int cp = -1;
		if(k > 0) {
			ldP16(W, r0 + k - 1, j, Wn);
			na = G2[128*(k-1)]; nb = G2[128*(k-1) + 64];
			cp = cl[64*(k-1)];
		}
		double y[4];
		#pragma unroll
		for(int i = 0; i < 4; i++) y[i] = Wk[i][0]*x.x + Wk[i][1]*x.y + Wk[i][2]*x.z + Wk[i][3]*x.w;
		x = make_double4(ga.x - y[0], ga.y - y[1], gb.x - y[2], gb.y - y[3]);
		z4[ck] = x;
		zz += x.x*x.x; zz += x.y*x.y; zz += x.z*x.z; zz += x.w*x.w;
		if(k == 0) break;
		#pragma unroll
		for(int i = 0; i < 4; i++)
			#pragma unroll
			for(int q = 0; q < 4; q++) Wk[i][q] = Wn[i][q];
		ga = na; gb = nb; ck = cp;
	}
	return zz;
}

template <typename T>
__global__ __launch_bounds__(64)
void k_line_solve(const int* __restrict__ gstart, const int* __restrict__ lcell, const int* __restrict__ llen,
                  int twisted_groups, const T* __restrict__ D, const T* __restrict__ Lb,
                  const T* __restrict__ W, double* __restrict__ G, const double* __restrict__ v, double* __restrict__ z,
                  double* __restrict__ zpart)
{
	double zz = line_solve_lane<T>(blockIdx.x, threadIdx.x, gstart, lcell, llen, twisted_groups, D, Lb, W, G, v, z);
	if(!zpart) return;
	// the group's sum of squares: a fixed shuffle tree over the 64 lanes
	#pragma unroll
	for(int off = 32; off > 0; off >>= 1) zz += __shfl_xor(zz, off);
	if(threadIdx.x == 0) zpart[blockIdx.x] = zz;
}

/// Row i (4 values) of slot j's 4x4 block in group row r of the pair-interleaved factor storage (ldP16's
/// rows q = 2i, 2i+1; fp32: the float4 of row i)
__device__ __forceinline__ void ldRow(const double* __restrict__ X, long long r, int j, int i, double (&a)[4])
{
	const double2* p = reinterpret_cast<const double2*>(X) + 512*r + 128*i + j;
	const double2 t0 = p[0], t1 = p[64];
	a[0] = t0.x; a[1] = t0.y; a[2] = t1.x; a[3] = t1.y;
}
__device__ __forceinline__ void ldRow(const float* __restrict__ X, long long r, int j, int i, double (&a)[4])
{
	const float4 t = reinterpret_cast<const float4*>(X)[256*r + 64*i + j];
	a[0] = t.x; a[1] = t.y; a[2] = t.z; a[3] = t.w;
}
/// lane Q's value of this lane's quad (DPP quad_perm, no LDS crossbar)
template <int Q>
__device__ __forceinline__ double quad_bcast(double x)
{
	constexpr int ctrl = Q | (Q << 2) | (Q << 4) | (Q << 6);
	const long long b = __double_as_longlong(x);
	const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(b), ctrl, 0xF, 0xF, false);
	const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(b >> 32), ctrl, 0xF, 0xF, false);
	return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}
__device__ __forceinline__ void quad_all(double x, double (&o)[4])
{
	o[0] = quad_bcast<0>(x); o[1] = quad_bcast<1>(x); o[2] = quad_bcast<2>(x); o[3] = quad_bcast<3>(x);
}

/// The line solve with four lanes per line (one block row each) for the twisted groups -- the long lines,
/// whose one-lane chains of dependent loads bound k_line_solve -- and the one-lane form for the others.
/// Block b < twisted_groups is twisted group b: wave w takes slots 8w..8w+7 (top halves) and their partners
/// 32+8w..32+8w+7 (bottom halves), lane 4 q + i row i of the q-th of those 16 slots, so a slot's partner is
/// lane ^ 32. Per cell a lane loads its rows of D, Lb (W backward) and its component of v (g, z): the
/// quad's four lanes read whole rows. The rows of the next P cells are in flight while a cell is computed
/// (a ring of P register slots, the cell ids 2P ahead), and the quad exchanges its four components by DPP.
/// Each row is computed in the lane that owns it with k_line_solve's expressions, and the z.z sums keep
/// that kernel's order (a quad's row-0 lane sums the rows its slot writes; the group's 64 slot sums go
/// through the same butterfly): z and zsq are bitwise k_line_solve's. Blocks past the twisted groups take
/// four one-lane groups each (a wave per group).
template <typename T, int P>
__global__ __launch_bounds__(256)
void k_line_solve_rows(const int* __restrict__ gstart, const int* __restrict__ lcell, const int* __restrict__ llen,
                       int twisted_groups, int ngroups, const T* __restrict__ D, const T* __restrict__ Lb,
                       const T* __restrict__ W, double* __restrict__ G, const double* __restrict__ v,
                       double* __restrict__ z, double* __restrict__ zpart)
{
	const int b = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
	if(b >= twisted_groups) {                             // block-uniform
		const int g = twisted_groups + 4*(b - twisted_groups) + w;
		if(g >= ngroups) return;
		double zz = line_solve_lane<T>(g, lane, gstart, lcell, llen, twisted_groups, D, Lb, W, G, v, z);
		if(!zpart) return;
		#pragma unroll
		for(int off = 32; off > 0; off >>= 1) zz += __shfl_xor(zz, off);
		if(lane == 0) zpart[g] = zz;
		return;
	}
	__shared__ double zs[64];
	const int g = b, qd = lane >> 2, i = lane & 3;
	const bool top = qd < 8;
	const int j = top ? 8*w + qd : 24 + 8*w + qd;         // 32 + 8w + (qd - 8)
	const long long r0 = gstart[g];
	const int n = llen[64*g + j];
	const int* cl = lcell + 64*r0 + j;
	auto gix = [&](int k) { return 2*(128*(r0 + k) + 64*(i >> 1) + j) + (i & 1); };
	double zz = 0.0;
	double gp[4] = {0.0, 0.0, 0.0, 0.0};
	double vt = 0.0, s = 0.0;
	// forward over cells 0 .. n-2, then the twist cell n-1 (every slot of these groups ends in one). The
	// loads are unconditional (rows past the end are clamped to the last cell and land in slots whose cell
	// is done) and the loop runs whole rounds of P cells with the remainder after it: one back edge, no
	// early exits, so the compiler keeps the ring in flight across steps instead of draining it.
	auto fwd = [&](int k, double (&Dk)[4], double (&Lk)[4], double& vk, int& ck) {
		double r = vk;
		if(k > 0) r -= Lk[0]*gp[0] + Lk[1]*gp[1] + Lk[2]*gp[2] + Lk[3]*gp[3];
		double rq[4];
		quad_all(r, rq);
		const double y = Dk[0]*rq[0] + Dk[1]*rq[1] + Dk[2]*rq[2] + Dk[3]*rq[3];
		quad_all(y, gp);
		G[gix(k)] = y;
		const int kk = min(k + P, n - 1);
		ldRow(D, r0 + kk, j, i, Dk);
		ldRow(Lb, r0 + kk, j, i, Lk);
		vk = v[4*static_cast<size_t>(ck) + i];
		ck = cl[64*min(k + 2*P, n - 1)];
		__builtin_amdgcn_sched_barrier(0);              // the machine scheduler would sink these loads to the round's end
	};
	if(n > 0) {
		double Dr[P][4], Lr[P][4], vr[P];
		int cn[P];
		#pragma unroll
		for(int u = 0; u < P; u++) {
			const int kk = min(u, n - 1);
			ldRow(D, r0 + kk, j, i, Dr[u]);
			ldRow(Lb, r0 + kk, j, i, Lr[u]);
			vr[u] = v[4*static_cast<size_t>(cl[64*kk]) + i];
			cn[u] = cl[64*min(P + u, n - 1)];
		}
		const int nf = n - 1, full = nf - nf % P;
		for(int base = 0; base < full; base += P) {
			#pragma unroll
			for(int u = 0; u < P; u++) fwd(base + u, Dr[u], Lr[u], vr[u], cn[u]);
		}
		#pragma unroll
		for(int u = 0; u < P - 1; u++)
			if(full + u < nf) fwd(full + u, Dr[u], Lr[u], vr[u], cn[u]);
		// the twist: this side's term A[t][last] g_last, from the ring slot of cell n-1
		const int ut = nf % P;
		#pragma unroll
		for(int u = 0; u < P; u++)
			if(u == ut) {
				s = Lr[u][0]*gp[0] + Lr[u][1]*gp[1] + Lr[u][2]*gp[2] + Lr[u][3]*gp[3];
				vt = vr[u];
			}
	}
	// the twist cell: the top lane of the pair forms z_t = pivot_t (v_t - s_top - s_bottom), the bottom
	// lane receives it
	double x[4];
	{
		const double so = __shfl_xor(s, 32);
		x[0] = 0.0; x[1] = 0.0; x[2] = 0.0; x[3] = 0.0;
		if(top && n > 0) {
			double Dt[4];
			ldRow(D, r0 + n - 1, j, i, Dt);
			const double r = (vt - s) - so;
			double rq[4];
			quad_all(r, rq);
			const double y = Dt[0]*rq[0] + Dt[1]*rq[1] + Dt[2]*rq[2] + Dt[3]*rq[3];
			quad_all(y, x);
			z[4*static_cast<size_t>(cl[64*(n - 1)]) + i] = y;
			if(i == 0) { zz += x[0]*x[0]; zz += x[1]*x[1]; zz += x[2]*x[2]; zz += x[3]*x[3]; }
		}
		double xo[4];
		#pragma unroll
		for(int q = 0; q < 4; q++) xo[q] = __shfl_xor(x[q], 32);
		if(!top) {
			#pragma unroll
			for(int q = 0; q < 4; q++) x[q] = xo[q];
		}
	}
	// backward: z_k = g_k - W_k z_{k+1}, k = n-2 .. 0 (clamped loads, whole rounds, as forward)
	auto bwd = [&](int k, double (&Wk)[4], double& gk, int& ck) {
		const double y = Wk[0]*x[0] + Wk[1]*x[1] + Wk[2]*x[2] + Wk[3]*x[3];
		const double xi = gk - y;
		quad_all(xi, x);
		z[4*static_cast<size_t>(ck) + i] = xi;
		if(i == 0) { zz += x[0]*x[0]; zz += x[1]*x[1]; zz += x[2]*x[2]; zz += x[3]*x[3]; }
		const int k2 = max(k - P, 0);
		ldRow(W, r0 + k2, j, i, Wk); gk = G[gix(k2)]; ck = cl[64*k2];
		__builtin_amdgcn_sched_barrier(0);
	};
	if(n > 1) {
		double Wr[P][4], gr[P];
		int zc[P];
		#pragma unroll
		for(int u = 0; u < P; u++) {
			const int k = max(n - 2 - u, 0);
			ldRow(W, r0 + k, j, i, Wr[u]); gr[u] = G[gix(k)]; zc[u] = cl[64*k];
		}
		const int nb = n - 1, full = nb - nb % P;
		for(int base = 0; base < full; base += P) {
			#pragma unroll
			for(int u = 0; u < P; u++) bwd(n - 2 - (base + u), Wr[u], gr[u], zc[u]);
		}
		#pragma unroll
		for(int u = 0; u < P - 1; u++)
			if(full + u < nb) bwd(n - 2 - (full + u), Wr[u], gr[u], zc[u]);
	}
	if(!zpart) return;                                    // block-uniform
	if(i == 0) zs[j] = zz;
	__syncthreads();
	if(w == 0) {
		double t = zs[lane];
		#pragma unroll
		for(int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
		if(lane == 0) zpart[g] = t;
	}
}

/// z += e (4 doubles per cell)
__global__ __launch_bounds__(256)
void k_add_rows(int n, const double* __restrict__ e, double* __restrict__ z)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= n) return;
	const double4 a = reinterpret_cast<const double4*>(e)[c];
	double4 b = reinterpret_cast<double4*>(z)[c];
	b.x += a.x; b.y += a.y; b.z += a.z; b.w += a.w;
	reinterpret_cast<double4*>(z)[c] = b;
}

void launch_line_factor(const LineSet& Ls, const double* diag, const double* lower, const double* upper, hipStream_t s)
{
	if(Ls.ngroups <= 0) return;
	if(Ls.single)
		hipLaunchKernelGGL(k_line_factor<float>, dim3(Ls.ngroups), dim3(64), 0, s, Ls.gstart, Ls.cell, Ls.face, Ls.len,
		                   Ls.twisted_groups, diag, lower, upper, reinterpret_cast<float*>(Ls.D),
		                   reinterpret_cast<float*>(Ls.Lb), reinterpret_cast<float*>(Ls.W));
	else
		hipLaunchKernelGGL(k_line_factor<double>, dim3(Ls.ngroups), dim3(64), 0, s, Ls.gstart, Ls.cell, Ls.face, Ls.len,
		                   Ls.twisted_groups, diag, lower, upper, Ls.D, Ls.Lb, Ls.W);
}

#ifndef FVHIP_LINE_ROWS
#define FVHIP_LINE_ROWS 4
#endif
void launch_line_solve(const LineSet& Ls, const double* v, double* z, hipStream_t s, double* zsq)
{
	if(Ls.ngroups <= 0) return;
	double* zp = zsq ? Ls.zpart : nullptr;
	if(FVHIP_LINE_ROWS > 0) {
		constexpr int P = FVHIP_LINE_ROWS > 0 ? FVHIP_LINE_ROWS : 1;
		const int T = Ls.twisted_groups, nb = T + (Ls.ngroups - T + 3)/4;
		if(Ls.single)
			hipLaunchKernelGGL((k_line_solve_rows<float, P>), dim3(nb), dim3(256), 0, s, Ls.gstart, Ls.cell, Ls.len, T,
			                   Ls.ngroups, reinterpret_cast<const float*>(Ls.D), reinterpret_cast<const float*>(Ls.Lb),
			                   reinterpret_cast<const float*>(Ls.W), Ls.G, v, z, zp);
		else
			hipLaunchKernelGGL((k_line_solve_rows<double, P>), dim3(nb), dim3(256), 0, s, Ls.gstart, Ls.cell, Ls.len, T,
			                   Ls.ngroups, Ls.D, Ls.Lb, Ls.W, Ls.G, v, z, zp);
	}
	else if(Ls.single)
		hipLaunchKernelGGL(k_line_solve<float>, dim3(Ls.ngroups), dim3(64), 0, s, Ls.gstart, Ls.cell, Ls.len,
		                   Ls.twisted_groups, reinterpret_cast<const float*>(Ls.D), reinterpret_cast<const float*>(Ls.Lb),
		                   reinterpret_cast<const float*>(Ls.W), Ls.G, v, z, zp);
	else
		hipLaunchKernelGGL(k_line_solve<double>, dim3(Ls.ngroups), dim3(64), 0, s, Ls.gstart, Ls.cell, Ls.len,
		                   Ls.twisted_groups, Ls.D, Ls.Lb, Ls.W, Ls.G, v, z, zp);
	if(zp) k_sum_partials<<<1, 256, 0, s>>>(Ls.ngroups, zp, zsq);
}

void launch_add_rows(int n, const double* e, double* z, hipStream_t s)
{
	if(n > 0) hipLaunchKernelGGL(k_add_rows, dim3(nblk(n, 256)), dim3(256), 0, s, n, e, z);
}

void launch_bjac_invert(int n, const double* diag, double* dinv, hipStream_t s)
{ if(n > 0) k_bjac_invert<<<nblk(n,256), 256, 0, s>>>(n, diag, dinv); }
void launch_ilu_factor_colour(int ncell, int nbface, const int4* rfaces, const int4* nbrs, const int* colour, int q,
                              const double* diag, const double* lower, const double* upper, double* dinv,
                              const int* cells, int n, hipStream_t s)
{
	if(n > 0) k_ilu_factor_colour<<<nblk(n,256), 256, 0, s>>>(ncell, nbface, rfaces, nbrs, colour, q, diag, lower, upper,
	                                                           dinv, cells, n);
}
void launch_bjac_apply(int n, const double* dinv, const double* x, double* y, hipStream_t s)
{
	if(n <= 0) return;
	if(FVHIP_BLOCK_ROWS) k_bjac_apply_rows<double><<<nblk(4LL*n,256), 256, 0, s>>>(n, dinv, x, y);
	else k_bjac_apply<double><<<nblk(n,256), 256, 0, s>>>(n, dinv, x, y);
}
void launch_bjac_apply(int n, const float* dinv, const double* x, double* y, hipStream_t s)
{
	if(n <= 0) return;
	if(FVHIP_BLOCK_ROWS) k_bjac_apply_rows<float><<<nblk(4LL*n,256), 256, 0, s>>>(n, dinv, x, y);
	else k_bjac_apply<float><<<nblk(n,256), 256, 0, s>>>(n, dinv, x, y);
}
void launch_to_single(long long n, const double* a, float* b, hipStream_t s)
{ if(n > 0) k_to_single<<<nblk(n/4,256), 256, 0, s>>>(n, a, b); }
void launch_bjac_correct(int n, const double* dinv, const double* b, const double* y, double* z, hipStream_t s)
{ if(n > 0) k_bjac_correct<<<nblk(n,256), 256, 0, s>>>(n, dinv, b, y, z); }

size_t kry_scratch(int k)
{
	return static_cast<size_t>(KRY_DOT_BLOCKS)*static_cast<size_t>((k + KRY_GROUP)/KRY_GROUP*KRY_GROUP);
}

void launch_mdot(long long n, int k, const double* V, long long ld, const double* w, bool self,
                 double* part, double* out, hipStream_t s)
{
	const int kt = k + (self ? 1 : 0);
	if(kt <= 0) return;
	k_mdot_partial<<<dim3(KRY_DOT_BLOCKS, (kt + KRY_GROUP - 1)/KRY_GROUP), 256, 0, s>>>(n, k, kt, V, ld, w, part);
	k_sum_partials<<<kt, 256, 0, s>>>(KRY_DOT_BLOCKS, part, out);
}

void launch_maxpy(long long n, int k, const double* V, long long ld, const double* h, double* w, hipStream_t s)
{ if(n > 0 && k > 0) k_maxpy<<<nblk(n,256), 256, 0, s>>>(n, k, V, ld, h, w); }
void launch_maxpy_norm(long long n, int k, const double* V, long long ld, const double* h, double* w, double* part,
                       double* out, hipStream_t s)
{
	k_maxpy_norm<<<KRY_DOT_BLOCKS, 256, 0, s>>>(n, k, V, ld, h, w, part);
	k_sum_partials<<<1, 256, 0, s>>>(KRY_DOT_BLOCKS, part, out);
}
void launch_lincomb(long long n, int k, const double* V, long long ld, const double* c, double* out, hipStream_t s)
{ if(n > 0) k_lincomb<<<nblk(n,256), 256, 0, s>>>(n, k, V, ld, c, out); }
void launch_axpby(long long n, double a, const double* x, double b, double* y, hipStream_t s)
{ if(n > 0) k_axpby<<<nblk(n,256), 256, 0, s>>>(n, a, x, b, y); }
void launch_pertmag(const double* sq, double eps, double* pm, hipStream_t s)
{ k_pertmag<<<1, 64, 0, s>>>(sq, eps, pm); }

void launch_energy_sumsq(int n, const double* r, const double* area, double* part, double* out, hipStream_t s)
{
	k_energy_partial<<<KRY_BLOCKS, 256, 0, s>>>(n, r, area, part);
	k_sum_partials<<<1, 256, 0, s>>>(KRY_BLOCKS, part, out);
}

void launch_relaxed_update(int n, const gd::Gas& G, double minfactor, const double* du, double* u, hipStream_t s)
{ if(n > 0) k_relaxed_update<<<nblk(n,256), 256, 0, s>>>(n, G, minfactor, du, u); }

}
