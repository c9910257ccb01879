/** \file krylov.hip
 * \brief Device linear algebra of the implicit pseudo-time solver (declarations and sources in
 *   krylov.hpp). One thread per cell for the 4x4 block kernels (128 B of blocks and 64 B of
 *   vectors per cell, HBM-bound); the multi-dot reads w once per group of KRY_GROUP basis vectors
 *   and reduces with a fixed grid and a fixed tree, so every GMRES coefficient is reproducible.
 */
#include "krylov.hpp"

namespace fvhip {

constexpr int KRY_BLOCKS = 512;   ///< partial sums per dot product (= ode.hip's ODE_RED_BLOCKS)
constexpr int KRY_GROUP = 4;      ///< dot products per block row of the multi-dot

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

/// y = B x for a row-major 4x4 block
__device__ __forceinline__ void blk_mv(const double* __restrict__ B, const double4 x, double* y)
{
	const double4* b4 = reinterpret_cast<const double4*>(B);
	#pragma unroll
	for(int i = 0; i < 4; i++) {
		const double4 r = b4[i];
		y[i] = r.x*x.x + r.y*x.y + r.z*x.z + r.w*x.w;
	}
}

// -------------------------------------------------------------------------------------------------
// point-block Jacobi
// -------------------------------------------------------------------------------------------------
/// b = a^-1 for a 4x4 block (Gauss-Jordan, partial pivoting by selects: static register indices only);
/// a is destroyed
__device__ __forceinline__ void inv4(double (&a)[4][4], double (&b)[4][4])
{
	#pragma unroll
	for(int i = 0; i < 4; i++)
		#pragma unroll
		for(int j = 0; j < 4; j++) b[i][j] = i == j ? 1.0 : 0.0;
	#pragma unroll
	for(int k = 0; k < 4; k++) {
		// bring the largest |a[i][k]|, i >= k, to row k with selects (static register indices only)
		#pragma unroll
		for(int i = k+1; i < 4; i++) {
			const bool sw = fabs(a[i][k]) > fabs(a[k][k]);
			#pragma unroll
			for(int j = 0; j < 4; j++) {
				const double ta = a[k][j], tb = b[k][j];
				a[k][j] = sw ? a[i][j] : ta; a[i][j] = sw ? ta : a[i][j];
				b[k][j] = sw ? b[i][j] : tb; b[i][j] = sw ? tb : b[i][j];
			}
		}
		const double piv = 1.0/a[k][k];
		#pragma unroll
		for(int j = 0; j < 4; j++) { a[k][j] *= piv; b[k][j] *= piv; }
		#pragma unroll
		for(int i = 0; i < 4; i++) {
			if(i == k) continue;
			const double f = a[i][k];
			#pragma unroll
			for(int j = 0; j < 4; j++) { a[i][j] -= f*a[k][j]; b[i][j] -= f*b[k][j]; }
		}
	}
}

__device__ __forceinline__ void ld16(const double* __restrict__ p, double (&a)[4][4])
{
	const double4* d4 = reinterpret_cast<const double4*>(p);
	#pragma unroll
	for(int i = 0; i < 4; i++) { const double4 v = d4[i]; a[i][0] = v.x; a[i][1] = v.y; a[i][2] = v.z; a[i][3] = v.w; }
}

__device__ __forceinline__ void st16(double* __restrict__ p, const double (&a)[4][4])
{
	double4* o = reinterpret_cast<double4*>(p);
	#pragma unroll
	for(int i = 0; i < 4; i++) o[i] = make_double4(a[i][0], a[i][1], a[i][2], a[i][3]);
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
	for(long long i = blockIdx.x*256LL + threadIdx.x; i < n; i += 256LL*gridDim.x) {
		const double wi = w[i];
		#pragma unroll
		for(int q = 0; q < KRY_GROUP; q++) if(j0 + q < kt) acc[q] += vp[q][i]*wi;
	}
	block_sum<KRY_GROUP>(acc, part + static_cast<size_t>(j0)*KRY_BLOCKS + blockIdx.x, KRY_BLOCKS);
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

__global__ __launch_bounds__(256)
void k_maxpy(long long n, int k, const double* __restrict__ V, long long ld, const double* __restrict__ h,
             double* __restrict__ w)
{
	const long long i = blockIdx.x*256LL + threadIdx.x;
	if(i >= n) return;
	double s = 0.0;
	for(int j = 0; j < k; j++) s += h[j]*V[j*ld + i];
	w[i] -= s;
}

__global__ __launch_bounds__(256)
void k_lincomb(long long n, int k, const double* __restrict__ V, long long ld, const double* __restrict__ c,
               double* __restrict__ out)
{
	const long long i = blockIdx.x*256LL + threadIdx.x;
	if(i >= n) return;
	double s = 0.0;
	for(int j = 0; j < k; j++) s += c[j]*V[j*ld + i];
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

/// block-Thomas factorisation per line (one thread per line): dinvp_k = (D_k - A[k][k-1] dinvp_{k-1} A[k-1][k])^-1
__global__ __launch_bounds__(64)
void k_line_factor(int nlines, const int* __restrict__ lstart, const int* __restrict__ lcell, const int* __restrict__ lface,
                   const double* __restrict__ diag, const double* __restrict__ lower, const double* __restrict__ upper,
                   double* __restrict__ dinvp, int first)
{
	const int l = first + static_cast<int>(blockIdx.x*blockDim.x + threadIdx.x);
	if(l >= nlines) return;
	const int k0 = lstart[l], k1 = lstart[l+1];
	double prev[4][4];             // dinvp of the previous line cell
	for(int k = k0; k < k1; k++) {
		const int c = lcell[k];
		double a[4][4], b[4][4];
		ld16(diag + 16*static_cast<size_t>(c), a);
		if(k > k0) {
			const int fc = lface[k];
			double L[4][4], U[4][4], t[4][4];
			ld16(blk_cp(fc, lower, upper), L);
			ld16(blk_pc(fc, lower, upper), U);
			// t = prev * U ; a -= L * t
			#pragma unroll
			for(int i = 0; i < 4; i++)
				#pragma unroll
				for(int j = 0; j < 4; j++) t[i][j] = prev[i][0]*U[0][j] + prev[i][1]*U[1][j] + prev[i][2]*U[2][j] + prev[i][3]*U[3][j];
			#pragma unroll
			for(int i = 0; i < 4; i++)
				#pragma unroll
				for(int j = 0; j < 4; j++) a[i][j] -= L[i][0]*t[0][j] + L[i][1]*t[1][j] + L[i][2]*t[2][j] + L[i][3]*t[3][j];
		}
		inv4(a, b);
		st16(dinvp + 16*static_cast<size_t>(c), b);
		#pragma unroll
		for(int i = 0; i < 4; i++)
			#pragma unroll
			for(int j = 0; j < 4; j++) prev[i][j] = b[i][j];
	}
}

/// z = Lines^-1 v per line (one thread per line): forward g_k = dinvp_k (v_k - A[k][k-1] g_{k-1}) into z,
/// then backward z_k = g_k - dinvp_k A[k][k+1] z_{k+1}
__global__ __launch_bounds__(64)
void k_line_solve(int nlines, const int* __restrict__ lstart, const int* __restrict__ lcell, const int* __restrict__ lface,
                  const double* __restrict__ dinvp, const double* __restrict__ lower, const double* __restrict__ upper,
                  const double* __restrict__ v, double* __restrict__ z, int first)
{
	const int l = first + static_cast<int>(blockIdx.x*blockDim.x + threadIdx.x);
	if(l >= nlines) return;
	const int k0 = lstart[l], k1 = lstart[l+1];
	double4 g = make_double4(0, 0, 0, 0);
	for(int k = k0; k < k1; k++) {
		const int c = lcell[k];
		double4 r = reinterpret_cast<const double4*>(v)[c];
		if(k > k0) {
			double t[4];
			blk_mv(blk_cp(lface[k], lower, upper), g, t);
			r.x -= t[0]; r.y -= t[1]; r.z -= t[2]; r.w -= t[3];
		}
		double y[4];
		blk_mv(dinvp + 16*static_cast<size_t>(c), r, y);
		g = make_double4(y[0], y[1], y[2], y[3]);
		reinterpret_cast<double4*>(z)[c] = g;
	}
	double4 x = g;                 // z of the last cell
	for(int k = k1 - 2; k >= k0; k--) {
		const int c = lcell[k];
		double t[4], y[4];
		blk_mv(blk_pc(lface[k+1], lower, upper), x, t);
		blk_mv(dinvp + 16*static_cast<size_t>(c), make_double4(t[0], t[1], t[2], t[3]), y);
		const double4 gk = reinterpret_cast<const double4*>(z)[c];
		x = make_double4(gk.x - y[0], gk.y - y[1], gk.z - y[2], gk.w - y[3]);
		reinterpret_cast<double4*>(z)[c] = x;
	}
}

/// Wave-per-line forms of the two kernels above (one 64-lane workgroup per line): the lanes stage 64
/// cells' blocks of the line in LDS with independent loads, then one lane runs the recurrence over them
/// from LDS and the lanes write the results back. The recurrence is the same arithmetic in the same
/// order, so the results are bitwise those of the one-thread-per-line kernels; what goes is the global
/// load latency inside the sequential chain (a line of a few hundred cells walked by one thread paid
/// one memory round trip per cell).
constexpr int LCH = 64;

__global__ __launch_bounds__(64)
void k_line_factor_w(int nlines, const int* __restrict__ lstart, const int* __restrict__ lcell, const int* __restrict__ lface,
                     const double* __restrict__ diag, const double* __restrict__ lower, const double* __restrict__ upper,
                     double* __restrict__ dinvp)
{
	__shared__ __attribute__((aligned(32))) double sD[LCH][16], sL[LCH][16], sU[LCH][16];
	__shared__ int sc[LCH];
	const int l = blockIdx.x, j = threadIdx.x;
	if(l >= nlines) return;
	const int k0 = lstart[l], k1 = lstart[l+1];
	double prev[4][4];
	for(int base = k0; base < k1; base += LCH) {
		const int n = min(LCH, k1 - base);
		__syncthreads();                         // the previous chunk is written back
		if(j < n) {
			const int k = base + j, c = lcell[k];
			sc[j] = c;
			for(int e = 0; e < 16; e++) sD[j][e] = diag[16*static_cast<size_t>(c) + e];
			if(k > k0) {
				const double* L = blk_cp(lface[k], lower, upper);
				const double* U = blk_pc(lface[k], lower, upper);
				for(int e = 0; e < 16; e++) { sL[j][e] = L[e]; sU[j][e] = U[e]; }
			}
		}
		__syncthreads();
		if(j == 0) {
			for(int i = 0; i < n; i++) {
				double a[4][4], b[4][4];
				#pragma unroll
				for(int r = 0; r < 4; r++)
					#pragma unroll
					for(int q = 0; q < 4; q++) a[r][q] = sD[i][4*r+q];
				if(base + i > k0) {
					double t[4][4];
					#pragma unroll
					for(int r = 0; r < 4; r++)
						#pragma unroll
						for(int q = 0; q < 4; q++)
							t[r][q] = prev[r][0]*sU[i][q] + prev[r][1]*sU[i][4+q] + prev[r][2]*sU[i][8+q] + prev[r][3]*sU[i][12+q];
					#pragma unroll
					for(int r = 0; r < 4; r++)
						#pragma unroll
						for(int q = 0; q < 4; q++)
							a[r][q] -= sL[i][4*r]*t[0][q] + sL[i][4*r+1]*t[1][q] + sL[i][4*r+2]*t[2][q] + sL[i][4*r+3]*t[3][q];
				}
				inv4(a, b);
				#pragma unroll
				for(int r = 0; r < 4; r++)
					#pragma unroll
					for(int q = 0; q < 4; q++) { sD[i][4*r+q] = b[r][q]; prev[r][q] = b[r][q]; }
			}
		}
		__syncthreads();
		if(j < n) for(int e = 0; e < 16; e++) dinvp[16*static_cast<size_t>(sc[j]) + e] = sD[j][e];
	}
}

__global__ __launch_bounds__(64)
void k_line_solve_w(int nlines, const int* __restrict__ lstart, const int* __restrict__ lcell, const int* __restrict__ lface,
                    const double* __restrict__ dinvp, const double* __restrict__ lower, const double* __restrict__ upper,
                    const double* __restrict__ v, double* __restrict__ z)
{
	__shared__ __attribute__((aligned(32))) double sD[LCH][16], sB[LCH][16], sv[LCH][4];
	__shared__ int sc[LCH];
	const int l = blockIdx.x, j = threadIdx.x;
	if(l >= nlines) return;
	const int k0 = lstart[l], k1 = lstart[l+1];
	double4 g = make_double4(0, 0, 0, 0);
	// forward: g_k = dinvp_k (v_k - A[k][k-1] g_{k-1})
	for(int base = k0; base < k1; base += LCH) {
		const int n = min(LCH, k1 - base);
		__syncthreads();
		if(j < n) {
			const int k = base + j, c = lcell[k];
			sc[j] = c;
			for(int e = 0; e < 16; e++) sD[j][e] = dinvp[16*static_cast<size_t>(c) + e];
			for(int e = 0; e < 4; e++) sv[j][e] = v[4*static_cast<size_t>(c) + e];
			if(k > k0) { const double* L = blk_cp(lface[k], lower, upper); for(int e = 0; e < 16; e++) sB[j][e] = L[e]; }
		}
		__syncthreads();
		if(j == 0) {
			for(int i = 0; i < n; i++) {
				double4 r = make_double4(sv[i][0], sv[i][1], sv[i][2], sv[i][3]);
				if(base + i > k0) {
					double t[4];
					blk_mv(sB[i], g, t);
					r.x -= t[0]; r.y -= t[1]; r.z -= t[2]; r.w -= t[3];
				}
				double y[4];
				blk_mv(sD[i], r, y);
				g = make_double4(y[0], y[1], y[2], y[3]);
				sv[i][0] = y[0]; sv[i][1] = y[1]; sv[i][2] = y[2]; sv[i][3] = y[3];
			}
		}
		__syncthreads();
		if(j < n) for(int e = 0; e < 4; e++) z[4*static_cast<size_t>(sc[j]) + e] = sv[j][e];
	}
	// backward: z_k = g_k - dinvp_k A[k][k+1] z_{k+1}, chunks from the end (the last cell keeps g)
	double4 x = g;
	const int kl = k1 - 2;                      // last cell the backward pass updates
	for(int top = kl; top >= k0; top -= LCH) {
		const int n = min(LCH, top - k0 + 1);   // cells top, top-1, ..., top-n+1
		__syncthreads();
		if(j < n) {
			const int k = top - j, c = lcell[k];
			sc[j] = c;
			for(int e = 0; e < 16; e++) sD[j][e] = dinvp[16*static_cast<size_t>(c) + e];
			for(int e = 0; e < 4; e++) sv[j][e] = z[4*static_cast<size_t>(c) + e];
			const double* U = blk_pc(lface[k+1], lower, upper);
			for(int e = 0; e < 16; e++) sB[j][e] = U[e];
		}
		__syncthreads();
		if(j == 0) {
			for(int i = 0; i < n; i++) {
				double t[4], y[4];
				blk_mv(sB[i], x, t);
				blk_mv(sD[i], make_double4(t[0], t[1], t[2], t[3]), y);
				x = make_double4(sv[i][0] - y[0], sv[i][1] - y[1], sv[i][2] - y[2], sv[i][3] - y[3]);
				sv[i][0] = x.x; sv[i][1] = x.y; sv[i][2] = x.z; sv[i][3] = x.w;
			}
		}
		__syncthreads();
		if(j < n) for(int e = 0; e < 4; e++) z[4*static_cast<size_t>(sc[j]) + e] = sv[j][e];
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

void launch_line_factor(const LineSet& Ls, const double* diag, const double* lower, const double* upper, double* dinvp,
                        hipStream_t s)
{
	// long lines: a workgroup each; the short rest (same arithmetic, bitwise the same): a thread each
	if(Ls.nlong > 0)
		hipLaunchKernelGGL(k_line_factor_w, dim3(Ls.nlong), dim3(64), 0, s, Ls.nlines, Ls.start, Ls.cell, Ls.face,
		                   diag, lower, upper, dinvp);
	if(Ls.nlines > Ls.nlong)
		hipLaunchKernelGGL(k_line_factor, dim3(nblk(Ls.nlines - Ls.nlong, 64)), dim3(64), 0, s, Ls.nlines, Ls.start,
		                   Ls.cell, Ls.face, diag, lower, upper, dinvp, Ls.nlong);
}

void launch_line_solve(const LineSet& Ls, const double* dinvp, const double* lower, const double* upper, const double* v,
                       double* z, hipStream_t s)
{
	if(Ls.nlong > 0)
		hipLaunchKernelGGL(k_line_solve_w, dim3(Ls.nlong), dim3(64), 0, s, Ls.nlines, Ls.start, Ls.cell, Ls.face,
		                   dinvp, lower, upper, v, z);
	if(Ls.nlines > Ls.nlong)
		hipLaunchKernelGGL(k_line_solve, dim3(nblk(Ls.nlines - Ls.nlong, 64)), dim3(64), 0, s, Ls.nlines, Ls.start,
		                   Ls.cell, Ls.face, dinvp, lower, upper, v, z, Ls.nlong);
}

void launch_add_rows(int n, const double* e, double* z, hipStream_t s)
{
	if(n > 0) hipLaunchKernelGGL(k_add_rows, dim3(nblk(n, 256)), dim3(256), 0, s, n, e, z);
}

void launch_bjac_invert(int n, const double* diag, double* dinv, hipStream_t s)
{ if(n > 0) k_bjac_invert<<<nblk(n,256), 256, 0, s>>>(n, diag, dinv); }
void launch_bjac_apply(int n, const double* dinv, const double* x, double* y, hipStream_t s)
{ if(n > 0) k_bjac_apply<double><<<nblk(n,256), 256, 0, s>>>(n, dinv, x, y); }
void launch_bjac_apply(int n, const float* dinv, const double* x, double* y, hipStream_t s)
{ if(n > 0) k_bjac_apply<float><<<nblk(n,256), 256, 0, s>>>(n, dinv, x, y); }
void launch_to_single(long long n, const double* a, float* b, hipStream_t s)
{ if(n > 0) k_to_single<<<nblk(n/4,256), 256, 0, s>>>(n, a, b); }
void launch_bjac_correct(int n, const double* dinv, const double* b, const double* y, double* z, hipStream_t s)
{ if(n > 0) k_bjac_correct<<<nblk(n,256), 256, 0, s>>>(n, dinv, b, y, z); }

size_t kry_scratch(int k)
{
	return static_cast<size_t>(KRY_BLOCKS)*static_cast<size_t>((k + KRY_GROUP)/KRY_GROUP*KRY_GROUP);
}

void launch_mdot(long long n, int k, const double* V, long long ld, const double* w, bool self,
                 double* part, double* out, hipStream_t s)
{
	const int kt = k + (self ? 1 : 0);
	if(kt <= 0) return;
	k_mdot_partial<<<dim3(KRY_BLOCKS, (kt + KRY_GROUP - 1)/KRY_GROUP), 256, 0, s>>>(n, k, kt, V, ld, w, part);
	k_sum_partials<<<kt, 256, 0, s>>>(KRY_BLOCKS, part, out);
}

void launch_maxpy(long long n, int k, const double* V, long long ld, const double* h, double* w, hipStream_t s)
{ if(n > 0 && k > 0) k_maxpy<<<nblk(n,256), 256, 0, s>>>(n, k, V, ld, h, w); }
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
