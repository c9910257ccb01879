/** \file amg.hip
 * \brief Device kernels of the aggregation multigrid preconditioner (amg.hpp). Four lanes per block row,
 *   lane i holding row i of each 4x4 block (one 32-byte row load per lane, 128 contiguous bytes per block
 *   over the four lanes), every sum over a fixed, host-built list in ascending order: deterministic, no
 *   atomics. All of them move each block once per call: HBM-bound.
 */
#include "amg.hpp"
#include "blk4.hpp"

namespace fvhip {

static inline int nblk(long long n, int b) { return static_cast<int>((n + b - 1)/b); }

__device__ __forceinline__ const double* fine_block(int src, int nfine, int nif, const double* __restrict__ diag,
                                                    const double* __restrict__ lower, const double* __restrict__ upper)
{
	if(src < nfine) return diag + 16*static_cast<size_t>(src);
	src -= nfine;
	if(src < nif) return lower + 16*static_cast<size_t>(src);
	return upper + 16*static_cast<size_t>(src - nif);
}

/// coarse block k, row i: the sum of row i of the listed blocks (ascending list)
template <bool FINE>
__global__ __launch_bounds__(256)
void k_amg_galerkin(int nnz, const int* __restrict__ cstart, const int* __restrict__ csrc, int nfine, int nif,
                    const double* __restrict__ diag, const double* __restrict__ lower, const double* __restrict__ upper,
                    double* __restrict__ val)
{
	const long long g = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	const int k = static_cast<int>(g >> 2), i = static_cast<int>(g & 3);
	if(k >= nnz) return;
	double4 acc = make_double4(0.0, 0.0, 0.0, 0.0);
	for(int c = cstart[k]; c < cstart[k+1]; c++) {
		const double* B = FINE ? fine_block(csrc[c], nfine, nif, diag, lower, upper) : diag + 16*static_cast<size_t>(csrc[c]);
		const double4 r = reinterpret_cast<const double4*>(B)[i];
		acc.x += r.x; acc.y += r.y; acc.z += r.z; acc.w += r.w;
	}
	reinterpret_cast<double4*>(val + 16*static_cast<size_t>(k))[i] = acc;
}

__global__ __launch_bounds__(256)
void k_amg_invert(int n, const int* __restrict__ dpos, const double* __restrict__ val, double* __restrict__ dinv)
{
	const int r = blockIdx.x*blockDim.x + threadIdx.x;
	if(r >= n) return;
	double a[4][4], b[4][4];
	ld16(val + 16*static_cast<size_t>(dpos[r]), a);
	inv4(a, b);
	st16(dinv + 16*static_cast<size_t>(r), b);
}

__global__ __launch_bounds__(256)
void k_amg_restrict(int n, const int* __restrict__ mstart, const int* __restrict__ members,
                    const double* __restrict__ rf, double* __restrict__ b)
{
	const long long g = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	const int a = static_cast<int>(g >> 2), v = static_cast<int>(g & 3);
	if(a >= n) return;
	double s = 0.0;
	for(int m = mstart[a]; m < mstart[a+1]; m++) s += rf[4*static_cast<size_t>(members[m]) + v];
	b[4*static_cast<size_t>(a) + v] = s;
}

__global__ __launch_bounds__(256)
void k_amg_prolong(int nfine, const int* __restrict__ agg, const double* __restrict__ x, double* __restrict__ xf)
{
	const long long g = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	const int i = static_cast<int>(g >> 2), v = static_cast<int>(g & 3);
	if(i >= nfine) return;
	xf[4*static_cast<size_t>(i) + v] += x[4*static_cast<size_t>(agg[i]) + v];
}

/// row r, lane i: r_i = b_i - sum_k (A_k x_col(k))_i, k ascending
__global__ __launch_bounds__(256)
void k_amg_residual(int n, const int* __restrict__ rowptr, const int* __restrict__ col, const double* __restrict__ val,
                    const double* __restrict__ x, const double* __restrict__ b, double* __restrict__ r)
{
	const long long g = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	const int row = static_cast<int>(g >> 2), i = static_cast<int>(g & 3);
	if(row >= n) return;
	const double4* x4 = reinterpret_cast<const double4*>(x);
	double acc = b[4*static_cast<size_t>(row) + i];
	for(int k = rowptr[row]; k < rowptr[row+1]; k++) {
		const double4 a = reinterpret_cast<const double4*>(val + 16*static_cast<size_t>(k))[i];
		const double4 xv = x4[col[k]];
		acc -= a.x*xv.x + a.y*xv.y + a.z*xv.z + a.w*xv.w;
	}
	r[4*static_cast<size_t>(row) + i] = acc;
}

/// the listed rows (one colour: no two share a nonzero), lane i: s_i = b_i - sum_{k != diag} (A_k x)_i, then
/// x_row = dinv_row s with s gathered from the row's four lanes
__global__ __launch_bounds__(256)
void k_amg_gs(int cnt, const int* __restrict__ cells, const int* __restrict__ rowptr, const int* __restrict__ col,
              const int* __restrict__ dpos, const double* __restrict__ val, const double* __restrict__ dinv,
              const double* __restrict__ b, double* x)
{
	const long long g = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	const int t = static_cast<int>(g >> 2), i = static_cast<int>(g & 3);
	const bool live = t < cnt;
	const int row = cells[live ? t : cnt - 1];          // lanes past the end compute a copy and store nothing
	const double4* x4 = reinterpret_cast<const double4*>(x);
	double acc = b[4*static_cast<size_t>(row) + i];
	const int kd = dpos[row];
	for(int k = rowptr[row]; k < rowptr[row+1]; k++) {
		if(k == kd) continue;
		const double4 a = reinterpret_cast<const double4*>(val + 16*static_cast<size_t>(k))[i];
		const double4 xv = x4[col[k]];
		acc -= a.x*xv.x + a.y*xv.y + a.z*xv.z + a.w*xv.w;
	}
	const double4 s = make_double4(__shfl(acc, 0, 4), __shfl(acc, 1, 4), __shfl(acc, 2, 4), __shfl(acc, 3, 4));
	const double4 d = reinterpret_cast<const double4*>(dinv + 16*static_cast<size_t>(row))[i];
	const double o = d.x*s.x + d.y*s.y + d.z*s.z + d.w*s.w;
	if(live) x[4*static_cast<size_t>(row) + i] = o;
}

/// one workgroup of 1024 threads: every sweep, every colour, 256 rows at a time (4 lanes a row), a barrier
/// after each colour; the iterate lives in LDS for the whole call (the colour-to-colour chain waits on LDS,
/// not on L2 round trips), read from / written back to x at the ends
__global__ __launch_bounds__(1024)
void k_amg_gs_block(int n, int ncol, const int* __restrict__ cstart, const int* __restrict__ cells,
                    const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ dpos,
                    const double* __restrict__ val, const double* __restrict__ dinv, const double* __restrict__ b,
                    double* xg, int sweeps, int fwd, int alternate, int zero)
{
	extern __shared__ __attribute__((aligned(16))) double x[];
	const int t = static_cast<int>(threadIdx.x), i = t & 3;
	for(int k = t; k < 4*n; k += 1024) x[k] = zero ? 0.0 : xg[k];
	__syncthreads();
	const double4* x4 = reinterpret_cast<const double4*>(x);
	for(int sw = 0; sw < sweeps; sw++) {
		const bool f = alternate ? (sw % 2 == 0) : (fwd != 0);
		for(int qq = 0; qq < ncol; qq++) {
			const int q = f ? qq : ncol - 1 - qq;
			const int b0 = cstart[q], cnt = cstart[q+1] - b0;
			for(int r0 = 0; r0 < cnt; r0 += 256) {
				const int rr = r0 + (t >> 2);
				const bool live = rr < cnt;
				const int row = cells[b0 + (live ? rr : cnt - 1)];
				double acc = b[4*static_cast<size_t>(row) + i];
				const int kd = dpos[row];
				for(int k = rowptr[row]; k < rowptr[row+1]; k++) {
					if(k == kd) continue;
					const double4 a = reinterpret_cast<const double4*>(val + 16*static_cast<size_t>(k))[i];
					const double4 xv = x4[col[k]];
					acc -= a.x*xv.x + a.y*xv.y + a.z*xv.z + a.w*xv.w;
				}
				const double4 s = make_double4(__shfl(acc, 0, 4), __shfl(acc, 1, 4), __shfl(acc, 2, 4), __shfl(acc, 3, 4));
				const double4 d = reinterpret_cast<const double4*>(dinv + 16*static_cast<size_t>(row))[i];
				const double o = d.x*s.x + d.y*s.y + d.z*s.z + d.w*s.w;
				if(live) x[4*static_cast<size_t>(row) + i] = o;
			}
			__syncthreads();
		}
	}
	for(int k = t; k < 4*n; k += 1024) xg[k] = x[k];
}

void launch_amg_gs_block(const AmgLevel& L, const double* b, double* x, int sweeps, bool fwd, bool alternate,
                         bool zero, hipStream_t s)
{
	if(L.n <= 0 || L.n > AMG_BLOCK_ROWS) return;
	hipLaunchKernelGGL(k_amg_gs_block, dim3(1), dim3(1024), 32*static_cast<size_t>(L.n), s, L.n, static_cast<int>(L.cstart_colour.size()) - 1,
	                   L.d_cstart_colour, L.cells, L.rowptr, L.col, L.dpos, L.val, L.dinv, b, x, sweeps, fwd ? 1 : 0,
	                   alternate ? 1 : 0, zero ? 1 : 0);
}

void launch_amg_galerkin_fine(const AmgLevel& L, int nfine, int nif, const double* diag, const double* lower,
                              const double* upper, hipStream_t s)
{
	if(L.nnz <= 0) return;
	hipLaunchKernelGGL(k_amg_galerkin<true>, dim3(nblk(4LL*L.nnz, 256)), dim3(256), 0, s, L.nnz, L.cstart, L.csrc,
	                   nfine, nif, diag, lower, upper, L.val);
}

void launch_amg_galerkin(const AmgLevel& L, const double* fval, hipStream_t s)
{
	if(L.nnz <= 0) return;
	hipLaunchKernelGGL(k_amg_galerkin<false>, dim3(nblk(4LL*L.nnz, 256)), dim3(256), 0, s, L.nnz, L.cstart, L.csrc,
	                   0, 0, fval, nullptr, nullptr, L.val);
}

void launch_amg_invert(const AmgLevel& L, hipStream_t s)
{
	if(L.n <= 0) return;
	hipLaunchKernelGGL(k_amg_invert, dim3(nblk(L.n, 256)), dim3(256), 0, s, L.n, L.dpos, L.val, L.dinv);
}

void launch_amg_restrict(const AmgLevel& L, const double* rfine, double* b, hipStream_t s)
{
	if(L.n <= 0) return;
	hipLaunchKernelGGL(k_amg_restrict, dim3(nblk(4LL*L.n, 256)), dim3(256), 0, s, L.n, L.mstart, L.members, rfine, b);
}

void launch_amg_prolong(const AmgLevel& L, const double* x, double* xfine, hipStream_t s)
{
	if(L.nfine <= 0) return;
	hipLaunchKernelGGL(k_amg_prolong, dim3(nblk(4LL*L.nfine, 256)), dim3(256), 0, s, L.nfine, L.agg, x, xfine);
}

void launch_amg_residual(const AmgLevel& L, const double* x, const double* b, double* r, hipStream_t s)
{
	if(L.n <= 0) return;
	hipLaunchKernelGGL(k_amg_residual, dim3(nblk(4LL*L.n, 256)), dim3(256), 0, s, L.n, L.rowptr, L.col, L.val, x, b, r);
}

void launch_amg_gs_colour(const AmgLevel& L, int q, const double* b, double* x, hipStream_t s)
{
	const int b0 = L.cstart_colour[q], cnt = L.cstart_colour[q+1] - b0;
	if(cnt <= 0) return;
	hipLaunchKernelGGL(k_amg_gs, dim3(nblk(4LL*cnt, 256)), dim3(256), 0, s, cnt, L.cells + b0, L.rowptr, L.col,
	                   L.dpos, L.val, L.dinv, b, x);
}

}
