/** \file blk4.hpp
 * \brief Device helpers on row-major 4x4 fp64 blocks shared by the preconditioner kernels (krylov.hip,
 *   amg.hip): block-vector product, inverse (Gauss-Jordan with pivoting by selects), loads and stores.
 */
#ifndef FVHIP_BLK4_HPP
#define FVHIP_BLK4_HPP

#include <hip/hip_runtime.h>

namespace fvhip {

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

/// c = a b for row-major 4x4 blocks
__device__ __forceinline__ void mm4(const double (&a)[4][4], const double (&b)[4][4], double (&c)[4][4])
{
	#pragma unroll
	for(int i = 0; i < 4; i++)
		#pragma unroll
		for(int j = 0; j < 4; j++) c[i][j] = a[i][0]*b[0][j] + a[i][1]*b[1][j] + a[i][2]*b[2][j] + a[i][3]*b[3][j];
}

}
#endif
