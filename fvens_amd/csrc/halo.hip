/** \file halo.hip
 * \brief Ghost-cell exchange helpers: packing the rows of owned cells that neighbour ranks hold as
 *   ghosts into one contiguous send buffer (received rows land directly in the ghost block, which
 *   is contiguous per neighbour), and the primitive conversion of received ghost states.
 *   The reference moves the same data with PETSc ghosted-Vec scatters (alinalg.cpp:17-29,
 *   flow_spatial.cpp:711-729) and its L2TraceVector (tracevector.cpp:213-340).
 */
#include "halo.hpp"

namespace fvhip {

__global__ void __launch_bounds__(256) k_pack_rows(const int* __restrict__ idx, int n, const double* __restrict__ src,
                                                   int width, double* __restrict__ dst)
{
	const long long i = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	if(i >= static_cast<long long>(n)*width) return;
	const int r = static_cast<int>(i / width), k = static_cast<int>(i % width);
	dst[i] = src[static_cast<size_t>(idx[r])*width + k];
}

__global__ void __launch_bounds__(256) k_cons2prim_rows(gd::Gas G, const double* __restrict__ u, double* __restrict__ up,
                                                        int first, int count)
{
	const int i = blockIdx.x*blockDim.x + threadIdx.x;
	if(i >= count) return;
	const int c = first + i;
	const double4 v = reinterpret_cast<const double4*>(u)[c];
	const double a[4] = {v.x, v.y, v.z, v.w};
	double b[4];
	gd::cons2prim(G, a, b);
	reinterpret_cast<double4*>(up)[c] = make_double4(b[0], b[1], b[2], b[3]);
}

__global__ void __launch_bounds__(256) k_unpack_rows(const int* __restrict__ idx, int n, const double* __restrict__ src,
                                                     int width, double* __restrict__ dst)
{
	const long long i = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	if(i >= static_cast<long long>(n)*width) return;
	const int r = static_cast<int>(i / width), k = static_cast<int>(i % width);
	dst[static_cast<size_t>(idx[r])*width + k] = src[i];
}

void launch_unpack_rows(const int* idx, int n, const double* src, int width, double* dst, hipStream_t s)
{
	const long long tot = static_cast<long long>(n)*width;
	if(tot > 0) k_unpack_rows<<<static_cast<int>((tot + 255)/256), 256, 0, s>>>(idx, n, src, width, dst);
}

void launch_pack_rows(const int* idx, int n, const double* src, int width, double* dst, hipStream_t s)
{
	const long long tot = static_cast<long long>(n)*width;
	if(tot > 0) k_pack_rows<<<static_cast<int>((tot + 255)/256), 256, 0, s>>>(idx, n, src, width, dst);
}

void launch_cons2prim_rows(const gd::Gas& G, const double* u, double* up, int first, int count, hipStream_t s)
{
	if(count > 0) k_cons2prim_rows<<<(count + 255)/256, 256, 0, s>>>(G, u, up, first, count);
}

}
