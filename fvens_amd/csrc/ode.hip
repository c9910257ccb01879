/** \file ode.hip
 * \brief Device-resident explicit pseudo-time stepping: SteadyForwardEulerSolver::solve
 *   (aodesolver.cpp:170-240) with the state, residual and time steps kept in HBM.
 *   Update u += cfl*dtm*(1/area)*r in the reference's operation order (:204-214), residual
 *   norm sqrt(sum r_energy^2 area) (:216-223) reduced in a fixed order (two stages).
 */
#include "ode.hpp"

namespace fvhip {

constexpr int ODE_RED_BLOCKS = 512;

__global__ void __launch_bounds__(256) k_fe_update(int n, const double* __restrict__ r, const double* __restrict__ dtm,
                                                   const double* __restrict__ area, double cfl, double* __restrict__ u)
{
	const int e = blockIdx.x*blockDim.x + threadIdx.x;
	if(e >= n) return;
	const double a = cfl*dtm[e] * 1.0/area[e];
	const double4 rr = reinterpret_cast<const double4*>(r)[e];
	double4 uu = reinterpret_cast<double4*>(u)[e];
	uu.x += a*rr.x; uu.y += a*rr.y; uu.z += a*rr.z; uu.w += a*rr.w;
	reinterpret_cast<double4*>(u)[e] = uu;
}

__global__ void __launch_bounds__(256) k_resnorm_partial(int n, const double* __restrict__ r, const double* __restrict__ area,
                                                         double* __restrict__ part)
{
	__shared__ double s[256];
	double acc = 0;
	for(int e = blockIdx.x*256 + threadIdx.x; e < n; e += 256*gridDim.x) acc += r[4*static_cast<size_t>(e)+3]*r[4*static_cast<size_t>(e)+3]*area[e];
	s[threadIdx.x] = acc;
	__syncthreads();
	for(int w = 128; w > 0; w >>= 1) {
		if(threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
		__syncthreads();
	}
	if(threadIdx.x == 0) part[blockIdx.x] = s[0];
}

__global__ void __launch_bounds__(256) k_resnorm_final(int np, const double* __restrict__ part, double* __restrict__ out)
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
	if(threadIdx.x == 0) out[0] = sqrt(s[0]);
}

/// one TVD Runge-Kutta stage (TVDRKSolver::solve, aodesolver.cpp:735-744) as written there:
/// ustage = c0*u + c1*ustage - c2*dtmin*cfl/area*r, with sc = (c2*dtmin)*cfl formed on the host
__global__ void __launch_bounds__(256) k_tvdrk_stage(int n, double c0, double c1, double sc, const double* __restrict__ area,
                                                     const double* __restrict__ r, const double* __restrict__ u,
                                                     double* __restrict__ us)
{
	const int e = blockIdx.x*blockDim.x + threadIdx.x;
	if(e >= n) return;
	const double t = sc/area[e];
	const double4 rr = reinterpret_cast<const double4*>(r)[e], uu = reinterpret_cast<const double4*>(u)[e];
	double4 ss = reinterpret_cast<double4*>(us)[e];
	ss.x = c0*uu.x + c1*ss.x - t*rr.x;
	ss.y = c0*uu.y + c1*ss.y - t*rr.y;
	ss.z = c0*uu.z + c1*ss.z - t*rr.z;
	ss.w = c0*uu.w + c1*ss.w - t*rr.w;
	reinterpret_cast<double4*>(us)[e] = ss;
}

/// minimum that propagates NaN (fmin skips it): one NaN time step makes the minimum NaN
__device__ __forceinline__ double nan_min(double a, double b) { return a != a ? a : (b != b ? b : fmin(a, b)); }

/// minimum over cells (order-free), two stages; a NaN anywhere gives -inf (finite values and +inf
/// otherwise as fmin), so the divergence check fires for it and ncclMin across ranks carries it
__global__ void __launch_bounds__(256) k_min_partial(int n, const double* __restrict__ x, double* __restrict__ part)
{
	__shared__ double s[256];
	double m = INFINITY;
	for(int e = blockIdx.x*256 + threadIdx.x; e < n; e += 256*gridDim.x) m = nan_min(m, x[e]);
	s[threadIdx.x] = m;
	__syncthreads();
	for(int w = 128; w > 0; w >>= 1) {
		if(threadIdx.x < w) s[threadIdx.x] = nan_min(s[threadIdx.x], s[threadIdx.x + w]);
		__syncthreads();
	}
	if(threadIdx.x == 0) part[blockIdx.x] = s[0];
}
__global__ void __launch_bounds__(256) k_min_final(int np, const double* __restrict__ part, double* __restrict__ out)
{
	__shared__ double s[256];
	double m = INFINITY;
	for(int i = threadIdx.x; i < np; i += 256) m = nan_min(m, part[i]);
	s[threadIdx.x] = m;
	__syncthreads();
	for(int w = 128; w > 0; w >>= 1) {
		if(threadIdx.x < w) s[threadIdx.x] = nan_min(s[threadIdx.x], s[threadIdx.x + w]);
		__syncthreads();
	}
	if(threadIdx.x == 0) out[0] = s[0] != s[0] ? -INFINITY : s[0];
}

void launch_tvdrk_stage(int n, double c0, double c1, double sc, const double* area, const double* r, const double* u,
                        double* us, hipStream_t s)
{
	if(n > 0) k_tvdrk_stage<<<(n + 255)/256, 256, 0, s>>>(n, c0, c1, sc, area, r, u, us);
}

void launch_min(int n, const double* x, double* part, double* out, hipStream_t s)
{
	k_min_partial<<<ODE_RED_BLOCKS, 256, 0, s>>>(n, x, part);
	k_min_final<<<1, 256, 0, s>>>(ODE_RED_BLOCKS, part, out);
}

void launch_fe_update(int n, const double* r, const double* dtm, const double* area, double cfl, double* u, hipStream_t s)
{
	if(n > 0) k_fe_update<<<(n + 255)/256, 256, 0, s>>>(n, r, dtm, area, cfl, u);
}

void launch_resnorm(int n, const double* r, const double* area, double* part, double* out, hipStream_t s)
{
	k_resnorm_partial<<<ODE_RED_BLOCKS, 256, 0, s>>>(n, r, area, part);
	k_resnorm_final<<<1, 256, 0, s>>>(ODE_RED_BLOCKS, part, out);
}

int resnorm_partials() { return ODE_RED_BLOCKS; }

}
