/** \file surface.hip
 * \brief FlowFV_base::computeSurfaceData (flow_spatial.cpp:130-310) on the device: per wall face the
 *   pressure and skin-friction coefficients and their lift / pressure-drag / friction-drag moments,
 *   summed in the reference's face order.
 *
 * One thread per face of the marker computes (x, y, Cp, Cf) and the four products
 * (Cp n.nw len, Cp n.w len, Cf t.w len, len); one thread then adds them face by face, which is the
 * reference's serial loop order, so the sums are those of a single-rank run bit for bit. The wind
 * direction and free-stream pressure come from the host (std::cos / std::sin, as the reference).
 */
#include "surface.hpp"

namespace fvhip {

using namespace gd;

__global__ __launch_bounds__(256)
void k_surface_faces(SurfaceFaces S, const double* __restrict__ u, const double* __restrict__ grad, Gas G,
                     double pinf, double2 wind, double* __restrict__ faceout, double* __restrict__ contrib)
{
	const int i = blockIdx.x*blockDim.x + threadIdx.x;
	if(i >= S.n) return;
	const int le = S.L[i];
	const double* geo = S.geo + 5*static_cast<size_t>(i);
	const double n[2] = {geo[0], geo[1]};
	const double len = geo[2];
	const double tangf[2] = {n[1], -n[0]};
	double urec[4];
	const double4 uc = reinterpret_cast<const double4*>(u)[le];
	urec[0] = uc.x; urec[1] = uc.y; urec[2] = uc.z; urec[3] = uc.w;
	// Cp = 2 (p - p_inf) (:204)
	const double cp = (pressure_cons(G, urec) - pinf)*2.0;
	// muhat = getViscosityCoeffFromConserved (Sutherland, aphysics_defs.hpp:417-421, :408-413), with
	// IEEE division throughout: inviscid runs carry Reinf = inf, where mu must come out as 0
	const double T = temperature(G, urec[0], pressure_cons(G, urec));
	const double muhat = (1.0 + G.sC/G.Tinf)/(T + G.sC/G.Tinf) * pow(T, 1.5) / G.Reinf;
	// velocity gradients from conserved gradients, grad(j, var) = g[var*2 + j] (:232-236)
	const double* g = grad + 8*static_cast<size_t>(le);
	double gradu[2][2];
	for(int a = 0; a < 2; a++)
		for(int b = 0; b < 2; b++)
			gradu[a][b] = (g[(a+1)*2+b]*urec[0] - urec[a+1]*g[b]) / (urec[0]*urec[0]);
	double force[2];
	for(int a = 0; a < 2; a++) {
		force[a] = 0;
		for(int b = 0; b < 2; b++) force[a] += (gradu[a][b] + gradu[b][a])*n[b];
	}
	const double tauw = muhat*dot2(force, tangf);
	const double cf = 2*tauw;
	const double w[2] = {wind.x, wind.y}, nw[2] = {-wind.y, wind.x};
	const double ndotw = dot2(n, w), ndotnw = dot2(n, nw), tdotw = dot2(tangf, w);
	double* fo = faceout + 4*static_cast<size_t>(i);
	fo[0] = geo[3]; fo[1] = geo[4]; fo[2] = cp; fo[3] = cf;
	double* c = contrib + 4*static_cast<size_t>(i);
	c[0] = cp*ndotnw*len; c[1] = cp*ndotw*len; c[2] = cf*tdotw*len; c[3] = len;
}

/// sums[0..3] = (Cl, Cdp, Cdf, total length) added face by face in order
__global__ void k_surface_sum(int n, const double* __restrict__ contrib, double* __restrict__ sums)
{
	if(threadIdx.x != 0 || blockIdx.x != 0) return;
	double cl = 0, cdp = 0, cdf = 0, area = 0;
	for(int i = 0; i < n; i++) {
		const double* c = contrib + 4*static_cast<size_t>(i);
		area += c[3];
		cl += c[0];
		cdp += c[1];
		cdf += c[2];
	}
	sums[0] = cl; sums[1] = cdp; sums[2] = cdf; sums[3] = area;
}

/// FlowOutput::compute_entropy_cell (aoutput.cpp:28-62): (s - s_inf)^2/s_inf^2 * area per cell,
/// s = p/rho^gamma (getEntropyFromConserved, aphysics_defs.hpp:204-207); each block sums its 256 cells by
/// a fixed tree, k_entropy_sum adds the block sums in block order (deterministic; the reference's is an
/// OpenMP reduction, so this is a tolerance-level match)
__global__ __launch_bounds__(256)
void k_entropy_partial(int N, const double* __restrict__ u, const double* __restrict__ area, Gas G, double sinf,
                       double* __restrict__ part)
{
	__shared__ double red[256];
	const int i = blockIdx.x*256 + threadIdx.x;
	double e = 0.0;
	if(i < N) {
		double uc[4];
		const double4 v = reinterpret_cast<const double4*>(u)[i];
		uc[0] = v.x; uc[1] = v.y; uc[2] = v.z; uc[3] = v.w;
		const double s = pressure_cons(G, uc)/pow(uc[0], G.g);
		const double serr = (s - sinf)/sinf;
		e = serr*serr*area[i];
	}
	red[threadIdx.x] = e;
	__syncthreads();
	for(int w = 128; w > 0; w >>= 1) {
		if(static_cast<int>(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
		__syncthreads();
	}
	if(threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void k_entropy_sum(int nb, const double* __restrict__ part, double* __restrict__ out)
{
	if(threadIdx.x != 0 || blockIdx.x != 0) return;
	double s = 0;
	for(int b = 0; b < nb; b++) s += part[b];
	out[0] = s;
}

int entropy_partials(int N) { return (N + 255)/256; }

void launch_entropy(int N, const double* u, const double* area, const Gas& G, double sinf, double* part,
                    double* out, hipStream_t s)
{
	const int nb = entropy_partials(N);
	if(nb > 0) hipLaunchKernelGGL(k_entropy_partial, dim3(nb), dim3(256), 0, s, N, u, area, G, sinf, part);
	hipLaunchKernelGGL(k_entropy_sum, dim3(1), dim3(64), 0, s, nb, part, out);
}

void launch_surface(const SurfaceFaces& S, const double* u, const double* grad, const Gas& G, double pinf,
                    double wx, double wy, double* faceout, double* contrib, double* sums, hipStream_t s)
{
	if(S.n > 0)
		hipLaunchKernelGGL(k_surface_faces, dim3((S.n + 255)/256), dim3(256), 0, s, S, u, grad, G, pinf,
		                   make_double2(wx, wy), faceout, contrib);
	hipLaunchKernelGGL(k_surface_sum, dim3(1), dim3(64), 0, s, S.n, contrib, sums);
}

}
