/** \file kernels.hip
 * \brief HIP kernels of the MI355X face sweep (gfx950, wave64).
 *
 * Pipeline of one residual evaluation (FlowFV::compute_residual, flow_spatial.cpp:636-816):
 *   k_prep_cells   conserved -> primitive cell states                     (:697-699)
 *   k_prep_bfaces  boundary ghost state of the cell value, and its primitive (:679-695)
 *   k_grad_*       cell-centred primitive gradients (WLS / Green-Gauss)   (:704-708)
 *   k_limiter/k_weno  per-cell limiter values for limited reconstructions (:720-723)
 *   k_sweep        THE HOT KERNEL: per patch, every touching face is reconstructed, converted,
 *                  given its BC ghost if on the boundary, its inviscid (+viscous) flux and
 *                  spectral radii computed into LDS; then every cell of the patch sums its faces
 *                  from LDS in ascending reference face index and writes -r and the time step
 *                  (:731-812 incl. compute_fluxes :488-563 and compute_max_timestep :565-634).
 * No atomics: the per-cell sum order is the reference's single-thread order, so results are
 * deterministic and, with -ffp-contract=off, bitwise equal to it.
 */
#include "kernels.hpp"
#include "layout.hpp"
#include <algorithm>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>

#ifndef FVHIP_NS
#define FVHIP_NS exact
#endif

namespace fvhip {
namespace FVHIP_NS {

using namespace gd;

/// XCD-aware block -> chunk mapping: the hardware deals consecutive blocks round-robin over the 8
/// XCDs; chunk p = (b%8)*q + b/8 keeps consecutive (Hilbert-adjacent) chunks on one XCD's L2.
/// Launch 8*q blocks; blocks with p >= nchunk return.
__device__ __forceinline__ int xcd_chunk(int nchunk) {
	const int q = (nchunk + 7) >> 3;
	return (static_cast<int>(blockIdx.x) & 7) * q + (static_cast<int>(blockIdx.x) >> 3);
}
static inline int xcd_blocks(long long nchunk) { return static_cast<int>(8*((nchunk + 7)/8)); }

__device__ __forceinline__ void ld4(const double* p, int i, double* o) {
	const double4 v = reinterpret_cast<const double4*>(p)[i];
	o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
__device__ __forceinline__ void st4(double* p, int i, const double* o) {
	reinterpret_cast<double4*>(p)[i] = make_double4(o[0], o[1], o[2], o[3]);
}
__device__ __forceinline__ void ld8(const double* p, int i, double* o) {
	const double4* q = reinterpret_cast<const double4*>(p) + 2*static_cast<size_t>(i);
	const double4 a = q[0], b = q[1];
	o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
__device__ __forceinline__ void st8(double* p, int i, const double* o) {
	double4* q = reinterpret_cast<double4*>(p) + 2*static_cast<size_t>(i);
	q[0] = make_double4(o[0], o[1], o[2], o[3]); q[1] = make_double4(o[4], o[5], o[6], o[7]);
}

/// Boundary ghost state out of line (abc.cpp via gasdyn.hpp ghost_state): boundary faces are rare
/// (~sqrt(N)), but every BC type inlined into the hot kernels' unrolled neighbour loops costs
/// registers, i.e. occupancy, on every cell and face. Arguments and result travel in registers.
__device__ __noinline__ double4 ghost_ool(const Gas G, const BCDev bc, const double4 uinf, const double4 ins,
                                          const double2 nn)
{
	const double ui[4] = {uinf.x, uinf.y, uinf.z, uinf.w}, in[4] = {ins.x, ins.y, ins.z, ins.w};
	const double n[2] = {nn.x, nn.y};
	double gs[4];
	ghost_state(G, bc, ui, in, n, gs);
	return make_double4(gs[0], gs[1], gs[2], gs[3]);
}
__device__ __forceinline__ void ghost(const DevPhys& P, int bc, const double* ins, const double* n, double* gs)
{
	const double4 g = ghost_ool(P.gas, P.bc[bc], make_double4(P.uinf[0], P.uinf[1], P.uinf[2], P.uinf[3]),
	                            make_double4(ins[0], ins[1], ins[2], ins[3]), make_double2(n[0], n[1]));
	gs[0] = g.x; gs[1] = g.y; gs[2] = g.z; gs[3] = g.w;
}

/// an empty register constraint: the value must exist in VGPRs here, so a load producing it cannot be
/// merged with another load behind a pointer select
__device__ __forceinline__ void pin_regs(double& x) { asm("" : "+v"(x)); }

// ------------------------------------------------------------------------------------------------
// preparation
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_prep_cells(int N, Gas G, const double* __restrict__ u, double* __restrict__ up)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= N) return;
	double a[4], b[4];
	ld4(u, c, a);
	cons2prim(G, a, b);
	st4(up, c, b);
}

__global__ void __launch_bounds__(256) k_prep_bfaces(DevMesh M, DevPhys P, const double* __restrict__ u,
                                                     double* __restrict__ ubc, double* __restrict__ ug)
{
	const int f = blockIdx.x*blockDim.x + threadIdx.x;
	if(f >= M.nbface) return;
	double a[4], g[4], p[4];
	ld4(u, M.bf_L[f], a);
	const double2 nn = M.bf_n[f];
	const double n[2] = {nn.x, nn.y};
	ghost_state(P.gas, P.bc[M.bf_bc[f]], P.uinf, a, n, g);
	st4(ubc, f, g);
	cons2prim(P.gas, g, p);
	st4(ug, f, p);
}

// ------------------------------------------------------------------------------------------------
// gradients (agradientschemes.cpp). One thread per cell; the cell's faces are visited in ascending
// reference face index, which is the reference's single-thread accumulation order.
// ------------------------------------------------------------------------------------------------
// WLS (agradientschemes.cpp:322-440). Each face contributes w2*dr*du with dr = rc(L)-rc(R),
// du = u(L)-u(R); computing both differences from this cell's side negates both factors exactly,
// so the product is bitwise the same and no face orientation is needed.
__global__ void __launch_bounds__(256) k_grad_wls(DevMesh M, const double* __restrict__ up,
                                                  const double* __restrict__ ug, double* __restrict__ grad)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= M.nown) return;
	const int N = M.ncell;     // cells incl. ghosts: codes >= N are boundary faces
	const int4 nb4 = M.cell_nbr_fo[c];
	const int nb[4] = {nb4.x, nb4.y, nb4.z, nb4.w};
	const double2 rcc = M.rc[c];
	double uc[4];
	ld4(up, c, uc);
	// issue all neighbour loads before the arithmetic
	double un[4][4];
	double2 rn[4];
	#pragma unroll
	for(int k = 0; k < 4; k++) {
		if(nb[k] < 0) continue;
		if(nb[k] >= N) { rn[k] = M.bf_rcbp[nb[k] - N]; ld4(ug, nb[k] - N, un[k]); }
		else           { rn[k] = M.rc[nb[k]];           ld4(up, nb[k], un[k]); }
	}
	const double4 V = M.wls_V[c];
	double f[8] = {0,0,0,0,0,0,0,0};
	#pragma unroll
	for(int k = 0; k < 4; k++) {
		if(nb[k] < 0) break;
		double w2 = 0;
		w2 += (rcc.x-rn[k].x)*(rcc.x-rn[k].x);
		w2 += (rcc.y-rn[k].y)*(rcc.y-rn[k].y);
		const double dr0 = rcc.x-rn[k].x, dr1 = rcc.y-rn[k].y;
		w2 = div_rn(1.0, w2);
		#pragma unroll
		for(int iv = 0; iv < 4; iv++) {
			const double du = uc[iv] - un[k][iv];
			f[iv*2+0] += w2*dr0*du;
			f[iv*2+1] += w2*dr1*du;
		}
	}
	double g[8];
	#pragma unroll
	for(int iv = 0; iv < 4; iv++) {
		g[iv*2+0] = V.x*f[iv*2+0] + V.y*f[iv*2+1];
		g[iv*2+1] = V.z*f[iv*2+0] + V.w*f[iv*2+1];
	}
	st8(grad, c, g);
}

/// Fused preparation + WLS gradient for the residual path: converts this cell's conserved state
/// (written as up[c]) and its neighbours' (k_prep_cells' cons2prim, bit for bit), builds the ghost
/// states of this cell's boundary faces (k_prep_bfaces; each boundary face has exactly one cell),
/// then the same WLS arithmetic as k_grad_wls. A block owns 256 consecutive (Hilbert-ordered)
/// cells; their primitive states and centres are staged in LDS, so only neighbours outside the
/// block are gathered from global memory.
/// limiter values of one cell (k_limiter's arithmetic): uc its primitive state, g its gradient,
/// un[j] / gp[j] the state across and the centre of its face j (any face order: dmin/dmax and the
/// minimum over faces do not depend on it), nf faces.
/// Venkatakrishnan (limitedlinearreconstruction.cpp:219-246) in fewer instructions, bitwise: 2*dp*dm
/// and 2*dm*dm scale exact products (2 RN(dp dm), 2 RN(dm dm)), so each sum that adds one is an fma with
/// the factor 2, and dp*dm is formed once for numerator and denominator; the running max / min are
/// v_max / v_min -- they differ from the reference's compare-and-assign only in the sign of a zero
/// dmin/dmax (max(+0, -0)), and a signed zero dp gives the same phi (dp*dp = +0, +0 + (+-0) = +0).
/// (A one-division-per-variable variant -- exact arg-min by cross-multiplication, only the winner divided --
/// was bitwise but 1.2-1.7 % slower: DESIGN.md section 8, profiles/r05/venk_onediv_ab.txt.)
template <bool VENK>
__device__ __forceinline__ void cell_limiter(const double* uc, const double* g, const double (*un)[4],
                                             const double2* gp, const bool* has, double2 r, double eps2,
                                             double* out)
{
	#pragma unroll
	for(int iv = 0; iv < 4; iv++) {
		double dmin = 0, dmax = 0;
		#pragma unroll
		for(int j = 0; j < 4; j++) {
			if(!has[j]) continue;
			const double d = un[j][iv]-uc[iv];
			if(VENK) { dmax = __builtin_fmax(dmax, d); dmin = __builtin_fmin(dmin, d); }
			else {
				if(d > dmax) dmax = d;
				if(d < dmin) dmin = d;
			}
		}
		double lim = 1.0;
		#pragma unroll
		for(int j = 0; j < 4; j++) {
			if(!has[j]) continue;
			double uf = uc[iv];
			uf += 1.0*g[iv*2+0]*(gp[j].x - r.x);
			uf += 1.0*g[iv*2+1]*(gp[j].y - r.y);
			double ph;
			if(VENK) {
				const double dm = uf - uc[iv];
				const double dp = dm < 0 ? dmin : dmax;
				const double pp = dp*dp, pm = dp*dm;
				// (dp*dp + 2*dp*dm + eps2)/(dp*dp + dp*dm + 2*dm*dm + eps2)
				const double n = __builtin_fma(pm, 2.0, pp) + eps2, d = __builtin_fma(dm*dm, 2.0, pp + pm) + eps2;
				lim = __builtin_fmin(lim, div_rn(n, d));
				continue;
			} else {
				const double diff = uf - uc[iv];
				if(diff > 0) ph = 1 < dmax/diff ? 1 : dmax/diff;
				else if(diff < 0) ph = 1 < dmin/diff ? 1 : dmin/diff;
				else ph = 1;
			}
			if(ph < lim) lim = ph;
		}
		out[iv] = lim;
	}
}

/// LIM (1 Barth-Jespersen, 2 Venkatakrishnan): the cell's limiter values follow from the same
/// neighbour states with k_limiter's arithmetic (face centres in reference face order from
/// cell_slots), so the separate limiter pass and its re-reads disappear
template <int LIM>
__global__ void __launch_bounds__(256) k_prep_grad_wls(DevMesh M, DevPhys P, const double* __restrict__ u,
                                                       double* __restrict__ up, double* __restrict__ ubc,
                                                       double* __restrict__ ug, double* __restrict__ grad,
                                                       int c_begin, int c_end, double* __restrict__ phi)
{
	__shared__ __attribute__((aligned(16))) double s_up[256][4];
	__shared__ __attribute__((aligned(16))) double2 s_rc[256];
	const int N = M.ncell;        // owned + ghost: neighbour codes >= N are boundary faces
	const int NO = c_end;         // this launch's cells: [c_begin, c_end) of the owned cells
	const int cb = c_begin + xcd_chunk(static_cast<int>((c_end - c_begin + 255) >> 8))*256;
	if(cb >= NO) return;
	const int t = static_cast<int>(threadIdx.x);
	const int c = cb + t;
	const int ncb = (NO - cb) < 256 ? (NO - cb) : 256;
	const Gas& G = P.gas;
	double ucons[4], uc[4];
	double2 rcc = make_double2(0, 0);
	if(c < NO) {
		ld4(u, c, ucons);
		cons2prim(G, ucons, uc);
		st4(up, c, uc);
		rcc = M.rc[c];
		st4(&s_up[t][0], 0, uc);
		s_rc[t] = rcc;
	}
	__syncthreads();
	if(c >= NO) return;
	const int4 nb4 = M.cell_nbr_fo[c];
	const int nb[4] = {nb4.x, nb4.y, nb4.z, nb4.w};
	double un[4][4];
	double2 rn[4];
	#pragma unroll
	for(int k = 0; k < 4; k++) {
		if(nb[k] < 0) continue;
		const int j = nb[k] - cb;
		if(static_cast<unsigned>(j) < static_cast<unsigned>(ncb)) {
			ld4(&s_up[j][0], 0, un[k]);
			rn[k] = s_rc[j];
		} else if(nb[k] >= N) {
			const int bf = nb[k] - N;
			const double2 nn = M.bf_n[bf];
			const double n[2] = {nn.x, nn.y};
			double gs[4];
			ghost(P, M.bf_bc[bf], ucons, n, gs);
			st4(ubc, bf, gs);
			cons2prim(G, gs, un[k]);
			st4(ug, bf, un[k]);
			rn[k] = M.bf_rcbp[bf];
		} else {
			double t4[4];
			ld4(u, nb[k], t4);
			rn[k] = M.rc[nb[k]];
			cons2prim(G, t4, un[k]);
		}
	}
	const double4 V = M.wls_V[c];
	double f[8] = {0,0,0,0,0,0,0,0};
	#pragma unroll
	for(int k = 0; k < 4; k++) {
		if(nb[k] < 0) break;
		double w2 = 0;
		w2 += (rcc.x-rn[k].x)*(rcc.x-rn[k].x);
		w2 += (rcc.y-rn[k].y)*(rcc.y-rn[k].y);
		const double dr0 = rcc.x-rn[k].x, dr1 = rcc.y-rn[k].y;
		w2 = div_rn(1.0, w2);
		#pragma unroll
		for(int iv = 0; iv < 4; iv++) {
			const double du = uc[iv] - un[k][iv];
			f[iv*2+0] += w2*dr0*du;
			f[iv*2+1] += w2*dr1*du;
		}
	}
	double g[8];
	#pragma unroll
	for(int iv = 0; iv < 4; iv++) {
		g[iv*2+0] = V.x*f[iv*2+0] + V.y*f[iv*2+1];
		g[iv*2+1] = V.z*f[iv*2+0] + V.w*f[iv*2+1];
	}
	st8(grad, c, g);
	if(LIM) {
		const int4 cs = M.cell_slots[c];
		const int sl[4] = {cs.x, cs.y, cs.z, cs.w};
		double2 gp[4];
		bool has[4];
		#pragma unroll
		for(int k = 0; k < 4; k++) {
			has[k] = nb[k] >= 0;
			if(has[k]) gp[k] = M.slot_gr[sl[k] >> 1];
		}
		double out[4];
		cell_limiter<LIM == 2>(uc, g, un, gp, has, rcc, LIM == 2 ? M.venk_eps2[c] : 0.0, out);
		st4(phi, c, out);
	}
}

/// WLS gradients of a list of owned cells (the cells other ranks hold as ghosts), all inputs from
/// global memory: same arithmetic as k_prep_grad_wls, written to grad for the halo exchange
__global__ void __launch_bounds__(256) k_grad_wls_list(DevMesh M, DevPhys P, const double* __restrict__ u,
                                                       const int* __restrict__ list, int n, double* __restrict__ grad)
{
	const int i = blockIdx.x*blockDim.x + threadIdx.x;
	if(i >= n) return;
	const int c = list[i];
	const int N = M.ncell;
	const Gas& G = P.gas;
	const int4 nb4 = M.cell_nbr_fo[c];
	const int nb[4] = {nb4.x, nb4.y, nb4.z, nb4.w};
	double ucons[4], uc[4];
	ld4(u, c, ucons);
	cons2prim(G, ucons, uc);
	const double2 rcc = M.rc[c];
	double f[8] = {0,0,0,0,0,0,0,0};
	#pragma unroll
	for(int k = 0; k < 4; k++) {
		if(nb[k] < 0) break;
		double un[4];
		double2 rn;
		if(nb[k] >= N) {
			const int bf = nb[k] - N;
			const double2 nn = M.bf_n[bf];
			const double n[2] = {nn.x, nn.y};
			double gs[4];
			ghost(P, M.bf_bc[bf], ucons, n, gs);
			cons2prim(G, gs, un);
			rn = M.bf_rcbp[bf];
		} else {
			double t4[4];
			ld4(u, nb[k], t4);
			cons2prim(G, t4, un);
			rn = M.rc[nb[k]];
		}
		double w2 = 0;
		w2 += (rcc.x-rn.x)*(rcc.x-rn.x);
		w2 += (rcc.y-rn.y)*(rcc.y-rn.y);
		const double dr0 = rcc.x-rn.x, dr1 = rcc.y-rn.y;
		w2 = div_rn(1.0, w2);
		#pragma unroll
		for(int iv = 0; iv < 4; iv++) {
			const double du = uc[iv] - un[iv];
			f[iv*2+0] += w2*dr0*du;
			f[iv*2+1] += w2*dr1*du;
		}
	}
	const double4 V = M.wls_V[c];
	double g[8];
	#pragma unroll
	for(int iv = 0; iv < 4; iv++) {
		g[iv*2+0] = V.x*f[iv*2+0] + V.y*f[iv*2+1];
		g[iv*2+1] = V.z*f[iv*2+0] + V.w*f[iv*2+1];
	}
	st8(grad, c, g);
}

/// WLS gradients of the layer-1 ghosts of a two-layer halo, from the received layer-1 and layer-2
/// states: the arithmetic of k_grad_wls_list on the ghost's own neighbour list (ascending global face
/// order; extra boundary faces for the physical faces no owned cell touches), so each value is the
/// owner's bit for bit and needs no exchange. LIM (1 Barth-Jespersen, 2 Venkatakrishnan): the ghost's
/// limiter values too, k_prep_grad_wls<LIM>'s cell_limiter on the same neighbour states (boundary:
/// the ghost primitive state) and the ghost's face centres -- the owner's values, since min / max over
/// the faces do not depend on their order (limitedlinearreconstruction.cpp:107-268)
template <int LIM>
__global__ void __launch_bounds__(256) k_grad_ghost(DevMesh M, DevPhys P, const double* __restrict__ u,
                                                    double* __restrict__ grad, double* __restrict__ phi)
{
	const int i = blockIdx.x*blockDim.x + threadIdx.x;
	if(i >= M.gg_n) return;
	const int c = M.gg_cells[i];
	const Gas& G = P.gas;
	const int4 nb4 = M.gg_nbr[i];
	const int nb[4] = {nb4.x, nb4.y, nb4.z, nb4.w};
	// every row this ghost reads is requested at once (a second dependent round trip after the cell
	// and neighbour ids), not one neighbour after another: the kernel is latency-bound (a few
	// thousand ghosts per rank) and sits on the halo's critical path
	double ucons[4], uc[4];
	ld4(u, c, ucons);
	const double2 rcc = M.rc[c];
	double t4[4][4];
	double2 rn4[4];
	#pragma unroll
	for(int k = 0; k < 4; k++) {
		const int j = nb[k] >= 0 ? nb[k] : c;
		ld4(u, j, t4[k]);
		rn4[k] = M.rc[j];
	}
	cons2prim(G, ucons, uc);
	double f[8] = {0,0,0,0,0,0,0,0};
	double un[4][4];
	#pragma unroll
	for(int k = 0; k < 4; k++) {
		if(nb[k] == -1) break;
		double2 rn;
		if(nb[k] < 0) {
			const int x = -2 - nb[k];
			const double2 nn = M.xb_n[x];
			const double n[2] = {nn.x, nn.y};
			double gs[4];
			ghost(P, M.xb_bc[x], ucons, n, gs);
			cons2prim(G, gs, un[k]);
			rn = M.xb_rcbp[x];
		} else {
			cons2prim(G, t4[k], un[k]);
			rn = rn4[k];
		}
		double w2 = 0;
		w2 += (rcc.x-rn.x)*(rcc.x-rn.x);
		w2 += (rcc.y-rn.y)*(rcc.y-rn.y);
		const double dr0 = rcc.x-rn.x, dr1 = rcc.y-rn.y;
		w2 = div_rn(1.0, w2);
		#pragma unroll
		for(int iv = 0; iv < 4; iv++) {
			const double du = uc[iv] - un[k][iv];
			f[iv*2+0] += w2*dr0*du;
			f[iv*2+1] += w2*dr1*du;
		}
	}
	const double4 V = M.gg_V[i];
	double g[8];
	#pragma unroll
	for(int iv = 0; iv < 4; iv++) {
		g[iv*2+0] = V.x*f[iv*2+0] + V.y*f[iv*2+1];
		g[iv*2+1] = V.z*f[iv*2+0] + V.w*f[iv*2+1];
	}
	st8(grad, c, g);
	if(LIM) {
		double2 gp[4];
		bool has[4];
		#pragma unroll
		for(int k = 0; k < 4; k++) {
			has[k] = nb[k] != -1;
			gp[k] = M.gg_gp[4*i + k];
		}
		double out[4];
		cell_limiter<LIM == 2>(uc, g, un, gp, has, rcc, LIM == 2 ? M.gg_eps2[i] : 0.0, out);
		st4(phi, c, out);
	}
}

__global__ void __launch_bounds__(256) k_grad_gg(DevMesh M, const double* __restrict__ up,
                                                 const double* __restrict__ ug, double* __restrict__ grad)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= M.nown) return;
	const int N = M.ncell;     // cells incl. ghosts: codes >= N are boundary faces
	const int4 cs = M.cell_slots[c];
	const int e[4] = {cs.x, cs.y, cs.z, cs.w};
	double g[8] = {0,0,0,0,0,0,0,0};
	const double ainv = div_rn(1.0, M.area[c]);
	#pragma unroll
	for(int k = 0; k < 4; k++) {
		if(e[k] < 0) break;
		const int s = e[k] >> 1;
		const int2 lr = M.slot_LR[s];
		const double2 mid = M.slot_gr[s];
		const double2 nn = M.slot_n[s];
		const double len = M.slot_len[s];
		double uL[4], uR[4];
		const double2 rl = M.rc[lr.x];
		double2 rr;
		ld4(up, lr.x, uL);
		if(lr.y >= N) { rr = M.bf_rcbp[lr.y - N]; ld4(ug, lr.y - N, uR); }
		else          { rr = M.rc[lr.y];           ld4(up, lr.y, uR); }
		double dL = 0, dR = 0;
		dL += (mid.x-rl.x)*(mid.x-rl.x); dR += (mid.x-rr.x)*(mid.x-rr.x);
		dL += (mid.y-rl.y)*(mid.y-rl.y); dR += (mid.y-rr.y)*(mid.y-rr.y);
		dL = div_rn(1.0, sqrt_rn(dL));
		dR = div_rn(1.0, sqrt_rn(dR));
		const bool right = e[k] & 1;
		#pragma unroll
		for(int iv = 0; iv < 4; iv++) {
			const double ut = div_rn(uL[iv]*dL + uR[iv]*dR, dL+dR) * len;
			if(!right) { g[iv*2+0] += (ut*nn.x)*ainv; g[iv*2+1] += (ut*nn.y)*ainv; }
			else       { g[iv*2+0] -= (ut*nn.x)*ainv; g[iv*2+1] -= (ut*nn.y)*ainv; }
		}
	}
	st8(grad, c, g);
}

// ------------------------------------------------------------------------------------------------
// limiters (limitedlinearreconstruction.cpp:107-268). Physical-boundary neighbours use the ghost
// primitive state (documented deviation: the reference reads past the end of its array there).
// ------------------------------------------------------------------------------------------------
template <bool VENK>
__global__ void __launch_bounds__(256) k_limiter(DevMesh M, const double* __restrict__ up, const double* __restrict__ ug,
                                                 const double* __restrict__ grad, double* __restrict__ phi)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= M.nown) return;
	const int N = M.ncell;     // cells incl. ghosts: codes >= N are boundary faces
	double uc[4], g[8];
	ld4(up, c, uc);
	ld8(grad, c, g);
	const int4 nb4 = M.cell_nbr[c], fs4 = M.cell_face[c];
	const int nbr[4] = {nb4.x, nb4.y, nb4.z, nb4.w}, fcs[4] = {fs4.x, fs4.y, fs4.z, fs4.w};
	const double2 r = M.rc[c];
	const double eps2 = VENK ? M.venk_eps2[c] : 0.0;
	double un[4][4];
	double2 gp[4];
	#pragma unroll
	for(int j = 0; j < 4; j++) {
		if(nbr[j] < 0) continue;
		if(nbr[j] >= N) ld4(ug, nbr[j]-N, un[j]); else ld4(up, nbr[j], un[j]);
		gp[j] = M.slot_gr[fcs[j]];
	}
	const bool has[4] = {nbr[0] >= 0, nbr[1] >= 0, nbr[2] >= 0, nbr[3] >= 0};
	double out[4];
	cell_limiter<VENK>(uc, g, un, gp, has, r, eps2, out);
	st4(phi, c, out);
}

// WENO-limited gradients (limitedlinearreconstruction.cpp:27-105)
__global__ void __launch_bounds__(256) k_weno(DevMesh M, double lambda, const double* __restrict__ grad,
                                              double* __restrict__ lgrad)
{
	const int c = blockIdx.x*blockDim.x + threadIdx.x;
	if(c >= M.nown) return;
	const int N = M.ncell;     // cells incl. ghosts: codes >= N are boundary faces
	const double gamma = 4.0, epsilon = 1.0e-5;
	double g0[8];
	ld8(grad, c, g0);
	const int4 nb4 = M.cell_nbr[c];
	const int nbr[4] = {nb4.x, nb4.y, nb4.z, nb4.w};
	double gn[4][8];
	#pragma unroll
	for(int j = 0; j < 4; j++) if(nbr[j] >= 0 && nbr[j] < N) ld8(grad, nbr[j], gn[j]);
	double out[8];
	#pragma unroll
	for(int iv = 0; iv < 4; iv++) {
		double wsum = 0, l0 = 0, l1 = 0;
		{
			double m2 = 0; m2 += g0[iv*2]*g0[iv*2]; m2 += g0[iv*2+1]*g0[iv*2+1];
			const double w = lambda / pow(m2 + epsilon, gamma);
			wsum += w; l0 += w*g0[iv*2]; l1 += w*g0[iv*2+1];
		}
		#pragma unroll
		for(int j = 0; j < 4; j++) {
			if(nbr[j] < 0 || nbr[j] >= N) continue;
			double m2 = 0; m2 += gn[j][iv*2]*gn[j][iv*2]; m2 += gn[j][iv*2+1]*gn[j][iv*2+1];
			const double w = 1.0 / pow(m2 + epsilon, gamma);
			wsum += w; l0 += w*gn[j][iv*2]; l1 += w*gn[j][iv*2+1];
		}
		out[iv*2] = l0/wsum; out[iv*2+1] = l1/wsum;
	}
	st8(lgrad, c, out);
}

// ------------------------------------------------------------------------------------------------
// THE SWEEP
// ------------------------------------------------------------------------------------------------

/// MUSCL / Van Albada pieces (musclreconstruction.cpp:33-59, 86-90, 112-120), bitwise in fewer
/// instructions: the numerator 2.0*d*du + eps as fma(d*du, 2, eps) (2d is exact, so RN(2d*du) =
/// 2 RN(d*du)); `phi < 0 -> 0` as one v_max (phi is never -0: the numerator RN(x + 1e-8) is +0 when
/// x = -1e-8, and the denominator is positive); ui + phi/4.0*S as fma(phi*S, 1/4, ui) (add_pow2)
__device__ __forceinline__ double muscl_phi(double d, double du) {
	const double eps = 1e-8;
	const double ph = div_rn(__builtin_fma(d*du, 2.0, eps), d*d + du*du + eps);
	return __builtin_fmax(ph, 0.0);
}
__device__ __forceinline__ double muscl_left(double ui, double uj, double dm, double ph) {
	const double k = 1.0/3.0;
	return add_pow2(ui, ph*( (1.0-k*ph)*dm + (1.0+k*ph)*(uj - ui) ), 0.25);
}
__device__ __forceinline__ double muscl_right(double ui, double uj, double dp, double ph) {
	const double k = 1.0/3.0;
	return add_pow2(uj, ph*( (1.0-k*ph)*dp + (1.0+k*ph)*(uj - ui) ), -0.25);
}

/// Per-cell words (doubles) staged in LDS for a sweep variant, one 16-byte-aligned row per cell:
///   order 2: [up 4][reconstruction gradient 8][rc 2] (+[phi 4] if limiter); the viscous flux
///            takes its primitive states from up as well
///   order 1: [u 4] (+[rc 2] if viscous)
template <int REC, int VISC, bool PHI> struct Stage {
	static constexpr bool O2 = REC != SR_FIRST;
	static constexpr bool V = VISC != SV_NONE;
	static constexpr int UP = 0, RG = 4;
	static constexpr int RC = O2 ? 12 : 4;
	static constexpr int UC = 0;            // order 1 only
	static constexpr int PH = 14;
	static constexpr int W0 = O2 ? (14 + (PHI ? 4 : 0)) : (V ? 6 : 4);
	static constexpr int W = (W0 + 1) & ~1;
	static constexpr int BUF = (W > 6 ? W : 6) * SLOTS_MAX;   // flux staging reuses the buffer
};

template <int FLUX, int REC, int VISC, bool DT, bool PHI>
__global__ void __launch_bounds__(SLOTS_MAX) k_sweep(const DevMesh M, const DevPhys P, const SweepBuffers B)
{
	typedef Stage<REC, VISC, PHI> S;
	constexpr int W = S::W;
	__shared__ __attribute__((aligned(16))) double sbuf[S::BUF];

	// XCD-aware mapping: consecutive patches (which share halo cells) land on the same XCD
	const int np = B.plist ? B.pcount : M.npatch;
	const int q = (np + 7) >> 3;
	const int pi = (blockIdx.x & 7) * q + (blockIdx.x >> 3);
	if(pi >= np) return;
	const int p = B.plist ? B.plist[pi] : pi;
	const int s0 = M.patch_slot[p], s1 = M.patch_slot[p+1];
	const int c0 = M.patch_cell[p], c1 = M.patch_cell[p+1];
	const int nc = c1 - c0;
	const int N = M.ncell;
	const Gas& G = P.gas;
	const int t = static_cast<int>(threadIdx.x);

	// phase 0: stage the patch's own cells (contiguous range) with coalesced loads
	if(t < nc) {
		const int c = c0 + t;
		double* row = &sbuf[t*W];
		double a[8];
		if(S::O2) {
			ld4(B.up, c, a); st4(row + S::UP, 0, a);
			ld8(B.rgrad, c, a); st8(row + S::RG, 0, a);
			const double2 r = M.rc[c]; *reinterpret_cast<double2*>(row + S::RC) = r;
			if(PHI) { ld4(B.phi, c, a); st4(row + S::PH, 0, a); }
		} else {
			ld4(B.u, c, a); st4(row + S::UC, 0, a);
			if(S::V) { const double2 r = M.rc[c]; *reinterpret_cast<double2*>(row + S::RC) = r; }
		}
	}
	__syncthreads();

	// cell data from LDS when the cell is in this patch, else from global memory (halo). The LDS row
	// is read unconditionally (row 0 for a halo cell) and pinned in registers before the global
	// values may replace it, so the two never merge into one generic (flat) load
	auto inp = [&](int cell) { return static_cast<unsigned>(cell - c0) < static_cast<unsigned>(nc); };
	auto lrow = [&](int cell, int off) { return &sbuf[(inp(cell) ? cell - c0 : 0)*W + off]; };
	auto get4 = [&](int cell, int off, const double* g, double* o) {
		ld4(lrow(cell, off), 0, o);
		for(int k = 0; k < 4; k++) pin_regs(o[k]);
		if(!inp(cell)) ld4(g, cell, o);
	};
	auto get8 = [&](int cell, int off, const double* g, double* o) {
		ld8(lrow(cell, off), 0, o);
		for(int k = 0; k < 8; k++) pin_regs(o[k]);
		if(!inp(cell)) ld8(g, cell, o);
	};
	auto getrc = [&](int cell) -> double2 {
		double2 v = *reinterpret_cast<const double2*>(lrow(cell, S::RC));
		pin_regs(v.x); pin_regs(v.y);
		if(!inp(cell)) v = M.rc[cell];
		return v;
	};

	const int s = s0 + t;
	double f[4] = {0, 0, 0, 0};
	double sri = 0, srj = 0;
	if(s < s1) {
		const int2 lr = M.slot_LR[s];
		const double2 nn = M.slot_n[s];
		const double len = M.slot_len[s];
		const double n[2] = {nn.x, nn.y};
		const bool bnd = lr.y >= N;
		const int bf = lr.y - N;
		double ul[4], ur[4];

		if(REC == SR_FIRST) {
			get4(lr.x, S::UC, B.u, ul);
			if(bnd) ghost(P, M.bf_bc[bf], ul, n, ur);
			else    get4(lr.y, S::UC, B.u, ur);
		}
		else if(REC == SR_MUSCL) {
			const double2 ri = getrc(lr.x);
			double ui[4], gi[8];
			get4(lr.x, S::UP, B.up, ui);
			get8(lr.x, S::RG, B.rgrad, gi);
			if(!bnd) {
				const double2 rj = getrc(lr.y);
				double uj[4], gj[8];
				get4(lr.y, S::UP, B.up, uj);
				get8(lr.y, S::RG, B.rgrad, gj);
				const double dx = rj.x-ri.x, dy = rj.y-ri.y;
				#pragma unroll
				for(int i = 0; i < 4; i++) {
					double dl = mul0(gi[i*2], dx); dl += gi[i*2+1]*dy;
					double dr = mul0(gj[i*2], dx); dr += gj[i*2+1]*dy;
					const double du = uj[i] - ui[i];
					const double dm = twice_minus(dl, du);
					const double dp = twice_minus(dr, du);
					ul[i] = muscl_left(ui[i], uj[i], dm, muscl_phi(dm, du));
					ur[i] = muscl_right(ui[i], uj[i], dp, muscl_phi(dp, du));
				}
				prim2cons(G, ul, ul);
				prim2cons(G, ur, ur);
			} else {
				const double2 rj = M.bf_rcbp[bf];
				double uj[4];
				ld4(B.ug, bf, uj);
				const double dx = rj.x-ri.x, dy = rj.y-ri.y;
				#pragma unroll
				for(int i = 0; i < 4; i++) {
					double dl = mul0(gi[i*2], dx); dl += gi[i*2+1]*dy;
					const double du = uj[i] - ui[i];
					const double dm = twice_minus(dl, du);
					ul[i] = muscl_left(ui[i], uj[i], dm, muscl_phi(dm, du));
				}
				prim2cons(G, ul, ul);
				ghost(P, M.bf_bc[bf], ul, n, ur);
			}
		}
		else {  // SR_LINEAR: unlimited, WENO-limited gradients or BJ/Venkatakrishnan limiter values
			const double2 gp = M.slot_gr[s];
			{
				const double2 ri = getrc(lr.x);
				double ui[4], gi[8], ph[4] = {1.0, 1.0, 1.0, 1.0};
				get4(lr.x, S::UP, B.up, ui);
				get8(lr.x, S::RG, B.rgrad, gi);
				if(PHI) get4(lr.x, S::PH, B.phi, ph);
				#pragma unroll
				for(int i = 0; i < 4; i++) {
					double v = ui[i];
					v += ph[i]*gi[i*2]*(gp.x - ri.x);
					v += ph[i]*gi[i*2+1]*(gp.y - ri.y);
					ul[i] = v;
				}
				prim2cons(G, ul, ul);
			}
			if(!bnd) {
				const double2 rj = getrc(lr.y);
				double uj[4], gj[8], ph[4] = {1.0, 1.0, 1.0, 1.0};
				get4(lr.y, S::UP, B.up, uj);
				get8(lr.y, S::RG, B.rgrad, gj);
				if(PHI) get4(lr.y, S::PH, B.phi, ph);
				#pragma unroll
				for(int i = 0; i < 4; i++) {
					double v = uj[i];
					v += ph[i]*gj[i*2]*(gp.x - rj.x);
					v += ph[i]*gj[i*2+1]*(gp.y - rj.y);
					ur[i] = v;
				}
				prim2cons(G, ur, ur);
			} else {
				ghost(P, M.bf_bc[bf], ul, n, ur);
			}
		}

		inviscid_flux_len<FLUX>(G, ul, ur, n, len, f);

		if(VISC != SV_NONE) {
			// order 2: primitive states (up / ghost ug); order 1: conserved states
			double ucl[4], ucr[4], gl[8], gr[8];
			const double2 rl = getrc(lr.x);
			double2 rr;
			if(REC == SR_FIRST) get4(lr.x, S::UC, B.u, ucl);
			else get4(lr.x, S::UP, B.up, ucl);
			if(bnd) {
				rr = M.bf_rcbp[bf];
				if(REC == SR_FIRST) { for(int k = 0; k < 4; k++) ucr[k] = ur[k]; }
				else ld4(B.ug, bf, ucr);
			} else {
				rr = getrc(lr.y);
				if(REC == SR_FIRST) get4(lr.y, S::UC, B.u, ucr);
				else get4(lr.y, S::UP, B.up, ucr);
			}
			if(REC != SR_FIRST) {
				const int cr = bnd ? lr.x : lr.y;
				if(B.grad == B.rgrad) { get8(lr.x, S::RG, B.grad, gl); get8(cr, S::RG, B.grad, gr); }
				else { ld8(B.grad, lr.x, gl); ld8(B.grad, cr, gr); }
			}
			const double rcl[2] = {rl.x, rl.y}, rcr[2] = {rr.x, rr.y};
			double vf[4];
			viscous_flux<REC != SR_FIRST, VISC == SV_CONST>(G, n, rcl, rcr, ucl, ucr, gl, gr, ul, ur, vf);
			#pragma unroll
			for(int k = 0; k < 4; k++) f[k] += vf[k]*len;
		}

		if(DT) {
			const double ci = sound_speed_cons(G, ul), cj = sound_speed_cons(G, ur);
			const double vni = div_rn(dot2(&ul[1],n), ul[0]);
			const double vnj = div_rn(dot2(&ur[1],n), ur[0]);
			sri = (fabs(vni)+ci)*len;
			srj = (fabs(vnj)+cj)*len;
			if(VISC != SV_NONE) {
				const double mui = VISC == SV_CONST ? G.rReinf : sutherland(G, ul);
				const double muj = VISC == SV_CONST ? G.rReinf : sutherland(G, ur);
				const double coi = visc_coef(G, ul[0]), coj = visc_coef(G, ur[0]);   // std::max(4/(3 rho), g/rho)
				// a ghost cell's spectral radius is never summed (and its area is not stored)
				if(lr.x < M.nown) sri += div_rn(div_rcp(coi*mui, G.Pr, G.rPr) * len*len, M.area[lr.x]);
				if(!bnd && lr.y < M.nown) srj += div_rn(div_rcp(coj*muj, G.Pr, G.rPr) * len*len, M.area[lr.y]);
			}
		}
	}
	// the cell's face list (and area) are requested before the two barriers of the flux staging,
	// once the face work no longer holds registers
	const int c = c0 + t;
	int4 cs = make_int4(-1, -1, -1, -1);
	double carea = 0.0;
	if(c < c1) { cs = M.cell_slots[c]; if(DT) carea = M.area[c]; }
	__syncthreads();   // every slot has read the staged cells: reuse the buffer for the fluxes
	double* sf = sbuf;                  // [4][SLOTS_MAX]
	double* ssr = sbuf + 4*SLOTS_MAX;   // [2][SLOTS_MAX]
	if(s < s1) {
		sf[0*SLOTS_MAX + t] = f[0]; sf[1*SLOTS_MAX + t] = f[1];
		sf[2*SLOTS_MAX + t] = f[2]; sf[3*SLOTS_MAX + t] = f[3];
		if(DT) { ssr[t] = sri; ssr[SLOTS_MAX + t] = srj; }
	}
	__syncthreads();

	if(c < c1) {
		double r[4];
		if(B.overwrite) { r[0] = r[1] = r[2] = r[3] = 0.0; }
		else ld4(B.r, c, r);
		double integ = 0.0;
		const int e[4] = {cs.x, cs.y, cs.z, cs.w};
		#pragma unroll
		for(int k = 0; k < 4; k++) {
			if(e[k] < 0) break;
			const int ls = (e[k] >> 1) - s0;
			if(e[k] & 1) {
				r[0] += sf[0*SLOTS_MAX + ls]; r[1] += sf[1*SLOTS_MAX + ls];
				r[2] += sf[2*SLOTS_MAX + ls]; r[3] += sf[3*SLOTS_MAX + ls];
				if(DT) integ += ssr[SLOTS_MAX + ls];
			} else {
				r[0] -= sf[0*SLOTS_MAX + ls]; r[1] -= sf[1*SLOTS_MAX + ls];
				r[2] -= sf[2*SLOTS_MAX + ls]; r[3] -= sf[3*SLOTS_MAX + ls];
				if(DT) integ += ssr[ls];
			}
		}
		st4(B.r, c, r);
		if(DT) B.dtm[c] = div_rn(carea, integ);
	}
}

// ------------------------------------------------------------------------------------------------
// THE FUSED RESIDUAL (WLS gradients + MUSCL / unlimited linear reconstruction, inviscid)
// One launch per residual: every patch stages its cells and its ring-1 cells (far side of its cut
// faces) in LDS as primitive states, recomputes their WLS gradients there (ring-2 neighbours come
// from global memory), then sweeps its faces and sums them per cell. Same operations, same order as
// k_prep_grad_wls + k_sweep: the result is bitwise the staged path's. Ring-1 gradients are computed
// by every patch that needs them (35 % more gradients on C4) instead of a round trip through HBM.
// LDS row per staged cell (14 doubles): [up 4][gradient 8][rc 2]; viscous instantiations 18:
// [up 4][gradient 8][rc 2][T, dT/dx, dT/dy, pad] (the temperature terms of fz_viscous, per gradient row)
// ------------------------------------------------------------------------------------------------
constexpr int FZW = 14;
constexpr int FZW_VISC = 18;
template <int VISC> constexpr int fz_w() { return VISC != SV_NONE ? FZW_VISC : FZW; }

/// primitive ghost state of a cell's value across boundary face bf (k_prep_bfaces arithmetic)
/// the fused residual's ghost states: the common BC types' ghost_state (gasdyn.hpp ghost_state_common)
/// inlined -- fusedEligible admits only configurations whose BCs are all of those types (the others
/// take the staged path). An out-of-line call in this kernel (ghost_ool: 82 VGPRs of its own, and the
/// caller's values kept live across the call) costs 28 VGPRs on every path: 118 instead of 90 for the
/// inviscid kernel, i.e. 4 instead of 5 waves per SIMD; 162 instead of 124 for the limited ones
__device__ __forceinline__ void ghost_c(const DevPhys& P, int bc, const double* ins, const double* n, double* gs)
{
	const double ui[4] = {P.uinf[0], P.uinf[1], P.uinf[2], P.uinf[3]};
	ghost_state_common(P.gas, P.bc[bc], ui, ins, n, gs);
}
/// the conserved state row of cell c the fused residual works on: u[c], or with the fused matrix-free
/// operator (SweepBuffers::mfx; MF: instantiations without time steps only) the perturbed state
/// u[c] + pm[1] x[c], k_mf_perturb's arithmetic
template <bool MF>
__device__ __forceinline__ void ld_state(const SweepBuffers& B, int c, double* o)
{
	ld4(B.u, c, o);
	if(MF && B.mfx) {
		double x[4];
		ld4(B.mfx, c, x);
		const double s = B.mfpm[1];
		#pragma unroll
		for(int i = 0; i < 4; i++) o[i] = o[i] + s*x[i];
	}
}
template <bool MF>
__device__ __forceinline__ double4 ghost_prim_of_cell(const DevMesh& M, const DevPhys& P, const SweepBuffers& B, int cell, int bf)
{
	const double2 nn = M.bf_n[bf];
	const double n[2] = {nn.x, nn.y};
	double ucons[4], gs[4], gp[4];
	ld_state<MF>(B, cell, ucons);
	ghost_c(P, M.bf_bc[bf], ucons, n, gs);
	cons2prim(P.gas, gs, gp);
	return make_double4(gp[0], gp[1], gp[2], gp[3]);
}

/// phase 0 of the fused residual: a staged row [up 4][gradient 8][rc 2] from the conserved state
__device__ __forceinline__ void stage_row(const Gas& G, double* row, const double* ucons, double2 r)
{
	double b[4];
	cons2prim(G, ucons, b);
	st4(row, 0, b);
	*reinterpret_cast<double2*>(row + 12) = r;
}

/// The fused residual rebuilds each cell's WLS inverse from the staged centres it already reads instead of
/// loading the precomputed one (32 B per gradient row less traffic).
/// One neighbour's term of the WLS normal matrix, V[2i+j] += w2*dr[i]*dr[j] (agradientschemes.cpp:
/// 218-317 as restated in layout.cpp: w2*dr[i] first, then times dr[j])
__device__ __forceinline__ void wls_normal_add(double* vm, double w2, double d0, double d1)
{
	const double a = w2*d0, b = w2*d1;
	vm[0] += a*d0; vm[1] += a*d1; vm[2] += b*d0; vm[3] += b*d1;
}
/// the first neighbour's term, 0 + w2*dr[i]*dr[j] (mul0)
__device__ __forceinline__ void wls_normal_first(double* vm, double w2, double d0, double d1)
{
	const double a = w2*d0, b = w2*d1;
	vm[0] = mul0(a, d0); vm[1] = mul0(a, d1); vm[2] = mul0(b, d0); vm[3] = mul0(b, d1);
}
/// its inverse, the host's 2x2 inverse arithmetic (layout.cpp, Eigen's inverse for 2x2)
__device__ __forceinline__ double4 wls_inverse(const double* v)
{
	const double det = v[0]*v[3] - v[2]*v[1];
	const double invdet = div_rn(1.0, det);
	return make_double4(v[3]*invdet, -v[1]*invdet, -v[2]*invdet, v[0]*invdet);
}

/// phase 1 of the fused residual: WLS gradient of staged row `row` (cell c) from the staged rows of
/// its neighbours nb4 (patch-local indices, boundary codes -2-bf, -1 padding), k_prep_grad_wls
/// arithmetic; a ghost cell takes the gradient received from its owner
/// the centres of cell c's faces in ascending reference face order (k_prep_grad_wls<LIM>'s source:
/// cell_slots -> slot_gr); padding entries (0, 0)
__device__ __forceinline__ void fz_face_centres(const DevMesh& M, int c, double2* gp)
{
	const int4 cs = M.cell_slots[c];
	const int sl[4] = {cs.x, cs.y, cs.z, cs.w};
	#pragma unroll
	for(int k = 0; k < 4; k++) gp[k] = sl[k] >= 0 ? M.slot_gr[sl[k] >> 1] : make_double2(0, 0);
}
template <int LIM, int W = FZW, bool MF = false>
__device__ __forceinline__ void fused_limit_row(const DevMesh& M, const DevPhys& P, const SweepBuffers& B,
                                                const double* fz, const double* row, int c, int4 nb4,
                                                const double2* gp, double eps2, double* g);
/// viscous rows (W = FZW_VISC): the temperature and its gradient of the row's cell, the arithmetic
/// fz_viscous applied per face side until round 4 (temperature(rho, p), grad_temperature per direction
/// from the density and pressure gradients), formed once per gradient row instead
template <int W>
__device__ __forceinline__ void fz_row_temperature(const Gas& G, double* row, const double* g)
{
	if constexpr(W == FZW_VISC) {
		const double rho = row[0], p = row[3];
		const double tx = grad_temperature(G, rho, g[0*2+0], p, g[3*2+0]);
		const double ty = grad_temperature(G, rho, g[0*2+1], p, g[3*2+1]);
		*reinterpret_cast<double2*>(row + 14) = make_double2(temperature(G, rho, p), tx);
		row[16] = ty;
	}
}
template <int LIM, int W = FZW, bool MF = false>
__device__ __forceinline__ void fused_wls_row(const DevMesh& M, const DevPhys& P, const SweepBuffers& B,
                                              const double* fz, double* row, int c, int4 nb4,
                                              const double2* gp = nullptr, double eps2 = 0.0)
{
	static_assert(!(LIM && W == FZW_VISC), "limited reconstructions are not fused with the viscous flux");
	if(c >= M.nown) {
		double g[8];
		ld8(B.grad, c, g);
		if(LIM) {
			// layer-1 ghost of a two-layer halo: its limiter values were computed locally
			// (k_grad_ghost<LIM>); lim*g as fused_limit_row forms it
			double lim[4];
			ld4(B.phi, c, lim);
			#pragma unroll
			for(int iv = 0; iv < 4; iv++) { g[iv*2+0] = lim[iv]*g[iv*2+0]; g[iv*2+1] = lim[iv]*g[iv*2+1]; }
		}
		st8(row + 4, 0, g);
		fz_row_temperature<W>(P.gas, row, g);
		return;
	}
	double uc[4];
	ld4(row, 0, uc);
	const double2 rcc = *reinterpret_cast<const double2*>(row + 12);
	double f[8] = {0,0,0,0,0,0,0,0};
	double vm[4] = {0, 0, 0, 0};     // WLS normal matrix, same terms and order as the host's
	if(nb4.x >= 0 && nb4.y >= 0 && nb4.z >= 0 && nb4.w >= -1) {
		// no boundary neighbour (all but ~0.1 % of the rows): every neighbour is an LDS row. The
		// first three (every triangle and quad has them) are requested at once and their weights
		// computed side by side instead of one LDS round trip and one division chain after another;
		// the fourth (quads) follows
		const int nb[3] = {nb4.x, nb4.y, nb4.z};
		double w[3], d0[3], d1[3], un[3][4];
		#pragma unroll
		for(int k = 0; k < 3; k++) {
			const double* nrow = &fz[nb[k]*W];
			const double2 rn = *reinterpret_cast<const double2*>(nrow + 12);
			ld4(nrow, 0, un[k]);
			double w2 = mul0(rcc.x-rn.x, rcc.x-rn.x);
			w2 += (rcc.y-rn.y)*(rcc.y-rn.y);
			d0[k] = rcc.x-rn.x; d1[k] = rcc.y-rn.y;
			w[k] = div_rn(1.0, w2);
		}
		// the sums start from zero: the first neighbour's terms are 0 + a*b (mul0)
		#pragma unroll
		for(int iv = 0; iv < 4; iv++) {
			const double du = uc[iv] - un[0][iv];
			f[iv*2+0] = mul0(w[0]*d0[0], du);
			f[iv*2+1] = mul0(w[0]*d1[0], du);
		}
		wls_normal_first(vm, w[0], d0[0], d1[0]);
		#pragma unroll
		for(int k = 1; k < 3; k++) {
			#pragma unroll
			for(int iv = 0; iv < 4; iv++) {
				const double du = uc[iv] - un[k][iv];
				f[iv*2+0] += w[k]*d0[k]*du;
				f[iv*2+1] += w[k]*d1[k]*du;
			}
			wls_normal_add(vm, w[k], d0[k], d1[k]);
		}
		if(nb4.w >= 0) {
			const double* nrow = &fz[nb4.w*W];
			const double2 rn = *reinterpret_cast<const double2*>(nrow + 12);
			double u3[4];
			ld4(nrow, 0, u3);
			double w2 = mul0(rcc.x-rn.x, rcc.x-rn.x);
			w2 += (rcc.y-rn.y)*(rcc.y-rn.y);
			const double e0 = rcc.x-rn.x, e1 = rcc.y-rn.y;
			w2 = div_rn(1.0, w2);
			#pragma unroll
			for(int iv = 0; iv < 4; iv++) {
				const double du = uc[iv] - u3[iv];
				f[iv*2+0] += w2*e0*du;
				f[iv*2+1] += w2*e1*du;
			}
			wls_normal_add(vm, w2, e0, e1);
		}
	} else
	#pragma unroll
	for(int k = 0; k < 4; k++) {
		const int nbk = k == 0 ? nb4.x : (k == 1 ? nb4.y : (k == 2 ? nb4.z : nb4.w));
		if(nbk == -1) break;
		// the LDS row is read unconditionally (row 0 for a boundary code) and pinned in registers
		// before the boundary values may replace it: otherwise the compiler merges the two loads
		// into one generic (flat) load of a selected pointer, which waits on every outstanding
		// global load of the wave
		double un[4];
		const double* nrow = &fz[(nbk >= 0 ? nbk : 0)*W];
		ld4(nrow, 0, un);
		double2 rn = *reinterpret_cast<const double2*>(nrow + 12);
		pin_regs(un[0]); pin_regs(un[1]); pin_regs(un[2]); pin_regs(un[3]); pin_regs(rn.x); pin_regs(rn.y);
		if(nbk < 0) {
			const int bf = -2 - nbk;
			const double4 gp = ghost_prim_of_cell<MF>(M, P, B, c, bf);
			un[0] = gp.x; un[1] = gp.y; un[2] = gp.z; un[3] = gp.w;
			rn = M.bf_rcbp[bf];
		}
		double w2 = 0;
		w2 += (rcc.x-rn.x)*(rcc.x-rn.x);
		w2 += (rcc.y-rn.y)*(rcc.y-rn.y);
		const double dr0 = rcc.x-rn.x, dr1 = rcc.y-rn.y;
		w2 = div_rn(1.0, w2);
		#pragma unroll
		for(int iv = 0; iv < 4; iv++) {
			const double du = uc[iv] - un[iv];
			f[iv*2+0] += w2*dr0*du;
			f[iv*2+1] += w2*dr1*du;
		}
		wls_normal_add(vm, w2, dr0, dr1);
	}
	const double4 V = wls_inverse(vm);
	double g[8];
	#pragma unroll
	for(int iv = 0; iv < 4; iv++) {
		g[iv*2+0] = V.x*f[iv*2+0] + V.y*f[iv*2+1];
		g[iv*2+1] = V.z*f[iv*2+0] + V.w*f[iv*2+1];
	}
	if(LIM) fused_limit_row<LIM, W, MF>(M, P, B, fz, row, c, nb4, gp, eps2, g);
	st8(row + 4, 0, g);
	fz_row_temperature<W>(P.gas, row, g);
}

/// limited reconstructions in the fused residual: the row's Barth-Jespersen / Venkatakrishnan limiter
/// values from the staged neighbour states (boundary: the ghost primitive state, as the staged path)
/// and its face centres, k_prep_grad_wls<LIM>'s arithmetic; the staged row then holds lim*g, which is
/// the product linearExtrapolate forms first ((lim*grad)*(gp - rc), reconstruction_utils.hpp:28-30)
template <int LIM, int W, bool MF>
__device__ __forceinline__ void fused_limit_row(const DevMesh& M, const DevPhys& P, const SweepBuffers& B,
                                                const double* fz, const double* row, int c, int4 nb4,
                                                const double2* gpre, double eps2, double* g)
{
	double uc[4];
	ld4(row, 0, uc);
	const double2 rcc = *reinterpret_cast<const double2*>(row + 12);
	double2 gp[4];
	if(gpre) { gp[0] = gpre[0]; gp[1] = gpre[1]; gp[2] = gpre[2]; gp[3] = gpre[3]; }
	else { fz_face_centres(M, c, gp); eps2 = LIM == 2 ? M.venk_eps2[c] : 0.0; }
	const int nb[4] = {nb4.x, nb4.y, nb4.z, nb4.w};
	double un[4][4];
	bool has[4];
	#pragma unroll
	for(int k = 0; k < 4; k++) {
		has[k] = nb[k] != -1;
		un[k][0] = un[k][1] = un[k][2] = un[k][3] = 0.0;
		if(!has[k]) continue;
		if(nb[k] >= 0) ld4(&fz[nb[k]*W], 0, un[k]);
		else {
			const double4 q = ghost_prim_of_cell<MF>(M, P, B, c, -2 - nb[k]);
			un[k][0] = q.x; un[k][1] = q.y; un[k][2] = q.z; un[k][3] = q.w;
		}
	}
	double lim[4];
	cell_limiter<LIM == 2>(uc, g, un, gp, has, rcc, eps2, lim);
	#pragma unroll
	for(int iv = 0; iv < 4; iv++) { g[iv*2+0] = lim[iv]*g[iv*2+0]; g[iv*2+1] = lim[iv]*g[iv*2+1]; }
}

/// the modified-average viscous flux of one face in the fused residual (gasdyn.hpp viscous_flux_core's
/// arithmetic, same operations in the same order, so bitwise its result), streamed from the staged LDS
/// rows variable by variable: first the temperature terms (density and pressure values and gradients),
/// then the velocity terms, each group read after a compiler fence, so only one group's LDS values are
/// live at a time instead of both cells' full rows (24 doubles) -- register pressure. The density
/// face gradient (unused by the flux) is not formed. Boundary face: rowj = nullptr, the right state is
/// the ghost primitive state gpr and the right gradient the cell's own.
__device__ __forceinline__ void fz_viscous(const Gas& G, const double* rowi, const double* rowj, const double4 gpr,
                                           double4 vg, const double* n, double muRe, const double* va, double* vf)
{
	const double* gsrc = rowj ? rowj : rowi;          // right gradient: the boundary cell's own
	// the face's unit vector between the centres (vg: left xy, right xy) and their distance (0 + dx^2 + dy^2,
	// correctly rounded root and quotients; reading them per slot from HBM was slower)
	double dr[2], dist = 0;
	dr[0] = vg.z - vg.x; dist += dr[0]*dr[0];
	dr[1] = vg.w - vg.y; dist += dr[1]*dr[1];
	dist = sqrt_rn(dist);
	dr[0] = div_rn(dr[0], dist); dr[1] = div_rn(dr[1], dist);
	double grad[2][4];
	{   // temperature: T and dT of each side, formed per staged row in phase 1 (fz_row_temperature); a
		// boundary face's right side is the ghost state with the cell's own gradients, formed here
		__asm__ volatile("" ::: "memory");
		const double2 tgl = *reinterpret_cast<const double2*>(rowi + 14);
		const double gL[2] = {tgl.y, rowi[16]}, tl = tgl.x;
		double gR[2], tr;
		if(rowj) {
			const double2 tgr = *reinterpret_cast<const double2*>(rowj + 14);
			gR[0] = tgr.y; gR[1] = rowj[16]; tr = tgr.x;
		} else {
			const double rrr = gpr.x, prr = gpr.w;
			for(int j = 0; j < 2; j++) gR[j] = grad_temperature(G, rrr, gsrc[4 + 0*2 + j], prr, gsrc[4 + 3*2 + j]);
			tr = temperature(G, rrr, prr);
		}
		double davg[2];
		davg[0] = 0.5*(gL[0] + gR[0]);
		davg[1] = 0.5*(gL[1] + gR[1]);
		const double corr = div_rn(tr-tl, dist);
		const double ddr = dot2(davg,dr);
		grad[0][3] = davg[0] - ddr*dr[0] + corr*dr[0];
		grad[1][3] = davg[1] - ddr*dr[1] + corr*dr[1];
	}
	#pragma unroll
	for(int i = 1; i < 3; i++) {   // velocity components
		__asm__ volatile("" ::: "memory");
		const double tl = rowi[i], tr = rowj ? rowj[i] : (i == 1 ? gpr.y : gpr.z);
		double davg[2];
		davg[0] = 0.5*(rowi[4 + i*2 + 0] + gsrc[4 + i*2 + 0]);
		davg[1] = 0.5*(rowi[4 + i*2 + 1] + gsrc[4 + i*2 + 1]);
		const double corr = div_rn(tr-tl, dist);
		const double ddr = dot2(davg,dr);
		grad[0][i] = davg[0] - ddr*dr[0] + corr*dr[0];
		grad[1][i] = davg[1] - ddr*dr[1] + corr*dr[1];
	}
	const double kd = div_rcp(muRe, G.kden, G.rkden);
	double ldiv = 0;
	ldiv += grad[0][1]; ldiv += grad[1][2];
	ldiv *= 2.0/3.0*muRe;
	// s[i][i] = muRe*(g + g) - ldiv: muRe*(2g) = 2 RN(muRe g) exactly, so one fma with the factor 2
	double s[2][2];
	s[0][0] = __builtin_fma(muRe*grad[0][1], 2.0, -ldiv); s[0][1] = muRe*(grad[0][2] + grad[1][1]);
	s[1][0] = muRe*(grad[1][1] + grad[0][2]); s[1][1] = __builtin_fma(muRe*grad[1][2], 2.0, -ldiv);
	vf[0] = 0;
	for(int i = 0; i < 2; i++) { double t = 0; t -= s[i][0]*n[0]; t -= s[i][1]*n[1]; vf[i+1] = t; }
	double e = 0;
	for(int i = 0; i < 2; i++) {
		double comp = 0;
		comp += s[i][0]*va[0]; comp += s[i][1]*va[1];
		comp += kd*grad[i][3];
		e -= comp * n[i];
	}
	vf[3] = e;
}

/// one patch of the fused residual: uniform (scalar) metadata
struct FzPatch { int p, s0, s1, c0, c1, nc, e0, nl, ng; const uint2* gnbr; const int* gbf; };
/// what one thread loads for its patch before phase 0: its first staged row (state, centre), the
/// neighbour list and WLS inverse of the gradient it computes first, and the geometry of its face
struct FzPre { int cf; double ua[4]; double2 rca; int4 nb4a; int2 lrl; double2 nn; double len;
               double2 gpa[4]; double eps2a; };     // gpa, eps2a: limited reconstructions' first-row inputs

__device__ __forceinline__ FzPatch fz_patch(const DevMesh& M, const SweepBuffers& B, int pi)
{
	FzPatch q;
	q.p = B.plist ? B.plist[pi] : pi;
	q.s0 = M.patch_slot[q.p]; q.s1 = M.patch_slot[q.p+1];
	q.c0 = M.patch_cell[q.p]; q.c1 = M.patch_cell[q.p+1];
	q.nc = q.c1 - q.c0;
	q.e0 = M.fz_ext_start[q.p];
	q.nl = q.nc + (M.fz_ext_start[q.p+1] - q.e0);    // staged rows: patch, ring 1, ring 2
	q.ng = q.nc + M.fz_n1[q.p];                       // rows whose gradients the patch computes
	q.gnbr = M.fz_gnbr16 + M.fz_g_start[q.p];
	q.gbf = M.fz_gbf + M.fz_gbf_start[q.p];
	return q;
}
/// a gradient row's four packed neighbour codes (layout.hpp fz_gnbr16) as patch-local index,
/// -2-bf (boundary face) or -1 (none)
__device__ __forceinline__ int fz_nbr_code(unsigned x, const int* gbf)
{
	if(x == 0xFFFFu) return -1;
	if(x & 0x8000u) return -2 - gbf[x & 0x7FFFu];
	return static_cast<int>(x);
}
__device__ __forceinline__ int4 fz_nbrs(const FzPatch& q, int i)
{
	const uint2 v = q.gnbr[i];
	return make_int4(fz_nbr_code(v.x & 0xFFFFu, q.gbf), fz_nbr_code(v.x >> 16, q.gbf),
	                 fz_nbr_code(v.y & 0xFFFFu, q.gbf), fz_nbr_code(v.y >> 16, q.gbf));
}
__device__ __forceinline__ int fz_cell(const DevMesh& M, const FzPatch& q, int i)
{
	return i < q.nc ? q.c0 + i : M.fz_ext[q.e0 + (i - q.nc)];
}
/// the loads of FzPre (a.cf already set): the staged row and the face
template <bool MF>
__device__ __forceinline__ void fz_load_rows(const DevMesh& M, const SweepBuffers& B, const FzPatch& q, int t, FzPre& a)
{
	a.ua[0] = a.ua[1] = a.ua[2] = a.ua[3] = 0.0;
	a.rca = make_double2(0, 0);
	if(t < q.nl) { ld_state<MF>(B, a.cf, a.ua); a.rca = M.rc[a.cf]; }
	const int s = q.s0 + t;
	a.lrl = make_int2(0, -1); a.nn = make_double2(0, 0); a.len = 0;
	if(s < q.s1) {
		const unsigned v = M.fz_slot_lr16[s];    // R 0xFFFF: boundary face (bf from slot_LR)
		a.lrl = make_int2(static_cast<int>(v & 0xFFFFu), (v >> 16) == 0xFFFFu ? -2 : static_cast<int>(v >> 16));
		a.nn = M.slot_n[s]; a.len = M.slot_len[s];
	}
}
/// the gradient inputs of the thread's first gradient row
__device__ __forceinline__ void fz_load_grad(const DevMesh& M, const FzPatch& q, int t, FzPre& a)
{
	a.nb4a = make_int4(-1, -1, -1, -1);
	if(t < q.ng && a.cf < M.nown) a.nb4a = fz_nbrs(q, t);
}

/// one patch (512 threads): phase 0 stages the primitive states and centres of the patch, ring-1 and
/// ring-2 cells in LDS; phase 1 computes the WLS gradients of the patch and ring-1 cells; phase 2 one
/// face per thread (reconstruction, flux, spectral radii); then the fluxes go through LDS and every
/// cell sums its faces in reference order. hookA runs at the start of phase 1, hookB after the face
/// work (points at which a caller may issue loads of later work).
template <int FLUX, int REC, bool DT, int VISC, int LIM, typename HA, typename HB>
__device__ __forceinline__ void fz_body(const DevMesh& M, const DevPhys& P, const SweepBuffers& B, double* fz,
                                        const FzPatch& q, const FzPre& a, HA&& hookA, HB&& hookB)
{
	const Gas& G = P.gas;
	const int t = static_cast<int>(threadIdx.x);
	const int s = q.s0 + t;
	constexpr int W = fz_w<VISC>();

	// phase 0: primitive states and centres of the staged cells
	if(t < q.nl) stage_row(G, &fz[t*W], a.ua, a.rca);
	for(int i = t + SLOTS_MAX; i < q.nl; i += SLOTS_MAX) {
		const int c = fz_cell(M, q, i);
		double b[4];
		ld_state<!DT>(B, c, b);
		stage_row(G, &fz[i*W], b, M.rc[c]);
	}
	__syncthreads();

	// phase 1: WLS gradients of the patch and ring-1 cells from the staged states
	// (k_prep_grad_wls arithmetic, neighbours in the same ascending reference face order)
	hookA();
	if(t < q.ng) fused_wls_row<LIM, W, !DT>(M, P, B, fz, &fz[t*W], a.cf, a.nb4a, LIM ? a.gpa : nullptr, a.eps2a);
	for(int i = t + SLOTS_MAX; i < q.ng; i += SLOTS_MAX) {
		const int c = fz_cell(M, q, i);
		fused_wls_row<LIM, W, !DT>(M, P, B, fz, &fz[i*W], c, c < M.nown ? fz_nbrs(q, i) : make_int4(-1, -1, -1, -1));
	}
	__syncthreads();

	// phase 2: one face per thread (k_sweep arithmetic)
	double f[4] = {0, 0, 0, 0};
	double sri = 0, srj = 0;
	if(s < q.s1) {
		const int2 lrl = a.lrl;
		const double2 nn = a.nn;
		const double flen = a.len;
		const double n[2] = {nn.x, nn.y};
		const bool bnd = lrl.y < -1;
		int bf = 0, bcell = 0;          // boundary face: its index and cell from the global slot
		if(bnd) { const int2 g = M.slot_LR[s]; bf = g.y - M.ncell; bcell = g.x; }
		double ul[4], ur[4];
		const double* rowi = &fz[lrl.x*W];
		const double2 ri = *reinterpret_cast<const double2*>(rowi + 12);
		double ui[4], gi[8];
		ld4(rowi, 0, ui);
		ld8(rowi + 4, 0, gi);
		if(REC == SR_MUSCL) {
			if(!bnd) {
				const double* rowj = &fz[lrl.y*W];
				const double2 rj = *reinterpret_cast<const double2*>(rowj + 12);
				double uj[4], gj[8];
				ld4(rowj, 0, uj);
				ld8(rowj + 4, 0, gj);
				const double dx = rj.x-ri.x, dy = rj.y-ri.y;
				#pragma unroll
				for(int i = 0; i < 4; i++) {
					double dl = mul0(gi[i*2], dx); dl += gi[i*2+1]*dy;
					double dr = mul0(gj[i*2], dx); dr += gj[i*2+1]*dy;
					const double du = uj[i] - ui[i];
					const double dm = twice_minus(dl, du);
					const double dp = twice_minus(dr, du);
					ul[i] = muscl_left(ui[i], uj[i], dm, muscl_phi(dm, du));
					ur[i] = muscl_right(ui[i], uj[i], dp, muscl_phi(dp, du));
				}
				prim2cons(G, ul, ul);
				prim2cons(G, ur, ur);
			} else {
				// ghost of the cell value (k_prep_grad_wls / k_prep_bfaces arithmetic)
				const double4 gp = ghost_prim_of_cell<!DT>(M, P, B, bcell, bf);
				const double uj[4] = {gp.x, gp.y, gp.z, gp.w};
				const double2 rj = M.bf_rcbp[bf];
				const double dx = rj.x-ri.x, dy = rj.y-ri.y;
				#pragma unroll
				for(int i = 0; i < 4; i++) {
					double dl = mul0(gi[i*2], dx); dl += gi[i*2+1]*dy;
					const double du = uj[i] - ui[i];
					const double dm = twice_minus(dl, du);
					ul[i] = muscl_left(ui[i], uj[i], dm, muscl_phi(dm, du));
				}
				prim2cons(G, ul, ul);
				ghost_c(P, M.bf_bc[bf], ul, n, ur);
			}
		} else {  // unlimited linear
			const double2 gp = M.slot_gr[s];
			#pragma unroll
			for(int i = 0; i < 4; i++) {
				double v = ui[i];
				v += 1.0*gi[i*2]*(gp.x - ri.x);
				v += 1.0*gi[i*2+1]*(gp.y - ri.y);
				ul[i] = v;
			}
			prim2cons(G, ul, ul);
			if(!bnd) {
				const double* rowj = &fz[lrl.y*W];
				const double2 rj = *reinterpret_cast<const double2*>(rowj + 12);
				double uj[4], gj[8];
				ld4(rowj, 0, uj);
				ld8(rowj + 4, 0, gj);
				#pragma unroll
				for(int i = 0; i < 4; i++) {
					double v = uj[i];
					v += 1.0*gj[i*2]*(gp.x - rj.x);
					v += 1.0*gj[i*2+1]*(gp.y - rj.y);
					ur[i] = v;
				}
				prim2cons(G, ur, ur);
			} else {
				ghost_c(P, M.bf_bc[bf], ul, n, ur);
			}
		}
		inviscid_flux_len<FLUX>(G, ul, ur, n, flen, f);
		// Sutherland viscosities of the two face states: the time step's and the viscous flux's
		// (viscous_face_terms forms the same two values), formed once
		double mui = 0, muj = 0;
		if(VISC != SV_NONE) {
			mui = VISC == SV_CONST ? G.rReinf : sutherland(G, ul);
			muj = VISC == SV_CONST ? G.rReinf : sutherland(G, ur);
		}
		if(DT) {
			const double ci = sound_speed_cons(G, ul), cj = sound_speed_cons(G, ur);
			const double vni = div_rn(dot2(&ul[1],n), ul[0]);
			const double vnj = div_rn(dot2(&ur[1],n), ur[0]);
			sri = (fabs(vni)+ci)*flen;
			srj = (fabs(vnj)+cj)*flen;
			if(VISC != SV_NONE) {
				const double coi = visc_coef(G, ul[0]), coj = visc_coef(G, ur[0]);   // std::max(4/(3 rho), g/rho)
				// a ghost cell's spectral radius is never summed (and its area is not stored)
				const int2 g = M.slot_LR[s];
				if(g.x < M.nown) sri += div_rn(div_rcp(coi*mui, G.Pr, G.rPr) * flen*flen, M.area[g.x]);
				if(!bnd && g.y < M.nown) srj += div_rn(div_rcp(coj*muj, G.Pr, G.rPr) * flen*flen, M.area[g.y]);
			}
		}
		if(VISC != SV_NONE) {
			// modified-average viscous flux, k_sweep's arithmetic, from the staged primitive states,
			// gradients and centres; a boundary face takes its cell's ghost primitive state (B.ug of
			// the staged path) and the cell's own gradient. Register pressure: the face states enter
			// only through the averaged viscosity and velocity, formed first (the time step above has
			// used the face states too), and the fence makes the cell rows fresh LDS reads instead of
			// the reconstruction's copies kept live through the inviscid flux -- 4 waves per SIMD
			double muRe, va[2];
			viscous_face_terms_mu<VISC == SV_CONST>(G, ul, ur, mui, muj, muRe, va);
			double4 gpr = make_double4(0, 0, 0, 0);
			const double* rowj = nullptr;
			double2 rr;
			if(bnd) { gpr = ghost_prim_of_cell<!DT>(M, P, B, bcell, bf); rr = M.bf_rcbp[bf]; }
			else { rowj = &fz[lrl.y*W]; rr = *reinterpret_cast<const double2*>(rowj + 12); }
			const double4 vg = make_double4(ri.x, ri.y, rr.x, rr.y);    // the two centres
			double vf[4] = {0, 0, 0, 0};
			fz_viscous(G, rowi, rowj, gpr, vg, n, muRe, va, vf);
			#pragma unroll
			for(int k = 0; k < 4; k++) f[k] += vf[k]*flen;
		}
	}
	hookB();
	// the cell's face list (and area) are requested before the two barriers of the flux staging,
	// once the face work no longer holds registers
	const int c = q.c0 + t;
	uint2 cs = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
	double carea = 0.0;
	if(c < q.c1) { cs = M.fz_cslot16[c]; if(DT) carea = M.area[c]; }
	__syncthreads();   // all staged rows read: reuse LDS for the face fluxes
	double* sf = fz;
	double* ssr = fz + 4*SLOTS_MAX;
	if(s < q.s1) {
		sf[0*SLOTS_MAX + t] = f[0]; sf[1*SLOTS_MAX + t] = f[1];
		sf[2*SLOTS_MAX + t] = f[2]; sf[3*SLOTS_MAX + t] = f[3];
		if(DT) { ssr[t] = sri; ssr[SLOTS_MAX + t] = srj; }
	}
	__syncthreads();

	if(c < q.c1) {
		double r[4];
		if(B.overwrite) { r[0] = r[1] = r[2] = r[3] = 0.0; }
		else ld4(B.r, c, r);
		double integ = 0.0;
		const unsigned e[4] = {cs.x & 0xFFFFu, cs.x >> 16, cs.y & 0xFFFFu, cs.y >> 16};
		#pragma unroll
		for(int k = 0; k < 4; k++) {
			if(e[k] == 0xFFFFu) break;
			const int ls = static_cast<int>(e[k] >> 1);     // patch-local slot
			if(e[k] & 1) {
				r[0] += sf[0*SLOTS_MAX + ls]; r[1] += sf[1*SLOTS_MAX + ls];
				r[2] += sf[2*SLOTS_MAX + ls]; r[3] += sf[3*SLOTS_MAX + ls];
				if(DT) integ += ssr[SLOTS_MAX + ls];
			} else {
				r[0] -= sf[0*SLOTS_MAX + ls]; r[1] -= sf[1*SLOTS_MAX + ls];
				r[2] -= sf[2*SLOTS_MAX + ls]; r[3] -= sf[3*SLOTS_MAX + ls];
				if(DT) integ += ssr[ls];
			}
		}
		if(!DT && B.mfx) {
			// y = mdt x + (-yg + res)/pert, k_mf_combine's arithmetic, with yg the sum just formed
			double x[4], rs[4];
			ld4(B.mfx, c, x);
			ld4(B.mfres, c, rs);
			const double d = B.mfmdt[c], pert = B.mfpm[1];
			#pragma unroll
			for(int i = 0; i < 4; i++) r[i] = d*x[i] + (-r[i] + rs[i])/pert;
		}
		st4(B.r, c, r);
		if(DT) B.dtm[c] = div_rn(carea, integ);
	}
}

// waves per SIMD the fused instantiations are compiled for (VGPR budgets 96 / 128 / 168); the layout
// caps the staged rows to match (layout.cpp fusedRowCap: 5 blocks of 32 KB LDS per CU)
#ifndef FVHIP_FUSED_WAVES
#define FVHIP_FUSED_WAVES 5          // inviscid, unlimited: 90 VGPRs
#endif
#ifndef FVHIP_FUSED_WAVES_LIM
#define FVHIP_FUSED_WAVES_LIM 4      // Barth-Jespersen / Venkatakrishnan: 124-126 VGPRs
#endif
#ifndef FVHIP_FUSED_WAVES_VISC
#define FVHIP_FUSED_WAVES_VISC 4     // viscous: 110-122 VGPRs (fz_viscous streams the LDS rows; 144-156 before)
#endif

template <int FLUX, int REC, bool DT, int VISC, int LIM>
__global__ void __launch_bounds__(SLOTS_MAX, VISC != SV_NONE ? FVHIP_FUSED_WAVES_VISC : (LIM ? FVHIP_FUSED_WAVES_LIM : FVHIP_FUSED_WAVES)) k_residual_wls(const DevMesh M, const DevPhys P, const SweepBuffers B)
{
	extern __shared__ __attribute__((aligned(16))) double fz[];
	const int np = B.plist ? B.pcount : M.npatch;
	const int t = static_cast<int>(threadIdx.x);
	const int q = (np + 7) >> 3;
	const int pi = (blockIdx.x & 7) * q + (blockIdx.x >> 3);
	if(pi >= np) return;
	const FzPatch cur = fz_patch(M, B, pi);
	FzPre pre;
	pre.cf = t < cur.nl ? fz_cell(M, cur, t) : 0;
	fz_load_rows<!DT>(M, B, cur, t, pre);
	fz_load_grad(M, cur, t, pre);
	pre.eps2a = 0.0;
	if(LIM) {   // the first row's face centres and eps^2, requested before the staging barrier
		// (owned gradient rows only: a ghost row's limiter values come with its gradient)
		const bool own = t < cur.ng && pre.cf < M.nown;
		fz_face_centres(M, own ? pre.cf : 0, pre.gpa);
		if(LIM == 2) pre.eps2a = M.venk_eps2[own ? pre.cf : 0];
	}
	fz_body<FLUX, REC, DT, VISC, LIM>(M, P, B, fz, cur, pre, []() {}, []() {});
}

// ------------------------------------------------------------------------------------------------
// misc
// ------------------------------------------------------------------------------------------------
__global__ void k_fill(double* p, double v, long long n)
{
	const long long i = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	if(i < n) p[i] = v;
}

__global__ void k_local_flux(int type, Gas G, int nf, const double* ul, const double* ur, const double* n, double* f)
{
	const int i = blockIdx.x*blockDim.x + threadIdx.x;
	if(i >= nf) return;
	double a[4], b[4], o[4];
	ld4(ul, i, a); ld4(ur, i, b);
	const double nn[2] = {n[2*i], n[2*i+1]};
	inviscid_flux_rt(type, G, a, b, nn, o);
	st4(f, i, o);
}

__global__ void k_gather(const int* perm, const double* src, double* dst, int n, int width)
{
	const long long i = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	if(i >= static_cast<long long>(n)*width) return;
	const int c = static_cast<int>(i / width), w = static_cast<int>(i % width);
	dst[i] = src[static_cast<size_t>(perm[c])*width + w];
}

/// dst row perm[c] = src row c (internal -> reference order, the inverse of k_gather)
__global__ void k_scatter(const int* perm, const double* src, double* dst, int n, int width)
{
	const long long i = static_cast<long long>(blockIdx.x)*blockDim.x + threadIdx.x;
	if(i >= static_cast<long long>(n)*width) return;
	const int c = static_cast<int>(i / width), w = static_cast<int>(i % width);
	dst[static_cast<size_t>(perm[c])*width + w] = src[i];
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
static inline int nblk(long long n, int b) { return static_cast<int>((n + b - 1)/b); }

void launch_prep(const DevMesh& M, const DevPhys& P, const double* u, double* up, double* ubc, double* ug,
                 bool cells, hipStream_t s)
{
	if(cells && M.nown > 0) k_prep_cells<<<nblk(M.nown,256), 256, 0, s>>>(M.nown, P.gas, u, up);
	if(M.nbface > 0) k_prep_bfaces<<<nblk(M.nbface,256), 256, 0, s>>>(M, P, u, ubc, ug);
}
void launch_grad_wls(const DevMesh& M, const double* up, const double* ug, double* grad, hipStream_t s)
{ if(M.nown > 0) k_grad_wls<<<nblk(M.nown,256), 256, 0, s>>>(M, up, ug, grad); }
void launch_prep_grad_wls(const DevMesh& M, const DevPhys& P, const double* u, double* up, double* ubc,
                          double* ug, double* grad, hipStream_t s, int c_begin, int c_end, int lim, double* phi)
{
	if(c_end < 0) c_end = M.nown;
	if(c_end <= c_begin) return;
	const dim3 g(xcd_blocks((c_end - c_begin + 255)/256)), b(256);
	if(lim == 1) k_prep_grad_wls<1><<<g, b, 0, s>>>(M, P, u, up, ubc, ug, grad, c_begin, c_end, phi);
	else if(lim == 2) k_prep_grad_wls<2><<<g, b, 0, s>>>(M, P, u, up, ubc, ug, grad, c_begin, c_end, phi);
	else k_prep_grad_wls<0><<<g, b, 0, s>>>(M, P, u, up, ubc, ug, grad, c_begin, c_end, phi);
}
void launch_grad_wls_list(const DevMesh& M, const DevPhys& P, const double* u, const int* list, int n,
                          double* grad, hipStream_t s)
{ if(n > 0) k_grad_wls_list<<<nblk(n,256), 256, 0, s>>>(M, P, u, list, n, grad); }
void launch_grad_gg(const DevMesh& M, const double* up, const double* ug, double* grad, hipStream_t s)
{ if(M.nown > 0) k_grad_gg<<<nblk(M.nown,256), 256, 0, s>>>(M, up, ug, grad); }
void launch_limiter(const DevMesh& M, const DevPhys& P, int venk, const double* up, const double* ug,
                    const double* grad, double* phi, hipStream_t s)
{
	if(M.nown <= 0) return;
	if(venk) k_limiter<true><<<nblk(M.nown,256), 256, 0, s>>>(M, up, ug, grad, phi);
	else     k_limiter<false><<<nblk(M.nown,256), 256, 0, s>>>(M, up, ug, grad, phi);
}

void launch_grad_ghost(const DevMesh& M, const DevPhys& P, const double* u, double* grad, hipStream_t s, int lim, double* phi)
{
	if(M.gg_n <= 0) return;
	if(lim && !phi) throw std::invalid_argument("launch_grad_ghost: limiter values need a phi buffer");
	if(lim == 2 && !M.gg_eps2) throw std::invalid_argument("launch_grad_ghost: Venkatakrishnan eps^2 of the ghosts missing");
	if(lim && !M.gg_gp) throw std::invalid_argument("launch_grad_ghost: ghost face centres missing");
	const int nb = (M.gg_n + 255)/256;
	if(lim == 2) k_grad_ghost<2><<<nb, 256, 0, s>>>(M, P, u, grad, phi);
	else if(lim == 1) k_grad_ghost<1><<<nb, 256, 0, s>>>(M, P, u, grad, phi);
	else k_grad_ghost<0><<<nb, 256, 0, s>>>(M, P, u, grad, phi);
}
void launch_weno(const DevMesh& M, const DevPhys& P, const double* grad, double* lgrad, hipStream_t s)
{ if(M.nown > 0) k_weno<<<nblk(M.nown,256), 256, 0, s>>>(M, P.limiter_param, grad, lgrad); }
void launch_fill(double* p, double v, long long n, hipStream_t s)
{ if(n > 0) k_fill<<<nblk(n,256), 256, 0, s>>>(p, v, n); }
void launch_local_flux(int flux, const Gas& G, int nf, const double* ul, const double* ur,
                       const double* n, double* f, hipStream_t s)
{ if(nf > 0) k_local_flux<<<nblk(nf,256), 256, 0, s>>>(flux, G, nf, ul, ur, n, f); }
/// parity-mode division and square root against the device's IEEE a/b and sqrt(a): out[i] =
/// {div_rn(a,b), a/b, sqrt_rn(a), sqrt(a)} (the check of gasdyn.hpp's bitwise claim)
__global__ void k_divsqrt_probe(int n, const double* __restrict__ a, const double* __restrict__ b, double* __restrict__ out)
{
	const int i = blockIdx.x*blockDim.x + threadIdx.x;
	if(i >= n) return;
	const double x = a[i], y = b[i];
	out[4*i+0] = div_rn(x, y);
	out[4*i+1] = x / y;
	out[4*i+2] = sqrt_rn(x);
	out[4*i+3] = sqrt(x);
}
void launch_divsqrt_probe(int n, const double* a, const double* b, double* out, hipStream_t s)
{ if(n > 0) k_divsqrt_probe<<<nblk(n,256), 256, 0, s>>>(n, a, b, out); }

void launch_gather_cells(const int* perm, const double* src, double* dst, int n, int width, hipStream_t s)
{ if(n > 0) k_gather<<<nblk(static_cast<long long>(n)*width,256), 256, 0, s>>>(perm, src, dst, n, width); }
void launch_scatter_cells(const int* perm, const double* src, double* dst, int n, int width, hipStream_t s)
{ if(n > 0) k_scatter<<<nblk(static_cast<long long>(n)*width,256), 256, 0, s>>>(perm, src, dst, n, width); }

// sweep dispatch over (flux, reconstruction, viscous, dt, phi)
typedef void (*SweepFn)(const DevMesh, const DevPhys, const SweepBuffers);

template <int FLUX, int REC, int VISC>
static SweepFn pick4(bool dt, bool phi) {
	if(REC == SR_LINEAR) {
		if(dt) return phi ? k_sweep<FLUX,REC,VISC,true,true> : k_sweep<FLUX,REC,VISC,true,false>;
		return phi ? k_sweep<FLUX,REC,VISC,false,true> : k_sweep<FLUX,REC,VISC,false,false>;
	}
	return dt ? k_sweep<FLUX,REC,VISC,true,false> : k_sweep<FLUX,REC,VISC,false,false>;
}
template <int FLUX, int REC>
static SweepFn pick3(int visc, bool dt, bool phi) {
	switch(visc) {
		case SV_NONE: return pick4<FLUX,REC,SV_NONE>(dt, phi);
		case SV_SUTHERLAND: return pick4<FLUX,REC,SV_SUTHERLAND>(dt, phi);
		default: return pick4<FLUX,REC,SV_CONST>(dt, phi);
	}
}
template <int FLUX>
static SweepFn pick2(int rec, int visc, bool dt, bool phi) {
	switch(rec) {
		case SR_FIRST: return pick3<FLUX,SR_FIRST>(visc, dt, phi);
		case SR_MUSCL: return pick3<FLUX,SR_MUSCL>(visc, dt, phi);
		default: return pick3<FLUX,SR_LINEAR>(visc, dt, phi);
	}
}

#ifdef FVHIP_FAST
static const char* kSweepNames[7] = {"k_sweep_fast<LLF>", "k_sweep_fast<VANLEER>", "k_sweep_fast<AUSM>",
                                     "k_sweep_fast<AUSMPLUS>", "k_sweep_fast<ROE>", "k_sweep_fast<HLL>",
                                     "k_sweep_fast<HLLC>"};
#else
static const char* kSweepNames[7] = {"k_sweep<LLF>", "k_sweep<VANLEER>", "k_sweep<AUSM>", "k_sweep<AUSMPLUS>",
                                     "k_sweep<ROE>", "k_sweep<HLL>", "k_sweep<HLLC>"};
#endif

const char* launch_sweep(const DevMesh& M, const DevPhys& P, const SweepBuffers& B, int flux, int rec,
                         int visc, bool dt, hipStream_t s)
{
	const bool phi = B.phi != nullptr;
	SweepFn fn;
	switch(flux) {
		case 0: fn = pick2<0>(rec, visc, dt, phi); break;
		case 1: fn = pick2<1>(rec, visc, dt, phi); break;
		case 2: fn = pick2<2>(rec, visc, dt, phi); break;
		case 3: fn = pick2<3>(rec, visc, dt, phi); break;
		case 4: fn = pick2<4>(rec, visc, dt, phi); break;
		case 5: fn = pick2<5>(rec, visc, dt, phi); break;
		default: fn = pick2<6>(rec, visc, dt, phi); break;
	}
	const int np = B.plist ? B.pcount : M.npatch;
	if(np > 0) hipLaunchKernelGGL(fn, dim3(8*((np + 7)/8)), dim3(SLOTS_MAX), 0, s, M, P, B);
	return kSweepNames[flux < 0 || flux > 6 ? 6 : flux];
}

// fused residual dispatch
typedef void (*FusedFn)(const DevMesh, const DevPhys, const SweepBuffers);
template <int FLUX, int VISC>
static FusedFn pickFused3(int rec, bool dt) {
	if(rec == SR_MUSCL) return dt ? k_residual_wls<FLUX,SR_MUSCL,true,VISC,0> : k_residual_wls<FLUX,SR_MUSCL,false,VISC,0>;
	return dt ? k_residual_wls<FLUX,SR_LINEAR,true,VISC,0> : k_residual_wls<FLUX,SR_LINEAR,false,VISC,0>;
}
/// lim: 0 none, 1 Barth-Jespersen, 2 Venkatakrishnan (inviscid; linear reconstruction of lim*g)
template <int FLUX>
static FusedFn pickFused(int rec, int visc, int lim, bool dt) {
	if(lim == 1) return dt ? k_residual_wls<FLUX,SR_LINEAR,true,SV_NONE,1> : k_residual_wls<FLUX,SR_LINEAR,false,SV_NONE,1>;
	if(lim == 2) return dt ? k_residual_wls<FLUX,SR_LINEAR,true,SV_NONE,2> : k_residual_wls<FLUX,SR_LINEAR,false,SV_NONE,2>;
	if(visc == SV_SUTHERLAND) return pickFused3<FLUX,SV_SUTHERLAND>(rec, dt);
	if(visc == SV_CONST) return pickFused3<FLUX,SV_CONST>(rec, dt);
	return pickFused3<FLUX,SV_NONE>(rec, dt);
}

#ifdef FVHIP_FAST
static const char* kFusedNames[7] = {"k_residual_wls_fast<LLF>", "k_residual_wls_fast<VANLEER>",
	"k_residual_wls_fast<AUSM>", "k_residual_wls_fast<AUSMPLUS>", "k_residual_wls_fast<ROE>",
	"k_residual_wls_fast<HLL>", "k_residual_wls_fast<HLLC>"};
#else
static const char* kFusedNames[7] = {"k_residual_wls<LLF>", "k_residual_wls<VANLEER>", "k_residual_wls<AUSM>",
	"k_residual_wls<AUSMPLUS>", "k_residual_wls<ROE>", "k_residual_wls<HLL>", "k_residual_wls<HLLC>"};
#endif

const char* launch_residual_wls(const DevMesh& M, const DevPhys& P, const SweepBuffers& B, int flux, int rec,
                                int visc, int lim, bool dt, hipStream_t s)
{
	FusedFn fn;
	switch(flux) {
		case 0: fn = pickFused<0>(rec, visc, lim, dt); break;
		case 1: fn = pickFused<1>(rec, visc, lim, dt); break;
		case 2: fn = pickFused<2>(rec, visc, lim, dt); break;
		case 3: fn = pickFused<3>(rec, visc, lim, dt); break;
		case 4: fn = pickFused<4>(rec, visc, lim, dt); break;
		case 5: fn = pickFused<5>(rec, visc, lim, dt); break;
		default: fn = pickFused<6>(rec, visc, lim, dt); break;
	}
	const size_t W = visc != SV_NONE ? FZW_VISC : FZW;
	const size_t lds = std::max(static_cast<size_t>(M.fz_max_cells)*W, static_cast<size_t>(6*SLOTS_MAX))*sizeof(double);
	// raise the dynamic-LDS limit once per instantiation and device to the largest patch the layout
	// allows (hipFuncSetAttribute is a host-side runtime call: not on every launch)
	{
		static std::mutex mu;
		static std::set<std::pair<const void*, int>> configured;
		int dev = 0;
		if(hipGetDevice(&dev) != hipSuccess) throw std::runtime_error("k_residual_wls: hipGetDevice failed");
		std::lock_guard<std::mutex> lock(mu);
		if(configured.insert({reinterpret_cast<const void*>(fn), dev}).second) {
			const size_t maxlds = std::max(static_cast<size_t>(FUSED_LDS_CELLS)*W, static_cast<size_t>(6*SLOTS_MAX))*sizeof(double);
			const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
			                                         hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(maxlds));
			if(e != hipSuccess) {
				configured.erase({reinterpret_cast<const void*>(fn), dev});
				throw std::runtime_error(std::string("k_residual_wls: raising the dynamic LDS limit failed: ")
				                         + hipGetErrorString(e));
			}
		}
	}
	const int np = B.plist ? B.pcount : M.npatch;
	if(np > 0) hipLaunchKernelGGL(fn, dim3(8*((np + 7)/8)), dim3(SLOTS_MAX), lds, s, M, P, B);
	return kFusedNames[flux < 0 || flux > 6 ? 6 : flux];
}

}
}
