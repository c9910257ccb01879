/** \file gasdyn.hpp
 * \brief Point-wise gas dynamics for the MI355X face sweep: ideal-gas relations, the seven
 *   numerical inviscid fluxes, boundary ghost states and the viscous face flux.
 *
 * Every expression keeps the reference's operation order and association, so that with
 * -ffp-contract=off the device reproduces the reference's IEEE results (division and sqrt are
 * correctly rounded on gfx950 in the default float mode). Sources (under /root/reference/src):
 *   physics/aphysics_defs.hpp:13-487     ideal-gas relations
 *   spatial/anumericalflux.cpp:40-61, 202-250, 264-315, 479-553, 667-732, 973-1007, 1069-1228
 *   spatial/anumericalflux.hpp:175-189   Roe averages
 *   spatial/abc.cpp:41-437               boundary ghost states
 *   physics/viscousphysics.cpp:14-122, spatial/aspatial.cpp:172-205   viscous face flux
 * Marked __host__ __device__ so the same code is also compiled into the host self-check.
 */
#ifndef FVHIP_GASDYN_HPP
#define FVHIP_GASDYN_HPP

#include <hip/hip_runtime.h>
#include <cmath>

#define FVHIP_HD __host__ __device__ __forceinline__

namespace fvhip {
namespace gd {

/// Gas constants (IdealGasPhysics members, aphysics.hpp; sC = 110.5, aphysics.cpp:19), and run-time
/// constants of the viscous terms the host forms once, each with the reference's arithmetic, so that a
/// division by a constant becomes div_rcp (Markstein's correction with the correctly rounded
/// reciprocal: the same bits as the division, 3 instead of 8 instructions) -- build with make_gas
struct Gas {
	double g, Minf, Tinf, Reinf, Pr, sC;
	double rgm1;     ///< 1/(g-1) correctly rounded (host division), for div_rcp by g-1 on the device
	double sCT;      ///< sC/Tinf (getViscosityCoeffFromTemperature, aphysics_defs.hpp:411)
	double sCT1;     ///< 1.0 + sC/Tinf
	double rReinf;   ///< 1/Reinf (also the constant viscosity, aphysics_defs.hpp:444)
	double kden;     ///< Minf*Minf*(g-1.0)*Pr (getThermalConductivityFromViscosity, :449)
	double rkden;    ///< 1/kden
	double rPr;      ///< 1/Pr
	double g43;      ///< 1 when g > 4/3 with a margin far above rounding (visc_coef), else 0
};
/// Gas with its derived constants (host IEEE arithmetic in the reference's association order)
inline Gas make_gas(double g, double Minf, double Tinf, double Reinf, double Pr) {
	Gas G{g, Minf, Tinf, Reinf, Pr, 110.5, 1.0/(g - 1.0), 0, 0, 0, 0, 0, 0};
	G.sCT = G.sC/G.Tinf;
	G.sCT1 = 1.0 + G.sCT;
	G.rReinf = 1.0/G.Reinf;
	G.kden = G.Minf*G.Minf*(G.g-1.0)*G.Pr;
	G.rkden = 1.0/G.kden;
	G.rPr = 1.0/G.Pr;
	G.g43 = G.g > 4.0/3.0*(1.0 + 1e-9) ? 1.0 : 0.0;
	return G;
}

/// `0 + a*b`: the first term of a sum the reference accumulates from zero. On the device this is
/// fma(a, b, +0) -- one instruction instead of a multiply and an add. fma rounds a*b once and adds
/// +0, which is bitwise 0 + RN(a*b) for all a, b (a zero product of either sign gives +0 both ways)
/// except a nonzero product below half the smallest subnormal (|a*b| < 2^-1075), where fma keeps the
/// product's sign on the zero.
FVHIP_HD double mul0(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FVHIP_FAST)
	return __builtin_fma(a, b, 0.0);
#else
	double d = 0; d += a*b; return d;
#endif
}
/// `2*a - b` as fma(a, 2, -b): 2a is exact, so the single rounding is the same (bitwise, short of
/// 2a overflowing)
FVHIP_HD double twice_minus(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FVHIP_FAST)
	return __builtin_fma(a, 2.0, -b);
#else
	return 2.0*a - b;
#endif
}

FVHIP_HD double dot2(const double* a, const double* b) { double d = mul0(a[0], b[0]); d += a[1]*b[1]; return d; }

/// `c + s*p` for a power of two s (here +-0.5, +-0.25), which scales exactly: on the device one fma,
/// bitwise c + RN(s*p) short of s*p leaving the normal range. The reference's `c - 0.5*a*b` and
/// `c + x/4.0*y` forms are this with p = RN(a*b) resp. RN(x*y): (0.5*a)*b is exactly 0.5*RN(a*b) and
/// (x/4)*y exactly RN(x*y)/4 -- one multiply less per term
FVHIP_HD double add_pow2(double c, double p, double s) {
#if defined(__HIP_DEVICE_COMPILE__)
	return __builtin_fma(p, s, c);
#else
	return c + s*p;
#endif
}

/// a/b and sqrt(x), correctly rounded, for the parity kernels. On the device these are the compiler's
/// own f64 sequences -- division: v_rcp, two Newton steps, Markstein's correction; square root:
/// v_rsq and Goldschmidt steps -- without their range scaling and special-value fix-ups
/// (v_div_scale / v_div_fmas / v_div_fixup; ldexp and class selects). Inside their domain -- |a|, |b|
/// and |a/b| in [2^-1000, 2^1000] for the division, x in [2^-766, 2^1000] for the root (below 2^-767
/// the IEEE root first scales x by 2^256; sqrt_rn may then be one ulp off) -- they execute the same
/// instructions on the same values, i.e. return bitwise a/b and sqrt(x) (tests/test_gpu_edge.py
/// test_div_sqrt_rn_domain), in 8 instead of 11 and 10 instead of 19 instructions (the sweep is FP64-
/// issue bound). Every division and root of the sweep lies far inside (densities, pressures, sound
/// speeds, eps-shifted limiter sums, squared distances: 1e-12..1e12); an overflowing quotient gives NaN
/// instead of inf. Host builds and the fast-math kernels use / and sqrt.
FVHIP_HD double div_rn(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FVHIP_FAST)
	double r = __builtin_amdgcn_rcp(b);
	double e = fma(-b, r, 1.0);
	r = fma(r, e, r);
	e = fma(-b, r, 1.0);
	r = fma(r, e, r);
	const double q = a*r;
	e = fma(-b, q, a);
	return fma(e, r, q);
#else
	return a/b;
#endif
}
FVHIP_HD double sqrt_rn(double x) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FVHIP_FAST)
	const double y = __builtin_amdgcn_rsq(x);
	double g = x*y, h = y*0.5;
	const double r = fma(-h, g, 0.5);
	g = fma(g, r, g);
	h = fma(h, r, h);
	double d = fma(-g, g, x);
	g = fma(d, h, g);
	d = fma(-g, g, x);
	return fma(d, h, g);
#else
	return sqrt(x);
#endif
}

FVHIP_HD void directional_flux(const Gas& G, const double* uc, const double* n, double vn, double p, double* f) {
	f[0] = vn*uc[0];
	f[1] = vn*uc[1] + p*n[0];
	f[2] = vn*uc[2] + p*n[1];
	f[3] = vn*(uc[3] + p);
}

/// getVarsFromConserved: velocity, normal velocity, pressure, total enthalpy
FVHIP_HD void flow_vars(const Gas& G, const double* uc, const double* n, double* v, double& vn, double& p, double& H) {
	v[0] = div_rn(uc[1], uc[0]);
	v[1] = div_rn(uc[2], uc[0]);
	vn = dot2(v,n);
	const double vm2 = dot2(v,v);
	p = (G.g-1.0)*add_pow2(uc[3], uc[0]*vm2, -0.5);           // uc[3] - 0.5*uc[0]*vm2
	H = div_rn(uc[3]+p, uc[0]);
}

FVHIP_HD double pressure_cons(const Gas& G, const double* uc) {
	return (G.g-1.0)*add_pow2(uc[3], div_rn(dot2(&uc[1],&uc[1]), uc[0]), -0.5);   // uc[3] - (0.5*|m|^2)/uc[0]
}
FVHIP_HD double sound_speed(const Gas& G, double rho, double p) { return sqrt_rn(div_rn(G.g * p, rho)); }
FVHIP_HD double sound_speed_cons(const Gas& G, const double* uc) { return sound_speed(G, uc[0], pressure_cons(G, uc)); }
FVHIP_HD double temperature(const Gas& G, double rho, double p) { return div_rn(p, rho) * G.g*G.Minf*G.Minf; }
/// a/b given r = RN(1/b): Markstein's correction alone (q = RN(a r), e = a - b q exact by fma,
/// RN(q + e r) is a/b correctly rounded when r is the correctly rounded reciprocal) -- for divisions by
/// a run-time constant, whose reciprocal the host computes once
FVHIP_HD double div_rcp(double a, double b, double r) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FVHIP_FAST)
	const double q = a*r;
	const double e = fma(-b, q, a);
	return fma(e, r, q);
#else
	return a/b;
#endif
}
FVHIP_HD double energy_from_pressure(const Gas& G, double p, double d, double vm2) {
	return add_pow2(div_rcp(p, G.g-1.0, G.rgm1), d*vm2, 0.5);          // p/(g-1) + 0.5*d*vm2
}
FVHIP_HD double energy_from_temperature(const Gas& G, double T, double d, double vm2) {
	return d * (div_rn(T, G.g*(G.g-1.0)*G.Minf*G.Minf) + 0.5*vm2);
}
FVHIP_HD double freestream_pressure(const Gas& G) { return div_rn(1.0, G.g*G.Minf*G.Minf); }

/// conserved -> (rho, vx, vy, p); in-place safe
FVHIP_HD void cons2prim(const Gas& G, const double* uc, double* up) {
	const double rho = uc[0];
	const double p = pressure_cons(G, uc);
	const double vx = div_rn(uc[1], rho), vy = div_rn(uc[2], rho);
	up[0] = rho; up[1] = vx; up[2] = vy; up[3] = p;
}
/// (rho, vx, vy, p) -> conserved; in-place safe
FVHIP_HD void prim2cons(const Gas& G, const double* up, double* uc) {
	const double rhoE = energy_from_pressure(G, up[3], up[0], dot2(&up[1],&up[1]));
	const double r = up[0];
	uc[0] = r; uc[1] = r*up[1]; uc[2] = r*up[2]; uc[3] = rhoE;
}
/// conserved -> (rho, vx, vy, T)
FVHIP_HD void cons2prim2(const Gas& G, const double* uc, double* up) {
	const double p = pressure_cons(G, uc);
	up[0] = uc[0]; up[1] = div_rn(uc[1], uc[0]); up[2] = div_rn(uc[2], uc[0]);
	up[3] = temperature(G, uc[0], p);
}
FVHIP_HD double grad_temperature(const Gas& G, double rho, double grho, double p, double gp) {
	return div_rn(gp*rho - p*grho, rho*rho) * G.g*G.Minf*G.Minf;
}
/// T^1.5 of Sutherland's law. The reference calls std::pow(T,1.5); device code forms T*sqrt(T)
/// (within 2 ulp of it; the device pow is a ~150-instruction log/exp sequence and not glibc's bits
/// either, so Sutherland terms are compared to the reference to 1e-12 in both cases) -- three of them
/// per face in the viscous sweep.
FVHIP_HD double pow15(double T) {
#if defined(__HIP_DEVICE_COMPILE__)
	return T*sqrt_rn(T);
#else
	return pow(T, 1.5);
#endif
}
/// std::max(4.0/(3*rho), g/rho) of the viscous spectral radius (flow_spatial.cpp:612-613). For g > 4/3
/// and rho > 0 the second is always the larger -- the exact quotients differ by the factor 3g/4 (1.05
/// for air), the roundings (RN(3 rho), then RN(4/.)) by at most 2^-52 relative, and RN is monotone -- so
/// the max is g/rho bitwise and the first division is skipped; otherwise both are formed as written
FVHIP_HD double visc_coef(const Gas& G, double rho) {
	const double b = div_rn(G.g, rho);
	if(G.g43 != 0.0 && rho > 0) return b;
	const double a = div_rn(4.0, 3*rho);
	return (a < b) ? b : a;
}
FVHIP_HD double sutherland(const Gas& G, const double* uc) {
	const double T = temperature(G, uc[0], pressure_cons(G, uc));
	return div_rcp(div_rn(G.sCT1, T+G.sCT) * pow15(T), G.Reinf, G.rReinf);
}

/// Roe averages (anumericalflux.hpp:175-189)
struct RoeAvg { double R, rho, v[2], vm2, vn, H, c; };
FVHIP_HD RoeAvg roe_average(const Gas& G, const double* ul, const double* ur, const double* n,
                            const double* vi, double Hi, const double* vj, double Hj) {
	RoeAvg a;
	a.R = sqrt_rn(div_rn(ur[0], ul[0]));
	a.rho = a.R*ul[0];
	a.v[0] = div_rn(a.R*vj[0] + vi[0], a.R + 1.0);
	a.v[1] = div_rn(a.R*vj[1] + vi[1], a.R + 1.0);
	a.H = div_rn(a.R*Hj + Hi, a.R + 1.0);
	a.vm2 = dot2(a.v,a.v);
	a.vn = dot2(a.v,n);
	a.c = sqrt_rn( (G.g-1.0)*add_pow2(a.H, a.vm2, -0.5) );       // (g-1)*(H - vm2*0.5)
	return a;
}

// ---------------------------------------------------------------------------------------------
// Numerical fluxes. Output: flux per unit length along unit normal n (L -> R).
// ---------------------------------------------------------------------------------------------

/// HALVE = false: f = (...) without the final 0.5*(...) (inviscid_flux_len folds it into the length)
template <bool HALVE = true>
FVHIP_HD void flux_llf(const Gas& G, const double* ul, const double* ur, const double* n, double* f) {
	double vi[2], vj[2], vni, vnj, pi, pj, Hi, Hj;
	flow_vars(G, ul, n, vi, vni, pi, Hi);
	flow_vars(G, ur, n, vj, vnj, pj, Hj);
	const double ci = sound_speed(G, ul[0], pi), cj = sound_speed(G, ur[0], pj);
	const double si = fabs(vni)+ci, sj = fabs(vnj)+cj;
	const double eig = si > sj ? si : sj;
	// getDirectionalFluxFromConserved recomputes vn and p from the conserved state (aphysics.cpp:28-35)
	double fl[4], fr[4];
	{
		const double vn = div_rn(dot2(&ul[1],n), ul[0]);
		const double p = pressure_cons(G, ul);
		directional_flux(G, ul, n, vn, p, fl);
	}
	{
		const double vn = div_rn(dot2(&ur[1],n), ur[0]);
		const double p = pressure_cons(G, ur);
		directional_flux(G, ur, n, vn, p, fr);
	}
	for(int k = 0; k < 4; k++) {
		const double s = fl[k] + fr[k] - eig*(ur[k]-ul[k]);
		f[k] = HALVE ? 0.5*s : s;
	}
}

FVHIP_HD double sq(double x) { return x*x; }   // std::pow(x,2) folds to x*x

FVHIP_HD void flux_vanleer(const Gas& G, const double* ul, const double* ur, const double* n, double* f) {
	const double g = G.g;
	double vi[2], vj[2], vni, vnj, pi, pj, Hi, Hj;
	flow_vars(G, ul, n, vi, vni, pi, Hi);
	flow_vars(G, ur, n, vj, vnj, pj, Hj);
	const double ci = sound_speed(G, ul[0], pi), cj = sound_speed(G, ur[0], pj);
	const double Mni = div_rn(vni, ci), Mnj = div_rn(vnj, cj);
	double fp[4], fm[4];
	if(Mni < -1.0) { fp[0] = fp[1] = fp[2] = fp[3] = 0; }
	else if(Mni > 1.0) directional_flux(G, ul, n, vni, pi, fp);
	else {
		const double vmags = sq(ul[1]/ul[0]) + sq(ul[2]/ul[0]);
		fp[0] = ul[0]*ci*sq(Mni+1)/4.0;
		fp[1] = fp[0] * (ul[1]/ul[0] + n[0]*(2.0*ci - vni)/g);
		fp[2] = fp[0] * (ul[2]/ul[0] + n[1]*(2.0*ci - vni)/g);
		fp[3] = fp[0] * ( (vmags - vni*vni)/2.0 + sq((g-1)*vni+2*ci)/(2*(g*g-1)) );
	}
	if(Mnj > 1.0) { fm[0] = fm[1] = fm[2] = fm[3] = 0; }
	else if(Mnj < -1.0) directional_flux(G, ur, n, vnj, pj, fm);
	else {
		const double vmags = sq(ur[1]/ur[0]) + sq(ur[2]/ur[0]);
		fm[0] = -ur[0]*cj*sq(Mnj-1)/4.0;
		fm[1] = fm[0] * (ur[1]/ur[0] + n[0]*(-2.0*cj - vnj)/g);
		fm[2] = fm[0] * (ur[2]/ur[0] + n[1]*(-2.0*cj - vnj)/g);
		fm[3] = fm[0] * ( (vmags - vnj*vnj)/2.0 + sq((g-1)*vnj-2*cj)/(2*(g*g-1)) );
	}
	for(int k = 0; k < 4; k++) f[k] = fp[k] + fm[k];
}

FVHIP_HD void flux_ausm(const Gas& G, const double* ul, const double* ur, const double* n, double* f) {
	double vi[2], vj[2], vni, vnj, pi, pj, Hi, Hj;
	flow_vars(G, ul, n, vi, vni, pi, Hi);
	flow_vars(G, ur, n, vj, vnj, pj, Hj);
	const double ci = sound_speed(G, ul[0], pi), cj = sound_speed(G, ur[0], pj);
	const double Mni = div_rn(vni, ci), Mnj = div_rn(vnj, cj);
	double ML, MR, pL, pR;
	if(fabs(Mni) <= 1.0) { ML = 0.25*(Mni+1)*(Mni+1); pL = ML*pi*(2.0-Mni); }
	else if(Mni < -1.0) { ML = 0; pL = 0; }
	else { ML = Mni; pL = pi; }
	if(fabs(Mnj) <= 1.0) { MR = -0.25*(Mnj-1)*(Mnj-1); pR = -MR*pj*(2.0+Mnj); }
	else if(Mnj < -1.0) { MR = Mnj; pR = pj; }
	else { MR = 0; pR = 0; }
	const double Mh = ML+MR, ph = pL+pR;
	f[0] = Mh/2.0*(ul[0]*ci+ur[0]*cj) -fabs(Mh)/2.0*(ur[0]*cj-ul[0]*ci);
	f[1] = Mh/2.0*(ul[1]*ci+ur[1]*cj) -fabs(Mh)/2.0*(ur[1]*cj-ul[1]*ci) + ph*n[0];
	f[2] = Mh/2.0*(ul[2]*ci+ur[2]*cj) -fabs(Mh)/2.0*(ur[2]*cj-ul[2]*ci) + ph*n[1];
	f[3] = Mh/2.0*(ci*(ul[3]+pi)+cj*(ur[3]+pj)) -fabs(Mh)/2.0*(cj*(ur[3]+pj)-ci*(ul[3]+pi));
}

FVHIP_HD void flux_ausmplus(const Gas& G, const double* ul, const double* ur, const double* n, double* f) {
	const double g = G.g;
	double vi[2], vj[2], vni, vnj, pi, pj, Hi, Hj;
	flow_vars(G, ul, n, vi, vni, pi, Hi);
	flow_vars(G, ur, n, vj, vnj, pj, Hj);
	const double ci = sound_speed(G, ul[0], pi), cj = sound_speed(G, ur[0], pj);
	const double vm2i = dot2(vi,vi), vm2j = dot2(vj,vj);
	double csi = sqrt((ci*ci/(g-1.0)+0.5*vm2i)*2.0*(g-1.0)/(g+1.0));
	double csj = sqrt((cj*cj/(g-1.0)+0.5*vm2j)*2.0*(g-1.0)/(g+1.0));
	const double ki = csi > vni ? csi : vni;
	const double kj = csj > -vnj ? csj : -vnj;
	csi = csi*csi/ki;
	csj = csj*csj/kj;
	const double ch = (csi < csj) ? csi : csj;
	const double Mni = vni/ch, Mnj = vnj/ch;
	double ML, MR, pL, pR;
	if(fabs(Mni) <= 1.0) {
		ML = 0.25*(Mni+1)*(Mni+1) + 1.0/8.0*(Mni*Mni-1.0)*(Mni*Mni-1.0);
		pL = pi*(0.25*(Mni+1)*(Mni+1)*(2.0-Mni) + 3.0/16*Mni*(Mni*Mni-1.0)*(Mni*Mni-1.0));
	}
	else if(Mni < -1.0) { ML = 0; pL = 0; }
	else { ML = Mni; pL = pi; }
	if(fabs(Mnj) <= 1.0) {
		MR = -0.25*(Mnj-1)*(Mnj-1) - 1.0/8.0*(Mnj*Mnj-1.0)*(Mnj*Mnj-1.0);
		pR = pj*(0.25*(Mnj-1)*(Mnj-1)*(2.0+Mnj) - 3.0/16*Mnj*(Mnj*Mnj-1.0)*(Mnj*Mnj-1.0));
	}
	else if(Mnj < -1.0) { MR = Mnj; pR = pj; }
	else { MR = 0; pR = 0; }
	const double Mh = ML+MR, ph = pL+pR;
	f[0] = ch* (Mh/2.0*(ul[0]+ur[0]) -fabs(Mh)/2.0*(ur[0]-ul[0]));
	f[1] = ch* (Mh/2.0*(ul[1]+ur[1]) -fabs(Mh)/2.0*(ur[1]-ul[1])) + ph*n[0];
	f[2] = ch* (Mh/2.0*(ul[2]+ur[2]) -fabs(Mh)/2.0*(ur[2]-ul[2])) + ph*n[1];
	f[3] = ch* (Mh/2.0*(ul[3]+pi+ur[3]+pj) -fabs(Mh)/2.0*((ur[3]+pj)-(ul[3]+pi)));
}

template <bool HALVE = true>
FVHIP_HD void flux_roe(const Gas& G, const double* ul, const double* ur, const double* n, double* f) {
	double vi[2], vj[2], vni, vnj, pi, pj, Hi, Hj;
	flow_vars(G, ul, n, vi, vni, pi, Hi);
	flow_vars(G, ur, n, vj, vnj, pj, Hj);
	const RoeAvg a = roe_average(G, ul, ur, n, vi, Hi, vj, Hj);
	// |eigenvalues| with Harten's entropy fix, delta = 1e-4 c (anumericalflux.cpp:664, 686-692)
	double l0 = fabs(a.vn-a.c), l1 = fabs(a.vn), l3 = fabs(a.vn+a.c);
	const double delta = 1.0e-4*a.c;
	if(l0 < delta) l0 = div_rn(l0*l0 + delta*delta, 2.0*delta);
	if(l1 < delta) l1 = div_rn(l1*l1 + delta*delta, 2.0*delta);
	if(l3 < delta) l3 = div_rn(l3*l3 + delta*delta, 2.0*delta);
	const double devn = vnj-vni, dep = pj-pi, derho = ur[0]-ul[0];
	// 2*c*c = (c*c) + (c*c) exactly; on the device the two divisions by it are taken as halves of
	// divisions by c*c, sharing a1's reciprocal (div_rn is correctly rounded, and halving is exact)
	const double cc = a.c*a.c;
	const double a1 = l1*(derho - div_rn(dep, cc));
	const double a2 = l1*a.rho;
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FVHIP_FAST)
	const double a0 = 0.5*div_rn(l0*(dep-a.rho*a.c*devn), cc);
	const double a3 = 0.5*div_rn(l3*(dep+a.rho*a.c*devn), cc);
#else
	const double a0 = div_rn(l0*(dep-a.rho*a.c*devn), cc + cc);
	const double a3 = div_rn(l3*(dep+a.rho*a.c*devn), cc + cc);
#endif
	double d0 = a0, d1 = a0*(a.v[0]-a.c*n[0]), d2 = a0*(a.v[1]-a.c*n[1]), d3 = a0*(a.H-a.c*a.vn);
	d0 += a1;
	d1 += a1*a.v[0] +      a2*(vj[0]-vi[0] - devn*n[0]);
	d2 += a1*a.v[1] +      a2*(vj[1]-vi[1] - devn*n[1]);
	d3 += add_pow2(a2 *(a.v[0]*(vj[0]-vi[0]) +a.v[1]*(vj[1]-vi[1]) -a.vn*devn), a1*a.vm2, 0.5);   // a1*vm2/2.0 + a2*(...)
	d0 += a3;
	d1 += a3*(a.v[0]+a.c*n[0]);
	d2 += a3*(a.v[1]+a.c*n[1]);
	d3 += a3*(a.H+a.c*a.vn);
	double fi[4], fj[4];
	directional_flux(G, ul, n, vni, pi, fi);
	directional_flux(G, ur, n, vnj, pj, fj);
	const double s[4] = {fi[0]+fj[0] - d0, fi[1]+fj[1] - d1, fi[2]+fj[2] - d2, fi[3]+fj[3] - d3};
	for(int k = 0; k < 4; k++) f[k] = HALVE ? 0.5*s[k] : s[k];
}

FVHIP_HD void einfeldt(double vni, double ci, double vnj, double cj, const RoeAvg& a, double& sl, double& sr) {
	sl = vni - ci;
	if(sl > a.vn-a.c) sl = a.vn-a.c;
	sr = vnj+cj;
	if(sr < a.vn+a.c) sr = a.vn+a.c;
}

FVHIP_HD void flux_hll(const Gas& G, const double* ul, const double* ur, const double* n, double* f) {
	double vi[2], vj[2], vni, vnj, pi, pj, Hi, Hj;
	flow_vars(G, ul, n, vi, vni, pi, Hi);
	flow_vars(G, ur, n, vj, vnj, pj, Hj);
	const double ci = sound_speed(G, ul[0], pi), cj = sound_speed(G, ur[0], pj);
	const RoeAvg a = roe_average(G, ul, ur, n, vi, Hi, vj, Hj);
	double sl, sr;
	einfeldt(vni, ci, vnj, cj, a, sl, sr);
	const double sr0 = sr > 0 ? 0 : sr;
	const double sl0 = sl > 0 ? 0 : sl;
	const double t1 = div_rn(sr0 - sl0, sr-sl); const double t2 = 1.0 - t1;
	const double t3 = div_rn(0.5*(sr*fabs(sl)-sl*fabs(sr)), sr-sl);
	f[0] = t1*vnj*ur[0] + t2*vni*ul[0]                     - t3*(ur[0]-ul[0]);
	f[1] = t1*(vnj*ur[1]+pj*n[0]) + t2*(vni*ul[1]+pi*n[0]) - t3*(ur[1]-ul[1]);
	f[2] = t1*(vnj*ur[2]+pj*n[1]) + t2*(vni*ul[2]+pi*n[1]) - t3*(ur[2]-ul[2]);
	f[3] = t1*(vnj*ur[0]*Hj) + t2*(vni*ul[0]*Hi)           - t3*(ur[3]-ul[3]);
}

/// HLLC star state (anumericalflux.cpp:1069-1081), returned as the flux correction s*(u* - u)
FVHIP_HD void hllc_side(const double* u, const double* n, double vn, double p, double ss, double sm, double* f) {
	const double pstar = u[0]*(vn-ss)*(vn-sm) + p;
	const double us0 = div_rn(u[0] * (ss - vn), ss-sm);
	const double us1 = div_rn( (ss-vn)*u[1] + (pstar-p)*n[0], ss-sm );
	const double us2 = div_rn( (ss-vn)*u[2] + (pstar-p)*n[1], ss-sm );
	const double us3 = div_rn( (ss-vn)*u[3] - p*vn + pstar*sm, ss-sm );
	f[0] += ss * (us0 - u[0]);
	f[1] += ss * (us1 - u[1]);
	f[2] += ss * (us2 - u[2]);
	f[3] += ss * (us3 - u[3]);
}

FVHIP_HD void flux_hllc(const Gas& G, const double* ul, const double* ur, const double* n, double* f) {
	double vi[2], vj[2], vni, vnj, pi, pj, Hi, Hj;
	flow_vars(G, ul, n, vi, vni, pi, Hi);
	flow_vars(G, ur, n, vj, vnj, pj, Hj);
	const double ci = sound_speed(G, ul[0], pi), cj = sound_speed(G, ur[0], pj);
	const RoeAvg a = roe_average(G, ul, ur, n, vi, Hi, vj, Hj);
	double sl, sr;
	einfeldt(vni, ci, vnj, cj, a, sl, sr);
	const double sm = div_rn( ur[0]*vnj*(sr-vnj) - ul[0]*vni*(sl-vni) + pi-pj,
		ur[0]*(sr-vnj) - ul[0]*(sl-vni) );
	if(sl > 0)
		directional_flux(G, ul, n, vni, pi, f);
	else if(sl <= 0 && sm > 0) {
		directional_flux(G, ul, n, vni, pi, f);
		hllc_side(ul, n, vni, pi, sl, sm, f);
	}
	else if(sm <= 0 && sr >= 0) {
		directional_flux(G, ur, n, vnj, pj, f);
		hllc_side(ur, n, vnj, pj, sr, sm, f);
	}
	else
		directional_flux(G, ur, n, vnj, pj, f);
}

template <int FLUX>
FVHIP_HD void inviscid_flux(const Gas& G, const double* ul, const double* ur, const double* n, double* f) {
	switch(FLUX) {
		case 0: flux_llf(G, ul, ur, n, f); break;
		case 1: flux_vanleer(G, ul, ur, n, f); break;
		case 2: flux_ausm(G, ul, ur, n, f); break;
		case 3: flux_ausmplus(G, ul, ur, n, f); break;
		case 4: flux_roe(G, ul, ur, n, f); break;
		case 5: flux_hll(G, ul, ur, n, f); break;
		default: flux_hllc(G, ul, ur, n, f); break;
	}
}

/// the flux times the face length, f*len, as the sweeps form it. Roe and LLF end in 0.5*(...): on the
/// device the halving moves into the length, RN(RN(0.5 s) len) = RN(s (0.5 len)) bitwise (both
/// halvings exact), one multiply per face instead of four
template <int FLUX>
FVHIP_HD void inviscid_flux_len(const Gas& G, const double* ul, const double* ur, const double* n, double len, double* f) {
#if defined(__HIP_DEVICE_COMPILE__)
	if(FLUX == 0 || FLUX == 4) {
		if(FLUX == 0) flux_llf<false>(G, ul, ur, n, f);
		else flux_roe<false>(G, ul, ur, n, f);
		const double hl = 0.5*len;
		for(int k = 0; k < 4; k++) f[k] *= hl;
		return;
	}
#endif
	inviscid_flux<FLUX>(G, ul, ur, n, f);
	for(int k = 0; k < 4; k++) f[k] *= len;
}

FVHIP_HD void inviscid_flux_rt(int type, const Gas& G, const double* ul, const double* ur, const double* n, double* f) {
	switch(type) {
		case 0: flux_llf(G, ul, ur, n, f); break;
		case 1: flux_vanleer(G, ul, ur, n, f); break;
		case 2: flux_ausm(G, ul, ur, n, f); break;
		case 3: flux_ausmplus(G, ul, ur, n, f); break;
		case 4: flux_roe(G, ul, ur, n, f); break;
		case 5: flux_hll(G, ul, ur, n, f); break;
		default: flux_hllc(G, ul, ur, n, f); break;
	}
}

// ---------------------------------------------------------------------------------------------
// Boundary ghost states (abc.cpp). bc = {type, vals[0], vals[1]}; uinf = free stream.
// ---------------------------------------------------------------------------------------------
struct BCDev { int type; double v0, v1; };

FVHIP_HD void ghost_state_common(const Gas& G, const BCDev& bc, const double* uinf, const double* ins,
                                 const double* n, double* gs);
FVHIP_HD void ghost_state(const Gas& G, const BCDev& bc, const double* uinf, const double* ins,
                          const double* n, double* gs) {
	switch(bc.type) {
	case 3: {  // SUBSONIC_INFLOW (abc.cpp:145-175)
		const double g = G.g, ptotal = bc.v0, ttotal = bc.v1;
		const double ci = sound_speed_cons(G, ins);
		const double Rm = dot2(&ins[1],n)/ins[0] - ci/(2*g - 1.0);
		const double co2 = ci*ci + (g-1.0)/2.0 * dot2(&ins[1],&ins[1])/(ins[0]*ins[0]);
		const double q = sqrt((g+1)*co2/((g-1)*Rm*Rm) - (g-1)/2.0);
		const double cg = -Rm*(g-1)/(g+1) * (1.0 + q);
		const double tg = ttotal*cg*cg/co2;
		const double pg = ptotal * pow(tg/ttotal, g/(g-1.0));
		const double rho = g*G.Minf*G.Minf*pg/tg;
		const double vm = sqrt(2.0/(g-1.0)*(co2 - cg*cg));
		const double vx = vm*1.0*n[0], vy = vm*1.0*n[1];
		gs[0] = rho; gs[1] = rho*vx; gs[2] = rho*vy;
		gs[3] = energy_from_pressure(G, pg, rho, vm*vm);
		break;
	}
	case 6: {  // ISOTHERMAL_WALL (abc.cpp:349-366)
		const double p = pressure_cons(G, ins);
		const double gtemp = 2.0*bc.v1 - temperature(G, ins[0], p);
		const double r = ins[0];
		const double m0 = r*( 2.0*bc.v0*n[1] - div_rn(ins[1], ins[0]));
		const double m1 = r*(-2.0*bc.v0*n[0] - div_rn(ins[2], ins[0]));
		double mm[2] = {m0, m1};
		const double vm2 = div_rn(dot2(mm,mm), r*r);
		gs[0] = r; gs[1] = m0; gs[2] = m1; gs[3] = energy_from_temperature(G, gtemp, r, vm2);
		break;
	}
	default:
		ghost_state_common(G, bc, uinf, ins, n, gs);
		break;
	}
}

/// ghost_state for the common boundary conditions only (slip wall, far field, inflow-outflow,
/// adiabatic wall, extrapolation): the kernels inline this form when a configuration uses no other
/// BC type (the subsonic-inflow and isothermal-wall states are long, register-hungry sequences that
/// stay out of line)
FVHIP_HD void ghost_state_common(const Gas& G, const BCDev& bc, const double* uinf, const double* ins,
                          const double* n, double* gs) {
	switch(bc.type) {
	case 2: {  // INFLOW_OUTFLOW (abc.cpp:46-81)
		const double vni = div_rn(dot2(&ins[1],n), ins[0]);
		const double ci = sound_speed_cons(G, ins);
		const double Mni = div_rn(vni, ci);
		if(Mni <= 0) { gs[0] = uinf[0]; gs[1] = uinf[1]; gs[2] = uinf[2]; gs[3] = uinf[3]; }
		else if(Mni < 1) {
			const double pinf = freestream_pressure(G);
			const double e = energy_from_pressure(G, pinf, ins[0], div_rn(dot2(&ins[1],&ins[1]), ins[0]*ins[0]));
			gs[0] = ins[0]; gs[1] = ins[1]; gs[2] = ins[2]; gs[3] = e;
		}
		else { gs[0] = ins[0]; gs[1] = ins[1]; gs[2] = ins[2]; gs[3] = ins[3]; }
		break;
	}
	case 1:    // FARFIELD
		gs[0] = uinf[0]; gs[1] = uinf[1]; gs[2] = uinf[2]; gs[3] = uinf[3];
		break;
	case 0: {  // SLIP_WALL (abc.cpp:219-229)
		const double vni = div_rn(dot2(&ins[1],n), ins[0]);
		const double r = ins[0], e = ins[3];
		const double m0 = ins[1] - 2.0*vni*n[0]*ins[0];
		const double m1 = ins[2] - 2.0*vni*n[1]*ins[0];
		gs[0] = r; gs[1] = m0; gs[2] = m1; gs[3] = e;
		break;
	}
	case 7: {  // ADIABATIC_WALL -> Adiabaticwall2D (abc.cpp:278-287, factory :486-488)
		const double tm = bc.v0 * ins[0];
		const double r = ins[0], e = ins[3];
		const double m0 =  2.0*tm*n[1] - ins[1];
		const double m1 = -2.0*tm*n[0] - ins[2];
		gs[0] = r; gs[1] = m0; gs[2] = m1; gs[3] = e;
		break;
	}
	default:   // EXTRAPOLATION (and anything else, rejected at setup)
		gs[0] = ins[0]; gs[1] = ins[1]; gs[2] = ins[2]; gs[3] = ins[3];
		break;
	}
}

// ---------------------------------------------------------------------------------------------
// Viscous face flux (flow_spatial.cpp:348-395, aspatial.cpp:172-205, viscousphysics.cpp:14-122)
// gl, gr: primitive gradients in GradBlock layout [var][dim]; zero-gradient first order if !order2.
// ORDER2: pl, pr are the cells' primitive states (rho, vx, vy, p) = cons2prim(u) -- the residual
// stages them already, bit for bit what getPrimitive2StatesAndGradients derives from the conserved
// states; first order: pl, pr are the conserved states (converted here with cons2prim2).
// ---------------------------------------------------------------------------------------------
/// the face-state inputs of the viscous flux: the averaged viscosity (flow_spatial.cpp:379-383) and
/// the averaged velocity of the energy term (viscousphysics.cpp:108-111); split out so a caller can
/// form them while the face states are live and drop those states before the gradient terms
template <bool CONSTVISC>
FVHIP_HD void viscous_face_terms(const Gas& G, const double* ul, const double* ur, double& muRe, double* va) {
	muRe = CONSTVISC ? G.rReinf : 0.5*( sutherland(G, ul) + sutherland(G, ur) );
	va[0] = 0.5*( div_rn(ul[1], ul[0]) + div_rn(ur[1], ur[0]) );
	va[1] = 0.5*( div_rn(ul[2], ul[0]) + div_rn(ur[2], ur[0]) );
}
/// the same with the two face states' Sutherland viscosities already formed (mul = sutherland(G, ul),
/// mur = sutherland(G, ur); ignored for constant viscosity)
template <bool CONSTVISC>
FVHIP_HD void viscous_face_terms_mu(const Gas& G, const double* ul, const double* ur, double mul, double mur,
                                    double& muRe, double* va) {
	muRe = CONSTVISC ? G.rReinf : 0.5*( mul + mur );
	va[0] = 0.5*( div_rn(ul[1], ul[0]) + div_rn(ur[1], ur[0]) );
	va[1] = 0.5*( div_rn(ul[2], ul[0]) + div_rn(ur[2], ur[0]) );
}
template <bool ORDER2>
FVHIP_HD void viscous_flux_core(const Gas& G, const double* n, const double* rcl, const double* rcr,
                                const double* pl, const double* pr, const double* gl, const double* grr,
                                double muRe, const double* va, double* vf);
template <bool ORDER2, bool CONSTVISC>
FVHIP_HD void viscous_flux(const Gas& G, const double* n, const double* rcl, const double* rcr,
                           const double* pl, const double* pr, const double* gl, const double* grr,
                           const double* ul, const double* ur, double* vf) {
	double muRe, va[2];
	viscous_face_terms<CONSTVISC>(G, ul, ur, muRe, va);
	viscous_flux_core<ORDER2>(G, n, rcl, rcr, pl, pr, gl, grr, muRe, va, vf);
}
template <bool ORDER2>
FVHIP_HD void viscous_flux_core(const Gas& G, const double* n, const double* rcl, const double* rcr,
                                const double* pl, const double* pr, const double* gl, const double* grr,
                                double muRe, const double* va, double* vf) {
	double tl[4], tr[4], gL[8], gR[8];          // gL[dim*4 + var]
	if(ORDER2) {
		for(int i = 0; i < 2; i++) for(int j = 0; j < 4; j++) { gL[i*4+j] = gl[j*2+i]; gR[i*4+j] = grr[j*2+i]; }
		for(int i = 0; i < 4; i++) { tl[i] = pl[i]; tr[i] = pr[i]; }
		for(int j = 0; j < 2; j++) {
			gL[j*4+3] = grad_temperature(G, tl[0], gL[j*4], tl[3], gL[j*4+3]);
			gR[j*4+3] = grad_temperature(G, tr[0], gR[j*4], tr[3], gR[j*4+3]);
		}
		tl[3] = temperature(G, tl[0], tl[3]);
		tr[3] = temperature(G, tr[0], tr[3]);
	} else {
		cons2prim2(G, pl, tl);
		cons2prim2(G, pr, tr);
		for(int i = 0; i < 8; i++) { gL[i] = 0; gR[i] = 0; }
	}
	double grad[2][4];
	{
		double dr[2], dist = 0;
		dr[0] = rcr[0]-rcl[0]; dist += dr[0]*dr[0];
		dr[1] = rcr[1]-rcl[1]; dist += dr[1]*dr[1];
		dist = sqrt_rn(dist);
		dr[0] = div_rn(dr[0], dist); dr[1] = div_rn(dr[1], dist);
		for(int i = 0; i < 4; i++) {
			double davg[2];
			davg[0] = 0.5*(gL[i] + gR[i]);
			davg[1] = 0.5*(gL[4+i] + gR[4+i]);
			const double corr = div_rn(tr[i]-tl[i], dist);
			const double ddr = dot2(davg,dr);
			grad[0][i] = davg[0] - ddr*dr[0] + corr*dr[0];
			grad[1][i] = davg[1] - ddr*dr[1] + corr*dr[1];
		}
	}
	const double kd = div_rcp(muRe, G.kden, G.rkden);
	double ldiv = 0;
	ldiv += grad[0][1]; ldiv += grad[1][2];
	ldiv *= 2.0/3.0*muRe;
	double s[2][2];
	s[0][0] = muRe*(grad[0][1] + grad[0][1]); s[0][1] = muRe*(grad[0][2] + grad[1][1]);
	s[0][0] -= ldiv;
	s[1][0] = muRe*(grad[1][1] + grad[0][2]); s[1][1] = muRe*(grad[1][2] + grad[1][2]);
	s[1][1] -= ldiv;
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

}
}
#endif
