/** \file gasjac.hpp
 * \brief Analytic flux Jacobians for the MI355X Jacobian assembly, evaluated ONE COLUMN AT A TIME.
 *
 * The reference computes full 4x4 blocks with arrays of derivatives (anumericalflux.cpp:63-107,
 * 567-965, 1009-1061, 1083-1397; aphysics.cpp:60-153). Every derivative there is indexed by the
 * differentiation variable k and only combines quantities with the same k, so a column of
 * dfdl/dfdr needs a handful of scalars instead of ~200 live doubles. Each element below is the
 * reference's expression for that element, with the same association and the same literal zero
 * terms (so even signed zeros match).  dfdl = -dF/dul, dfdr = +dF/dur (anumericalflux.hpp:36-45).
 */
#ifndef FVHIP_GASJAC_HPP
#define FVHIP_GASJAC_HPP

#include "gasdyn.hpp"

namespace fvhip {
namespace gd {

/// Per-state quantities of getJacobianDirectionalFluxWrtConserved / getJacobianVarsWrtConserved
struct SideJ {
	double u[4];
	double pc, vnc;        ///< pressure and normal velocity recomputed from conserved variables
	double dp[4];          ///< dp/du (getJacobianPressureWrtConserved assigns)
	double dvnc[4];        ///< d(vnc)/du as in aphysics.cpp:101-106
};

FVHIP_HD void side_prepare(const Gas& G, const double* u, const double* n, SideJ& s) {
	for(int i = 0; i < 4; i++) s.u[i] = u[i];
	s.pc = pressure_cons(G, u);
	s.dp[0] = (G.g-1.0)*0.5*dot2(&u[1],&u[1])/(u[0]*u[0]);
	s.dp[1] = -(G.g-1.0)*u[1]/u[0];
	s.dp[2] = -(G.g-1.0)*u[2]/u[0];
	s.dp[3] = (G.g-1.0);
	s.vnc = dot2(&u[1],n)/u[0];
	s.dvnc[0] = -s.vnc/u[0];
	s.dvnc[1] = n[0]/u[0];
	s.dvnc[2] = n[1]/u[0];
	s.dvnc[3] = 0;
}

/// column k of getJacobianDirectionalFluxWrtConserved (aphysics.cpp:92-126)
FVHIP_HD void dirflux_jac_col(const SideJ& s, const double* n, int k, double* c) {
	const double* u = s.u; const double* dp = s.dp; const double* dvn = s.dvnc;
	const double vn = s.vnc, p = s.pc;
	// row 0
	c[0] = (k == 1) ? n[0] : (k == 2) ? n[1] : 0;
	// rows 1, 2
	for(int i = 1; i < 3; i++) {
		if(k == 0) c[i] = -vn*u[i]/u[0] + dp[0]*n[i-1];
		else if(k == 3) c[i] = dp[3]*n[i-1];
		else if(k == i) c[i] = dvn[k]*u[i] + vn + dp[k]*n[i-1];
		else c[i] = dvn[k]*u[i] + dp[k]*n[i-1];
	}
	// row 3
	if(k == 0) c[3] = -vn/u[0]*(u[3]+p) + vn*dp[0];
	else if(k == 3) c[3] = vn*(1.0 + dp[3]);
	else c[3] = n[k-1]/u[0]*(u[3]+p) + vn*dp[k];
}

/// column k of getJacobianVarsWrtConserved (aphysics.cpp:129-153) applied to zeroed arrays
struct VarsJ { double dvx, dvy, dvn, dp, dH; };
FVHIP_HD VarsJ vars_jac_col(const Gas& G, const SideJ& s, const double* n, int k) {
	const double* uc = s.u;
	VarsJ v;
	double dvx = 0, dvy = 0, dvn = 0;
	if(k == 0) { dvx += -uc[1]/(uc[0]*uc[0]); dvy += -uc[2]/(uc[0]*uc[0]); }
	if(k == 1) dvx += 1.0/uc[0];
	if(k == 2) dvy += 1.0/uc[0];
	if(k == 0) { dvn += dvx*n[0]; dvn += dvy*n[1]; }
	if(k == 1) dvn += n[0]/uc[0];
	if(k == 2) dvn += n[1]/uc[0];
	double dH = 0;
	if(k == 0) dH += (s.dp[0]*uc[0] - (uc[3]+s.pc))/(uc[0]*uc[0]);
	else if(k == 3) dH += (1.0+s.dp[3])/uc[0];
	else dH += s.dp[k]/uc[0];
	v.dvx = dvx; v.dvy = dvy; v.dvn = dvn; v.dp = s.dp[k]; v.dH = dH;
	return v;
}

/// sound-speed derivative column (getJacobianSoundSpeed, aphysics_defs.hpp:145-154) onto zero
FVHIP_HD double dc_col(const Gas& G, double rho, double p, double dpk, double c, int k) {
	double d = 0;
	if(k == 0) d += 0.5/c * G.g* (dpk*rho-p)/(rho*rho);
	else d += 0.5/c * G.g*dpk/rho;
	return d;
}

// ---------------------------------------------------------------------------------------------
// LLF (frozen spectral radius), anumericalflux.cpp:65-107
// ---------------------------------------------------------------------------------------------
struct LLFJ { SideJ L, R; double eig; };
FVHIP_HD void llf_jac_prepare(const Gas& G, const double* ul, const double* ur, const double* n, LLFJ& J) {
	double vi[2], vj[2], vni, vnj, pi, pj, Hi, Hj;
	flow_vars(G, ul, n, vi, vni, pi, Hi);
	flow_vars(G, ur, n, vj, vnj, pj, Hj);
	const double ci = sound_speed(G, ul[0], pi), cj = sound_speed(G, ur[0], pj);
	J.eig = (fabs(vni)+ci >= fabs(vnj)+cj) ? fabs(vni)+ci : fabs(vnj)+cj;
	side_prepare(G, ul, n, J.L);
	side_prepare(G, ur, n, J.R);
}
FVHIP_HD void llf_jac_col(const LLFJ& J, const double* n, int k, double* dl, double* dr) {
	double a[4], b[4];
	dirflux_jac_col(J.L, n, k, a);
	dirflux_jac_col(J.R, n, k, b);
	a[k] -= -J.eig;
	b[k] -= J.eig;
	for(int i = 0; i < 4; i++) { dl[i] = -0.5*a[i]; dr[i] = 0.5*b[i]; }
}

// ---------------------------------------------------------------------------------------------
// HLL (frozen signal speeds), anumericalflux.cpp:1012-1061
// ---------------------------------------------------------------------------------------------
struct HLLJ { SideJ L, R; double t1, t2, t3; };
FVHIP_HD void hll_jac_prepare(const Gas& G, const double* ul, const double* ur, const double* n, HLLJ& J) {
	double vi[2], vj[2], vni, vnj, pi, pj, Hi, Hj;
	flow_vars(G, ul, n, vi, vni, pi, Hi);
	flow_vars(G, ur, n, vj, vnj, pj, Hj);
	const double ci = sound_speed(G, ul[0], pi), cj = sound_speed(G, ur[0], pj);
	const RoeAvg a = roe_average(G, ul, ur, n, vi, Hi, vj, Hj);
	double sl, sr;
	einfeldt(vni, ci, vnj, cj, a, sl, sr);
	const double sr0 = sr > 0 ? 0 : sr;
	const double sl0 = sl > 0 ? 0 : sl;
	J.t1 = (sr0 - sl0)/(sr-sl);
	J.t2 = 1.0 - J.t1;
	J.t3 = 0.5*(sr*fabs(sl)-sl*fabs(sr))/(sr-sl);
	side_prepare(G, ul, n, J.L);
	side_prepare(G, ur, n, J.R);
}
FVHIP_HD void hll_jac_col(const HLLJ& J, const double* n, int k, double* dl, double* dr) {
	double a[4], b[4];
	dirflux_jac_col(J.L, n, k, a);
	dirflux_jac_col(J.R, n, k, b);
	for(int i = 0; i < 4; i++) { dl[i] = -J.t2*a[i]; dr[i] = J.t1*b[i]; }
	dl[k] = dl[k] - J.t3;
	dr[k] = dr[k] - J.t3;
}

// ---------------------------------------------------------------------------------------------
// Roe-average derivative columns, anumericalflux.cpp:567-660
// ---------------------------------------------------------------------------------------------
struct RoeBase {
	double vi[2], vj[2], vni, vnj, pi, pj, Hi, Hj;
	RoeAvg a;
	SideJ L, R;
};
FVHIP_HD void roe_base(const Gas& G, const double* ul, const double* ur, const double* n, RoeBase& B) {
	flow_vars(G, ul, n, B.vi, B.vni, B.pi, B.Hi);
	flow_vars(G, ur, n, B.vj, B.vnj, B.pj, B.Hj);
	B.a = roe_average(G, ul, ur, n, B.vi, B.Hi, B.vj, B.Hj);
	side_prepare(G, ul, n, B.L);
	side_prepare(G, ur, n, B.R);
}
struct RoeAvgJ { double dR, drho, dvx, dvy, dvm2, dvn, dH, dc; };
/// column k of the Roe-average derivatives w.r.t. the left (I) and right (J) states
FVHIP_HD void roe_avg_jac_col(const Gas& G, const RoeBase& B, const double* n, int k,
                              const VarsJ& Vi, const VarsJ& Vj, RoeAvgJ& I, RoeAvgJ& Jr) {
	const double* ul = B.L.u; const double* ur = B.R.u;
	const double Rij = B.a.R, vxi = B.vi[0], vyi = B.vi[1], vxj = B.vj[0], vyj = B.vj[1];
	const double Hi = B.Hi, Hj = B.Hj;
	const double dRiji = (k == 0) ? 0.5/Rij * (-ur[0])/(ul[0]*ul[0]) : 0;
	const double dRijj = (k == 0) ? 0.5/Rij / ul[0] : 0;
	const double rden2 = (Rij+1.0)*(Rij+1.0);
	double dvxiji, dvxijj, dvyiji, dvyijj;
	switch(k) {
	case 0:
		dvxiji = ((dRiji*ur[1]/ur[0] -ul[1]/(ul[0]*ul[0]))*(Rij+1.0) -(Rij*vxj+vxi)*dRiji)/rden2;
		dvxijj = ((dRijj*ur[1]/ur[0] +Rij/(ur[0]*ur[0])*(-ur[1]))*(Rij+1.0) -(Rij*vxj+vxi)*dRijj) / rden2;
		dvyiji = ((ur[2]/ur[0]*dRiji - ul[2]/(ul[0]*ul[0]))*(Rij+1.0) -(Rij*vyj+vyi)*dRiji) / rden2;
		dvyijj = ((dRijj*ur[2]/ur[0] + Rij/(ur[0]*ur[0])*(-ur[2]))*(Rij+1.0) -(Rij*vyj+vyi)*dRijj ) / rden2;
		break;
	case 1:
		dvxiji = ((dRiji*ur[1]/ur[0] + 1.0/ul[0])*(Rij+1.0)-(Rij*vxj+vxi)*dRiji)/rden2;
		dvxijj = ((dRijj*ur[1]/ur[0] +Rij/ur[0])*(Rij+1.0)-(Rij*vxj+vxi)*dRijj) / rden2;
		dvyiji = (ur[2]/ur[0]*dRiji *(Rij+1.0) - (Rij*vyj+vyi)*dRiji) / rden2;
		dvyijj = (dRijj*ur[2]/ur[0] *(Rij+1.0) -(Rij*vyj+vyi)*dRijj) / rden2;
		break;
	case 2:
		dvxiji = (dRiji*ur[1]/ur[0] *(Rij+1.0)- (Rij*vxj+vxi)*dRiji)/rden2;
		dvxijj = (dRijj*ur[1]/ur[0] *(Rij+1.0) - (Rij*vxj+vxi)*dRijj) / rden2;
		dvyiji = ((ur[2]/ur[0]*dRiji + 1.0/ul[0])*(Rij+1.0) -(Rij*vyj+vyi)*dRiji) / rden2;
		dvyijj = ((dRijj*ur[2]/ur[0] + Rij/ur[0])*(Rij+1.0) -(Rij*vyj+vyi)*dRijj) / rden2;
		break;
	default:
		dvxiji = (dRiji*ur[1]/ur[0] *(Rij+1.0)- (Rij*vxj+vxi)*dRiji)/rden2;
		dvxijj = (dRijj*ur[1]/ur[0] *(Rij+1.0) - (Rij*vxj+vxi)*dRijj) / rden2;
		dvyiji = (ur[2]/ur[0]*dRiji *(Rij+1.0) -(Rij*vyj+vyi)*dRiji) / rden2;
		dvyijj = (dRijj*ur[2]/ur[0] *(Rij+1.0) - (Rij*vyj+vyi)*dRijj) / rden2;
	}
	const double vxij = B.a.v[0], vyij = B.a.v[1], cij = B.a.c;
	I.dR = dRiji; Jr.dR = dRijj;
	I.dvx = dvxiji; I.dvy = dvyiji; Jr.dvx = dvxijj; Jr.dvy = dvyijj;
	I.dvn = dvxiji*n[0] + dvyiji*n[1];
	Jr.dvn = dvxijj*n[0] + dvyijj*n[1];
	I.dvm2 = 2.0*( vxij*dvxiji + vyij*dvyiji );
	Jr.dvm2 = 2.0*( vxij*dvxijj + vyij*dvyijj );
	I.dc = 0.5/cij*(G.g-1.0) * (((dRiji*Hj+Vi.dH)*(Rij+1)-(Rij*Hj+Hi)*dRiji)/rden2 - 0.5*I.dvm2);
	Jr.dc = 0.5/cij*(G.g-1.0) * (((dRijj*Hj+Rij*Vj.dH)*(Rij+1) - (Rij*Hj+Hi)*dRijj)/rden2 - 0.5*Jr.dvm2);
	I.drho = (k == 0) ? dRiji*ul[0] + Rij : 0;
	Jr.drho = (k == 0) ? dRijj*ul[0] : 0;
	I.dH = ((dRiji*Hj+Vi.dH)*(Rij+1.0)-(Rij*Hj+Hi)*dRiji)/rden2;
	Jr.dH = ((dRijj*Hj+Rij*Vj.dH)*(Rij+1.0)-(Rij*Hj+Hi)*dRijj)/rden2;
}

// ---------------------------------------------------------------------------------------------
// Roe, anumericalflux.cpp:736-965
// ---------------------------------------------------------------------------------------------
struct RoeJ {
	RoeBase B;
	double l[4]; bool fixed[4]; double delta, devn, dep, derho, la[4], cij4;
};
FVHIP_HD void roe_jac_prepare(const Gas& G, const double* ul, const double* ur, const double* n, RoeJ& J) {
	roe_base(G, ul, ur, n, J.B);
	const RoeAvg& a = J.B.a;
	const double fixeps = 1.0e-4;
	J.l[0] = fabs(a.vn-a.c); J.l[1] = fabs(a.vn); J.l[2] = J.l[1]; J.l[3] = fabs(a.vn+a.c);
	J.delta = fixeps*a.c;
	for(int iv = 0; iv < 4; iv++) {
		J.fixed[iv] = J.l[iv] < J.delta;
		if(J.fixed[iv]) J.l[iv] = (J.l[iv]*J.l[iv] + J.delta*J.delta)/(2.0*J.delta);
	}
	J.devn = J.B.vnj-J.B.vni; J.dep = J.B.pj-J.B.pi; J.derho = ur[0]-ul[0];
	const double rhoij = a.rho, cij = a.c, devn = J.devn, dep = J.dep;
	J.cij4 = cij*cij*cij*cij;
	J.la[0] = J.l[0]*(dep-rhoij*cij*devn)/(2.0*cij*cij);
	J.la[1] = J.l[1]*(J.derho - dep/(cij*cij));
	J.la[2] = J.l[1]*rhoij;
	J.la[3] = J.l[3]*(dep+rhoij*cij*devn)/(2.0*cij*cij);
}

FVHIP_HD void roe_jac_col(const Gas& G, const RoeJ& J, const double* n, int k, double* dl, double* dr) {
	const RoeBase& B = J.B;
	const VarsJ Vi = vars_jac_col(G, B.L, n, k), Vj = vars_jac_col(G, B.R, n, k);
	RoeAvgJ I, Jr;
	roe_avg_jac_col(G, B, n, k, Vi, Vj, I, Jr);
	const double vnij = B.a.vn, cij = B.a.c, rhoij = B.a.rho, vxij = B.a.v[0], vyij = B.a.v[1];
	const double Hij = B.a.H, vm2ij = B.a.vm2;
	const double vxi = B.vi[0], vyi = B.vi[1], vxj = B.vj[0], vyj = B.vj[1];
	const double fixeps = 1.0e-4, delta = J.delta;
	// eigenvalue derivatives
	double dli[4], dlj[4];
	dli[0] = (vnij-cij >= 0 ? 1.0:-1.0)*(I.dvn-I.dc);
	dli[1] = (vnij>=0 ? 1.0:-1.0)*I.dvn;
	dli[2] = dli[1];
	dli[3] = (vnij+cij >= 0 ? 1.0:-1.0)*(I.dvn+I.dc);
	dlj[0] = (vnij-cij >= 0 ? 1.0:-1.0)*(Jr.dvn-Jr.dc);
	dlj[1] = (vnij>=0 ? 1.0:-1.0)*Jr.dvn;
	dlj[2] = dlj[1];
	dlj[3] = (vnij+cij >= 0 ? 1.0:-1.0)*(Jr.dvn+Jr.dc);
	for(int iv = 0; iv < 4; iv++) {
		if(J.fixed[iv]) {
			const double l = J.l[iv];   // the reference differentiates with the already-fixed value
			dli[iv] = ((2.0*(l*dli[iv]+delta*fixeps*I.dc)*2.0*delta) - (l*l+delta*delta)*2.0*fixeps*I.dc) / (4.0*delta*delta);
			dlj[iv] = ((2.0*(l*dlj[iv]+delta*fixeps*Jr.dc)*2.0*delta) - (l*l+delta*delta)*2.0*fixeps*Jr.dc) / (4.0*delta*delta);
		}
	}
	const double devn = J.devn, dep = J.dep, derho = J.derho, cij4 = J.cij4;
	const double* l = J.l; const double* la = J.la;
	const double dderhoi = (k == 0) ? -1.0 : 0, dderhoj = (k == 0) ? 1.0 : 0;
	const double dpi = Vi.dp, dpj = Vj.dp, dvni = Vi.dvn, dvnj = Vj.dvn;
	double dlai[4], dlaj[4];
	dlai[0] = (( dli[0]*(dep-rhoij*cij*devn) +l[0]*(-dpi - I.drho*cij*devn
		-rhoij*I.dc*devn-rhoij*cij*(-dvni)))*2.0*cij*cij - l[0]*(dep-rhoij*cij*devn) *
		4.0*cij*I.dc ) / (4.0*cij4);
	dlaj[0] = (( dlj[0]*(dep-rhoij*cij*devn) +l[0]*(dpj - Jr.drho*cij*devn
		-rhoij*Jr.dc*devn-rhoij*cij*dvnj))*2.0*cij*cij - l[0]*(dep-rhoij*cij*devn) *
		4.0*cij*Jr.dc ) / (4.0*cij4);
	dlai[1] = dli[1]*(derho-dep/(cij*cij))+l[1]*(dderhoi - ((-dpi)*cij*cij - dep*2.0*cij*I.dc)/cij4);
	dlaj[1] = dlj[1]*(derho-dep/(cij*cij))+l[1]*(dderhoj - (dpj*cij*cij - dep*2.0*cij*Jr.dc)/cij4);
	dlai[2] = dli[1]*rhoij + l[1]*I.drho;
	dlaj[2] = dlj[1]*rhoij + l[1]*Jr.drho;
	dlai[3] = ((dli[3]*(dep+rhoij*cij*devn) + l[3]*(-dpi +I.drho*cij*devn
		+rhoij*I.dc*devn+rhoij*cij*(-dvni)))*2.0*cij*cij - l[3]*(dep+rhoij*cij*devn)
		*4.0*cij*I.dc) / (4.0*cij4);
	dlaj[3] = ((dlj[3]*(dep+rhoij*cij*devn) + l[3]*(dpj +Jr.drho*cij*devn
		+rhoij*Jr.dc*devn +rhoij*cij*dvnj))*2.0*cij*cij - l[3]*(dep+rhoij*cij*devn)
		*4.0*cij*Jr.dc) / (4.0*cij4);
	// dissipation derivatives, accumulated in the reference's three passes
	double ai[4], aj[4];
	ai[0] = dlai[0];
	ai[1] = dlai[0]*(vxij-cij*n[0]) + la[0]*(I.dvx-I.dc*n[0]);
	ai[2] = dlai[0]*(vyij-cij*n[1]) + la[0]*(I.dvy-I.dc*n[1]);
	ai[3] = dlai[0]*(Hij-cij*vnij) + la[0]*(I.dH-I.dc*vnij-cij*I.dvn);
	aj[0] = dlaj[0];
	aj[1] = dlaj[0]*(vxij-cij*n[0]) + la[0]*(Jr.dvx-Jr.dc*n[0]);
	aj[2] = dlaj[0]*(vyij-cij*n[1]) + la[0]*(Jr.dvy-Jr.dc*n[1]);
	aj[3] = dlaj[0]*(Hij-cij*vnij) + la[0]*(Jr.dH-Jr.dc*vnij-cij*Jr.dvn);
	ai[0] += dlai[1];
	ai[1] += dlai[1]*vxij+la[1]*I.dvx +dlai[2]*(vxj-vxi-devn*n[0]) +la[2]*(-Vi.dvx+dvni*n[0]);
	ai[2] += dlai[1]*vyij+la[1]*I.dvy +dlai[2]*(vyj-vyi-devn*n[1]) +la[2]*(-Vi.dvy+dvni*n[1]);
	ai[3] += dlai[1]*vm2ij/2.0+la[1]*I.dvm2/2.0
		+dlai[2]*(vxij*(vxj-vxi)+vyij*(vyj-vyi)-vnij*devn)
		+ la[2]*(I.dvx*(vxj-vxi)+vxij*(-Vi.dvx) + I.dvy*(vyj-vyi)+vyij*(-Vi.dvy) -I.dvn*devn-vnij*(-dvni));
	aj[0] += dlaj[1];
	aj[1] += dlaj[1]*vxij+la[1]*Jr.dvx +dlaj[2]*(vxj-vxi-devn*n[0]) +la[2]*(Vj.dvx-dvnj*n[0]);
	aj[2] += dlaj[1]*vyij+la[1]*Jr.dvy +dlaj[2]*(vyj-vyi-devn*n[1]) +la[2]*(Vj.dvy-dvnj*n[1]);
	aj[3] += dlaj[1]*vm2ij/2.0+la[1]*Jr.dvm2/2.0
		+dlaj[2]*(vxij*(vxj-vxi)+vyij*(vyj-vyi)-vnij*devn)
		+ la[2]*(Jr.dvx*(vxj-vxi)+vxij*Vj.dvx + Jr.dvy*(vyj-vyi)+vyij*Vj.dvy -Jr.dvn*devn-vnij*dvnj);
	ai[0] += dlai[3];
	ai[1] += dlai[3]*(vxij+cij*n[0]) + la[3]*(I.dvx+I.dc*n[0]);
	ai[2] += dlai[3]*(vyij+cij*n[1]) + la[3]*(I.dvy+I.dc*n[1]);
	ai[3] += dlai[3]*(Hij+cij*vnij) + la[3]*(I.dH+I.dc*vnij+cij*I.dvn);
	aj[0] += dlaj[3];
	aj[1] += dlaj[3]*(vxij+cij*n[0]) + la[3]*(Jr.dvx+Jr.dc*n[0]);
	aj[2] += dlaj[3]*(vyij+cij*n[1]) + la[3]*(Jr.dvy+Jr.dc*n[1]);
	aj[3] += dlaj[3]*(Hij+cij*vnij) + la[3]*(Jr.dH+Jr.dc*vnij+cij*Jr.dvn);
	double fl[4], fr[4];
	dirflux_jac_col(B.L, n, k, fl);
	dirflux_jac_col(B.R, n, k, fr);
	for(int iv = 0; iv < 4; iv++) {
		dl[iv] = - 0.5*(fl[iv] - ai[iv]);
		dr[iv] =   0.5*(fr[iv] - aj[iv]);
	}
}

// ---------------------------------------------------------------------------------------------
// HLLC, anumericalflux.cpp:1083-1171 (star state) and 1230-1397
// ---------------------------------------------------------------------------------------------
struct HLLCJ {
	RoeBase B;
	double ci, cj, sl, sr, sm, num, denom;
	bool slfromroe, srfromroe;
	int branch;   ///< 0: sl>0, 1: sl<=0<sm, 2: sm<=0<=sr, 3: else
};
FVHIP_HD void hllc_jac_prepare(const Gas& G, const double* ul, const double* ur, const double* n, HLLCJ& J) {
	roe_base(G, ul, ur, n, J.B);
	const RoeBase& B = J.B;
	J.ci = sound_speed(G, ul[0], B.pi);
	J.cj = sound_speed(G, ur[0], B.pj);
	J.sl = B.vni - J.ci;
	J.slfromroe = J.sl > B.a.vn-B.a.c;
	if(J.slfromroe) J.sl = B.a.vn-B.a.c;
	J.sr = B.vnj+J.cj;
	J.srfromroe = J.sr < B.a.vn+B.a.c;
	if(J.srfromroe) J.sr = B.a.vn+B.a.c;
	const double vni = B.vni, vnj = B.vnj, sl = J.sl, sr = J.sr;
	J.num = ( ur[0]*vnj*(sr-vnj) - ul[0]*vni*(sl-vni) + B.pi-B.pj );
	J.denom = (ur[0]*(sr-vnj) - ul[0]*(sl-vni));
	J.sm = J.num / J.denom;
	if(sl > 0) J.branch = 0;
	else if(sl <= 0 && J.sm > 0) J.branch = 1;
	else if(J.sm <= 0 && sr >= 0) J.branch = 2;
	else J.branch = 3;
}

/// column k of getStarStateAndJacobian: this-state derivative (dus_this) and other (dus_other),
/// returns the star state in ustr
FVHIP_HD void hllc_star_col(const double* u, const double* n, double vn, double p, double ss, double sm,
                            double dvn, double dp, double dssi, double dsmi, double dssj, double dsmj, int k,
                            double* ustr, double* dthis, double* dother) {
	const double pstar = u[0]*(vn-ss)*(vn-sm) + p;
	double dpsi, dpsj;
	if(k == 0) {
		dpsi = (vn-ss)*(vn-sm) +u[0]*(dvn-dssi)*(vn-sm) +u[0]*(vn-ss)*(dvn-dsmi) + dp;
		dpsj = u[0]*((-dssj)*(vn-sm) + (vn-ss)*(-dsmj));
	} else {
		dpsi = u[0]*((dvn-dssi)*(vn-sm)+(vn-ss)*(dvn-dsmi)) + dp;
		dpsj = u[0]*((-dssj)*(vn-sm)+(vn-ss)*(-dsmj));
	}
	ustr[0] = u[0] * (ss - vn)/(ss-sm);
	if(k == 0)
		dthis[0] = u[0]*((dssi-dvn)*(ss-sm)-(ss-vn)*(dssi-dsmi))/((ss-sm)*(ss-sm)) + (ss-vn)/(ss-sm);
	else
		dthis[0] = u[0]*((dssi-dvn)*(ss-sm)-(ss-vn)*(dssi-dsmi)) / ((ss-sm)*(ss-sm));
	dother[0] = u[0]*(dssj*(ss-sm)-(ss-vn)*(dssj-dsmj)) / ((ss-sm)*(ss-sm));
	for(int r = 1; r < 3; r++) {
		ustr[r] = ( (ss-vn)*u[r] + (pstar-p)*n[r-1] )/(ss-sm);
		if(k == r)
			dthis[r] = ( ((dssi-dvn)*u[r]+(ss-vn) + (dpsi-dp)*n[r-1])*(ss-sm)
				- ((ss-vn)*u[r]+(pstar-p)*n[r-1])*(dssi-dsmi) )/((ss-sm)*(ss-sm));
		else
			dthis[r] = ( ((dssi-dvn)*u[r] + (dpsi-dp)*n[r-1])*(ss-sm)
				- ((ss-vn)*u[r]+(pstar-p)*n[r-1])*(dssi-dsmi) )/((ss-sm)*(ss-sm));
		dother[r] = ( (dssj*u[r] + dpsj*n[r-1])*(ss-sm)
			- ((ss-vn)*u[r]+(pstar-p)*n[r-1])*(dssj-dsmj) )/((ss-sm)*(ss-sm));
	}
	ustr[3] = ( (ss-vn)*u[3] - p*vn + pstar*sm )/(ss-sm);
	if(k == 3)
		dthis[3] = ( ((dssi-dvn)*u[3]+(ss-vn) -dp*vn-p*dvn +dpsi*sm+pstar*dsmi) * (ss-sm)
			- ((ss-vn)*u[3]-p*vn+pstar*sm)*(dssi-dsmi) )/((ss-sm)*(ss-sm));
	else
		dthis[3] = ( ((dssi-dvn)*u[3] -dp*vn-p*dvn +dpsi*sm+pstar*dsmi) * (ss-sm)
			- ((ss-vn)*u[3]-p*vn+pstar*sm)*(dssi-dsmi) )/((ss-sm)*(ss-sm));
	dother[3] = ( (dssj*u[3] + dpsj*sm+pstar*dsmj)*(ss-sm)
		- ((ss-vn)*u[3]-p*vn+pstar*sm)*(dssj-dsmj) )/((ss-sm)*(ss-sm));
}

FVHIP_HD void hllc_jac_col(const Gas& G, const HLLCJ& J, const double* n, int k, double* dl, double* dr) {
	const RoeBase& B = J.B;
	const double* ul = B.L.u; const double* ur = B.R.u;
	const VarsJ Vi = vars_jac_col(G, B.L, n, k), Vj = vars_jac_col(G, B.R, n, k);
	RoeAvgJ I, Jr;
	roe_avg_jac_col(G, B, n, k, Vi, Vj, I, Jr);
	const double dci = dc_col(G, ul[0], B.pi, Vi.dp, J.ci, k);
	const double dcj = dc_col(G, ur[0], B.pj, Vj.dp, J.cj, k);
	const double dvni = Vi.dvn, dvnj = Vj.dvn, dpi = Vi.dp, dpj = Vj.dp;
	const double vni = B.vni, vnj = B.vnj, sl = J.sl, sr = J.sr, num = J.num, denom = J.denom;
	double dsli = dvni - dci, dslj = 0;
	if(J.slfromroe) { dsli = I.dvn - I.dc; dslj = Jr.dvn - Jr.dc; }
	double dsri = 0, dsrj = dvnj + dcj;
	if(J.srfromroe) { dsri = I.dvn + I.dc; dsrj = Jr.dvn + Jr.dc; }
	double dsmi, dsmj;
	if(k == 0) {
		dsmi = ( (ur[0]*vnj*dsri -vni*(sl-vni)-ul[0]*dvni*(sl-vni)-ul[0]*vni*(dsli-dvni) + dpi )*denom
			-num*(ur[0]*dsri - (sl-vni)-ul[0]*(dsli-dvni)) ) / (denom*denom);
		dsmj = ( (vnj*(sr-vnj)+ur[0]*dvnj*(sr-vnj)+ur[0]*vnj*(dsrj-dvnj) -ul[0]*vni*dslj - dpj)*denom
			-num*((sr-vnj)+ur[0]*(dsrj-dvnj) - ul[0]*dslj) ) / (denom*denom);
	} else {
		dsmi = ( (ur[0]*vnj*dsri - ul[0]*(dvni*(sl-vni)+vni*(dsli-dvni)) +dpi) * denom
			- num *(ur[0]*dsri -ul[0]*(dsli-dvni)) ) / (denom*denom);
		dsmj = ( (ur[0]*(dvnj*(sr-vnj)+vnj*(dsrj-dvnj)) -ul[0]*vni*dslj -dpj) * denom
			- num * (ur[0]*(dsrj-dvnj) - ul[0]*dslj) ) / (denom*denom);
	}
	double fl[4], fr[4];
	switch(J.branch) {
	case 0:
		dirflux_jac_col(B.L, n, k, fl);
		for(int i = 0; i < 4; i++) { dl[i] = fl[i]; dr[i] = 0; }
		break;
	case 1: {
		dirflux_jac_col(B.L, n, k, fl);
		for(int i = 0; i < 4; i++) { dl[i] = fl[i]; dr[i] = 0; }
		double us[4], dthis[4], doth[4];
		hllc_star_col(ul, n, vni, B.pi, sl, J.sm, dvni, dpi, dsli, dsmi, dslj, dsmj, k, us, dthis, doth);
		for(int i = 0; i < 4; i++) {
			dl[i] += dsli*(us[i]-ul[i]) + sl*(dthis[i] - (i==k ? 1.0 : 0.0));
			dr[i] += dslj*(us[i]-ul[i]) + sl*doth[i];
		}
		break;
	}
	case 2: {
		dirflux_jac_col(B.R, n, k, fr);
		for(int i = 0; i < 4; i++) { dr[i] = fr[i]; dl[i] = 0; }
		double us[4], dthis[4], doth[4];
		// reference passes (this = right, other = left): durstrj = d/d(right), durstri = d/d(left)
		hllc_star_col(ur, n, vnj, B.pj, sr, J.sm, dvnj, dpj, dsrj, dsmj, dsri, dsmi, k, us, dthis, doth);
		for(int i = 0; i < 4; i++) {
			dl[i] += dsri*(us[i]-ur[i]) +sr*doth[i];
			dr[i] += dsrj*(us[i]-ur[i]) + sr*(dthis[i] - (i==k ? 1.0:0.0));
		}
		break;
	}
	default:
		dirflux_jac_col(B.R, n, k, fr);
		for(int i = 0; i < 4; i++) { dr[i] = fr[i]; dl[i] = 0; }
	}
	for(int i = 0; i < 4; i++) dl[i] *= -1.0;
}

// ---------------------------------------------------------------------------------------------
// AUSM, anumericalflux.cpp:317-472 (the reference flags it as not working; reproduced as is)
// ---------------------------------------------------------------------------------------------
struct AUSMJ {
	SideJ L, R;
	double vni, vnj, pi, pj, ci, cj, Mni, Mnj, ML, MR, Mh, sg;
	int bl, br;   ///< Mach-split branch: 0 subsonic, 1 supersonic "zero/other side", 2 supersonic own side
};
FVHIP_HD void ausm_jac_prepare(const Gas& G, const double* ul, const double* ur, const double* n, AUSMJ& J) {
	double vi[2], vj[2], Hi, Hj;
	flow_vars(G, ul, n, vi, J.vni, J.pi, Hi);
	flow_vars(G, ur, n, vj, J.vnj, J.pj, Hj);
	J.ci = sound_speed(G, ul[0], J.pi); J.cj = sound_speed(G, ur[0], J.pj);
	J.Mni = J.vni/J.ci; J.Mnj = J.vnj/J.cj;
	if(fabs(J.Mni) <= 1.0) { J.bl = 0; J.ML = 0.25*(J.Mni+1)*(J.Mni+1); }
	else if(J.Mni < -1.0) { J.bl = 1; J.ML = 0; }
	else { J.bl = 2; J.ML = J.Mni; }
	if(fabs(J.Mnj) <= 1.0) { J.br = 0; J.MR = -0.25*(J.Mnj-1)*(J.Mnj-1); }
	else if(J.Mnj < -1.0) { J.br = 2; J.MR = J.Mnj; }
	else { J.br = 1; J.MR = 0; }
	J.Mh = J.ML+J.MR;
	J.sg = (J.Mh>=0 ? 1.0 : -1.0);
	side_prepare(G, ul, n, J.L);
	side_prepare(G, ur, n, J.R);
}
FVHIP_HD void ausm_jac_col(const Gas& G, const AUSMJ& J, const double* n, int k, double* dl, double* dr) {
	const double* ul = J.L.u; const double* ur = J.R.u;
	const double ci = J.ci, cj = J.cj, pi = J.pi, pj = J.pj, vni = J.vni, vnj = J.vnj;
	const double dpi = J.L.dp[k], dpj = J.R.dp[k];
	const double dci = dc_col(G, ul[0], pi, dpi, ci, k);
	const double dcj = dc_col(G, ur[0], pj, dpj, cj, k);
	double dmni, dmnj;
	switch(k) {
	case 0:
		dmni = (-1.0/(ul[0]*ul[0])*(ul[1]*n[0]+ul[2]*n[1])*ci - vni*dci)/(ci*ci);
		dmnj = (-1.0/(ur[0]*ur[0])*(ur[1]*n[0]+ur[2]*n[1])*cj - vnj*dcj)/(cj*cj);
		break;
	case 1:
		dmni = (n[0]/ul[0]*ci - vni*dci)/(ci*ci);
		dmnj = (n[0]/ur[0]*cj - vnj*dcj)/(cj*cj);
		break;
	case 2:
		dmni = (n[1]/ul[0]*ci - vni*dci)/(ci*ci);
		dmnj = (n[1]/ur[0]*cj - vnj*dcj)/(cj*cj);
		break;
	default:
		dmni = -vni*dci/(ci*ci);
		dmnj = -vnj*dcj/(cj*cj);
	}
	const double Mni = J.Mni, Mnj = J.Mnj, ML = J.ML, MR = J.MR, Mh = J.Mh, sg = J.sg;
	double dML = 0, dpL = 0, dMR = 0, dpR = 0;
	if(J.bl == 0) {
		dML = 0.5*(Mni+1)*dmni;
		dpL = dML*pi*(2.0-Mni) + ML*dpi*(2.0-Mni) - ML*pi*dmni;
	} else if(J.bl == 2) { dML = dmni; dpL = dpi; }
	if(J.br == 0) {
		dMR = -0.5*(Mnj-1)*dmnj;
		dpR = -dMR*pj*(2.0+Mnj) - MR*dpj*(2.0+Mnj) - MR*pj*dmnj;
	} else if(J.br == 2) { dMR = dmnj; dpR = dpj; }
	// row 0
	if(k == 0) {
		dl[0] = dML/2.0*(ul[0]*ci+ur[0]*cj) + Mh/2.0*(ci+ul[0]*dci)
			-( sg*dML/2.0*(ur[0]*cj-ul[0]*ci) + fabs(Mh)/2.0*(-ci-ul[0]*dci) );
		dr[0] = dMR/2.0*(ul[0]*ci+ur[0]*cj) + Mh/2.0*(cj+ur[0]*dcj)
			-( sg*dMR/2.0*(ur[0]*cj-ul[0]*ci) + fabs(Mh)/2.0*(cj+ur[0]*dcj) );
	} else {
		dl[0] = dML/2.0*(ul[0]*ci+ur[0]*cj) + Mh/2.0*ul[0]*dci -
			( sg*dML/2.0*(ur[0]*cj-ul[0]*ci) - fabs(Mh)/2.0*ul[0]*dci );
		dr[0] = dMR/2.0*(ul[0]*ci+ur[0]*cj) + Mh/2.0*ur[0]*dcj -
			( sg*dMR/2.0*(ur[0]*cj-ul[0]*ci) + fabs(Mh)/2.0*ur[0]*dcj );
	}
	// momentum rows
	for(int j = 1; j < 3; j++) {
		if(k == j) {
			dl[j] = dML/2.0*(ul[j]*ci+ur[j]*cj) + Mh/2.0*(ci+ul[j]*dci) -
				( sg*dML/2.0*(ur[j]*cj-ul[j]*ci) + fabs(Mh)/2.0*(-ci-ul[j]*dci) ) + dpL*n[j-1];
			dr[j] = dMR/2.0*(ul[j]*ci+ur[j]*cj) + Mh/2.0*(cj+ur[j]*dcj) -
				( sg*dMR/2.0*(ur[j]*cj-ul[j]*ci) + fabs(Mh)/2.0*(cj+ur[j]*dcj) ) + dpR*n[j-1];
		} else {
			dl[j] = dML/2.0*(ul[j]*ci+ur[j]*cj) + Mh/2.0*ul[j]*dci -
				( sg*dML/2.0*(ur[j]*cj-ul[j]*ci) - fabs(Mh)/2.0*ul[j]*dci ) + dpL*n[j-1];
			dr[j] = dMR/2.0*(ul[j]*ci+ur[j]*cj) + Mh/2.0*ur[j]*dcj -
				( sg*dMR/2.0*(ur[j]*cj-ul[j]*ci) + fabs(Mh)/2.0*ur[j]*dcj ) + dpR*n[j-1];
		}
	}
	// energy row
	if(k == 3) {
		dl[3] = dML/2.0*(ci*(ul[3]+pi)+cj*(ur[3]+pj)) + Mh/2.0*(dci*(ul[3]+pi)+ci*(1.0+dpi)) -
			( sg*dML/2.0*(cj*(ur[3]+pj)-ci*(ul[3]+pi)) + fabs(Mh)/2.0*(-dci*(ul[3]+pi)-ci*(1.0+dpi)) );
		dr[3] = dMR/2.0*(ci*(ul[3]+pi)+cj*(ur[3]+pj)) + Mh/2.0*(dcj*(ur[3]+pj)+cj*(1.0+dpj)) -
			( sg*dMR/2.0*(cj*(ur[3]+pj)-ci*(ul[3]+pi)) + fabs(Mh)/2.0*(dcj*(ur[3]+pj)+cj*(1.0+dpj)) );
	} else {
		dl[3] = dML/2.0*(ci*(ul[3]+pi)+cj*(ur[3]+pj)) +Mh/2.0*(dci*(ul[3]+pi)+ci*dpi) -
			( sg*dML/2.0*(cj*(ur[3]+pj)-ci*(ul[3]+pi)) + fabs(Mh)/2.0*(-dci*(ul[3]+pi)-ci*dpi) );
		dr[3] = dMR/2.0*(ci*(ul[3]+pi)+cj*(ur[3]+pj)) +Mh/2.0*(dcj*(ur[3]+pj)+cj*dpj) -
			( sg*dMR/2.0*(cj*(ur[3]+pj)-ci*(ul[3]+pi)) + fabs(Mh)/2.0*(dcj*(ur[3]+pj)+cj*dpj) );
	}
	for(int i = 0; i < 4; i++) dl[i] = -dl[i];
}

// ---------------------------------------------------------------------------------------------
// Dispatch: one object per face, then columns
// ---------------------------------------------------------------------------------------------
template <int FLUX> struct JacOf;
template <> struct JacOf<0> { typedef LLFJ T; };
template <> struct JacOf<2> { typedef AUSMJ T; };
template <> struct JacOf<4> { typedef RoeJ T; };
template <> struct JacOf<5> { typedef HLLJ T; };
template <> struct JacOf<6> { typedef HLLCJ T; };

template <int FLUX>
FVHIP_HD void jac_prepare(const Gas& G, const double* ul, const double* ur, const double* n, typename JacOf<FLUX>::T& J) {
	if constexpr(FLUX == 0) llf_jac_prepare(G, ul, ur, n, J);
	else if constexpr(FLUX == 2) ausm_jac_prepare(G, ul, ur, n, J);
	else if constexpr(FLUX == 4) roe_jac_prepare(G, ul, ur, n, J);
	else if constexpr(FLUX == 5) hll_jac_prepare(G, ul, ur, n, J);
	else hllc_jac_prepare(G, ul, ur, n, J);
}
template <int FLUX>
FVHIP_HD void jac_col(const Gas& G, const typename JacOf<FLUX>::T& J, const double* n, int k, double* dl, double* dr) {
	if constexpr(FLUX == 0) llf_jac_col(J, n, k, dl, dr);
	else if constexpr(FLUX == 2) ausm_jac_col(G, J, n, k, dl, dr);
	else if constexpr(FLUX == 4) roe_jac_col(G, J, n, k, dl, dr);
	else if constexpr(FLUX == 5) hll_jac_col(J, n, k, dl, dr);
	else hllc_jac_col(G, J, n, k, dl, dr);
}

// ---------------------------------------------------------------------------------------------
// Thin-layer viscous flux Jacobian, column k (flow_spatial.cpp:397-446, aspatial.cpp:207-240,
// viscousphysics.cpp:124-246). Adds to dvfi (left) and subtracts from dvfj (right).
// ---------------------------------------------------------------------------------------------
struct ViscJ {
	double upl[4], upr[4];
	double dist, dr[2];
	double grad[2][4];
	double muRe, kdiff;
	double stress[2][2];
	double vavg[2];
	double Tl, Tr;          ///< temperatures (Sutherland only)
	bool constvisc;
};

FVHIP_HD void visc_jac_prepare(const Gas& G, bool constvisc, const double* ul, const double* ur,
                               const double* cl, const double* cr, ViscJ& V) {
	V.constvisc = constvisc;
	cons2prim2(G, ul, V.upl);
	cons2prim2(G, ur, V.upr);
	double dist = 0;
	for(int i = 0; i < 2; i++) { V.dr[i] = cr[i]-cl[i]; dist += V.dr[i]*V.dr[i]; }
	dist = sqrt(dist);
	for(int i = 0; i < 2; i++) V.dr[i] /= dist;
	V.dist = dist;
	for(int i = 0; i < 4; i++) {
		const double corr = (V.upr[i]-V.upl[i])/dist;
		for(int j = 0; j < 2; j++) V.grad[j][i] = corr*V.dr[j];
	}
	V.muRe = constvisc ? 1.0/G.Reinf : 0.5*( sutherland(G, ul) + sutherland(G, ur) );
	V.kdiff = V.muRe / (G.Minf*G.Minf*(G.g-1.0)*G.Pr);
	const double div0 = 0 + V.grad[0][1];
	const double div = div0 + V.grad[1][2];
	const double ldiv = 2.0/3.0*V.muRe*div;
	for(int i = 0; i < 2; i++) {
		for(int j = 0; j < 2; j++) V.stress[i][j] = V.muRe*(V.grad[i][j+1] + V.grad[j][i+1]);
		V.stress[i][i] -= ldiv;
	}
	for(int j = 0; j < 2; j++) V.vavg[j] = 0.5*( ul[j+1]/ul[0] + ur[j+1]/ur[0] );
	V.Tl = temperature(G, ul[0], pressure_cons(G, ul));
	V.Tr = temperature(G, ur[0], pressure_cons(G, ur));
}

/// column k of jacPrim2 (rho, v, T w.r.t. conserved), added onto zero
FVHIP_HD void prim2_jac_col(const Gas& G, const double* uc, int k, double* c) {
	double j0 = 0, j1 = 0, j2 = 0, j3 = 0;
	if(k == 0) j0 += 1.0;
	if(k == 0) { j1 += -uc[1]/(uc[0]*uc[0]); j2 += -uc[2]/(uc[0]*uc[0]); }
	if(k == 1) j1 += 1.0/uc[0];
	if(k == 2) j2 += 1.0/uc[0];
	const double rho2vmag2 = dot2(&uc[1],&uc[1]);
	const double p = (G.g-1.0)*(uc[3] - 0.5*rho2vmag2/uc[0]);
	double dp;
	if(k == 0) dp = (G.g-1.0)*0.5*rho2vmag2/(uc[0]*uc[0]);
	else if(k == 3) dp = (G.g-1.0);
	else dp = -(G.g-1.0)*uc[k]/uc[0];
	const double coef = G.g*G.Minf*G.Minf;
	if(k == 0) j3 += coef*(dp*uc[0] - p)/(uc[0]*uc[0]);
	else j3 += coef/uc[0] * dp;
	c[0] = j0; c[1] = j1; c[2] = j2; c[3] = j3;
}

/// column k of jacSutherland, halved as flow_spatial.cpp:416-420 does
FVHIP_HD double sutherland_jac_col(const Gas& G, const double* uc, double T, int k) {
	const double p = pressure_cons(G, uc);
	double dp;
	if(k == 0) dp = (G.g-1.0)*0.5*dot2(&uc[1],&uc[1])/(uc[0]*uc[0]);
	else if(k == 3) dp = (G.g-1.0);
	else dp = -(G.g-1.0)*uc[k]/uc[0];
	const double coefT = G.g*G.Minf*G.Minf;
	double dT = 0;
	if(k == 0) dT += coefT*(dp*uc[0] - p)/(uc[0]*uc[0]);
	else dT += coefT/uc[0] * dp;
	const double sT = G.sC/G.Tinf;
	const double coef = (1.0+sT)/G.Reinf;
	const double T15 = pow(T,1.5), Tm15 = pow(T,-1.5);
	const double denom = (T + sT)*(T+sT);
	double dmu = 0;
	dmu += coef* (1.5*Tm15*dT*(T+sT) - T15*dT)/denom;
	return dmu * 0.5;
}

FVHIP_HD void visc_jac_col(const Gas& G, const ViscJ& V, const double* ul, const double* ur, const double* n,
                           int k, double* dvfi, double* dvfj) {
	double dupl[4], dupr[4];
	prim2_jac_col(G, ul, k, dupl);
	prim2_jac_col(G, ur, k, dupr);
	double dgl[2][4], dgr[2][4];
	for(int i = 0; i < 4; i++)
		for(int j = 0; j < 2; j++) {
			dgl[j][i] = -dupl[i]/V.dist * V.dr[j];
			dgr[j][i] = dupr[i]/V.dist * V.dr[j];
		}
	double dmul = 0, dmur = 0, dkdl = 0, dkdr = 0;
	if(!V.constvisc) {
		dmul = sutherland_jac_col(G, ul, V.Tl, k);
		dmur = sutherland_jac_col(G, ur, V.Tr, k);
		dkdl = dmul/(G.Minf*G.Minf*(G.g-1.0)*G.Pr);
		dkdr = dmur/(G.Minf*G.Minf*(G.g-1.0)*G.Pr);
	}
	const double mu = V.muRe;
	const double div0 = 0 + V.grad[0][1];
	const double div = div0 + V.grad[1][2];
	double dldl = 0, dldr = 0;
	dldl += dgl[0][1]; dldl += dgl[1][2];
	dldr += dgr[0][1]; dldr += dgr[1][2];
	dldl = 2.0/3.0 * (dmul*div + mu*dldl);
	dldr = 2.0/3.0 * (dmur*div + mu*dldr);
	double dsl[2][2], dsr[2][2];
	for(int i = 0; i < 2; i++) {
		for(int j = 0; j < 2; j++) {
			dsl[i][j] = dmul*(V.grad[i][j+1] + V.grad[j][i+1]) + mu*(dgl[i][j+1] + dgl[j][i+1]);
			dsr[i][j] = dmur*(V.grad[i][j+1] + V.grad[j][i+1]) + mu*(dgr[i][j+1] + dgr[j][i+1]);
		}
		dsl[i][i] -= dldl;
		dsr[i][i] -= dldr;
	}
	for(int i = 0; i < 2; i++)
		for(int j = 0; j < 2; j++) {
			dvfi[i+1] += dsl[i][j] * n[j];
			dvfj[i+1] -= dsr[i][j] * n[j];
		}
	double dval[2], dvar[2];
	for(int j = 0; j < 2; j++) {
		dval[j] = (k == 0) ? -0.5*ul[j+1]/(ul[0]*ul[0]) : (k == j+1) ? 0.5/ul[0] : 0;
		dvar[j] = (k == 0) ? -0.5*ur[j+1]/(ur[0]*ur[0]) : (k == j+1) ? 0.5/ur[0] : 0;
	}
	for(int i = 0; i < 2; i++) {
		double dcl = 0, dcr = 0;
		for(int j = 0; j < 2; j++) {
			dcl += dsl[i][j]*V.vavg[j] + V.stress[i][j]*dval[j];
			dcr += dsr[i][j]*V.vavg[j] + V.stress[i][j]*dvar[j];
		}
		dcl += dkdl*V.grad[i][3] + V.kdiff*dgl[i][3];
		dcr += dkdr*V.grad[i][3] + V.kdiff*dgr[i][3];
		dvfi[3] += dcl * n[i];
		dvfj[3] -= dcr * n[i];
	}
}

// ---------------------------------------------------------------------------------------------
// BC ghost state Jacobians (abc.cpp), full 4x4 (only boundary faces; few)
// ---------------------------------------------------------------------------------------------
FVHIP_HD void ghost_jacobian(const Gas& G, const BCDev& bc, const double* uinf, const double* ins,
                             const double* n, double* gs, double* dgs) {
	for(int k = 0; k < 16; k++) dgs[k] = 0;
	switch(bc.type) {
	case 2: {  // INFLOW_OUTFLOW (abc.cpp:83-133)
		const double vni = dot2(&ins[1],n)/ins[0];
		const double ci = sound_speed_cons(G, ins);
		const double Mni = vni/ci;
		const double pinf = pressure_cons(G, uinf);
		if(Mni <= 0) { for(int i = 0; i < 4; i++) gs[i] = uinf[i]; }
		else if(Mni <= 1) {
			gs[0] = ins[0]; gs[1] = ins[1]; gs[2] = ins[2];
			for(int k = 0; k < 3; k++) dgs[k*4+k] = 1.0;
			gs[3] = energy_from_pressure(G, pinf, ins[0], dot2(&ins[1],&ins[1])/(ins[0]*ins[0]));
			dgs[12] = -0.5*dot2(&ins[1],&ins[1])/(ins[0]*ins[0]);
			dgs[13] = ins[1]/ins[0];
			dgs[14] = ins[2]/ins[0];
			dgs[15] = 0;
		}
		else { for(int i = 0; i < 4; i++) { gs[i] = ins[i]; dgs[i*4+i] = 1.0; } }
		break;
	}
	case 1:
		for(int i = 0; i < 4; i++) gs[i] = uinf[i];
		break;
	case 0: {  // SLIP_WALL (abc.cpp:231-261)
		const double vni = dot2(&ins[1],n)/ins[0];
		double dvni[4];
		dvni[0] = -vni/ins[0]; dvni[1] = n[0]/ins[0]; dvni[2] = n[1]/ins[0]; dvni[3] = 0;
		gs[0] = ins[0]; dgs[0] = 1.0;
		for(int i = 1; i < 3; i++) {
			gs[i] = ins[i] - 2.0*n[i-1]*vni*ins[0];
			dgs[i*4] = -2.0*n[i-1]*(dvni[0]*ins[0] + vni);
			for(int j = 1; j < 3; j++) {
				if(i == j) dgs[i*4+j] = 1.0 - 2.0*n[i-1]*dvni[i]*ins[0];
				else dgs[i*4+j] = -2.0*n[i-1]*dvni[j]*ins[0];
			}
		}
		gs[3] = ins[3]; dgs[15] = 1.0;
		break;
	}
	case 7: {  // ADIABATIC_WALL 2D (abc.cpp:289-310)
		const double tv = bc.v0, tm = tv * ins[0];
		gs[0] = ins[0]; dgs[0] = 1.0;
		gs[1] =  2.0*tm*n[1] - ins[1]; dgs[4] = 2.0*tv*n[1]; dgs[5] = -1.0;
		gs[2] = -2.0*tm*n[0] - ins[2]; dgs[8] = -2.0*tv*n[0]; dgs[10] = -1.0;
		gs[3] = ins[3]; dgs[15] = 1.0;
		break;
	}
	case 6: {  // ISOTHERMAL_WALL (abc.cpp:368-404, reference marks it wrong; reproduced)
		const double tv = bc.v0, Tw = bc.v1, tm = tv * ins[0];
		gs[0] = ins[0]; dgs[0] = 1.0;
		gs[1] =  2.0*tm*n[1] - ins[1]; dgs[4] = 2.0*tv*n[1]; dgs[5] = -1.0;
		gs[2] = -2.0*tm*n[0] - ins[2]; dgs[8] = -2.0*tv*n[0]; dgs[10] = -1.0;
		const double vm2 = dot2(&gs[1],&gs[1])/(ins[0]*ins[0]);
		gs[3] = energy_from_temperature(G, Tw, ins[0], vm2);
		double dvm2[4];
		dvm2[0] = -2.0*dot2(&gs[1],&gs[1])/(ins[0]*ins[0]*ins[0]);
		dvm2[1] = 1.0/(ins[0]*ins[0]) * gs[1] * (-1.0);
		dvm2[2] = 1.0/(ins[0]*ins[0]) * gs[2] * (-1.0);
		dvm2[3] = 0;
		const double dT[4] = {0,0,0,0};
		const double coeff = 1.0/(G.g*(G.g-1.0)*G.Minf*G.Minf);
		dgs[12] += coeff * (Tw+ins[0]*dT[0]) + 0.5 * (vm2+ins[0]*dvm2[0]);
		for(int i = 1; i < 4; i++) dgs[12+i] += ins[0] * (coeff*dT[i] + 0.5*dvm2[i]);
		break;
	}
	default:   // EXTRAPOLATION (abc.cpp:422-433)
		for(int k = 0; k < 4; k++) { gs[k] = ins[k]; dgs[k*4+k] = 1.0; }
	}
}

}
}
#endif
