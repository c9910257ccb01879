/** \file orc_physics.cpp
 * \brief ORACLE (test infrastructure only): analytic flux Jacobians and boundary ghost states,
 *   restated from /root/reference/src/spatial/anumericalflux.cpp and spatial/abc.cpp in the
 *   reference's operation order. See orc_physics.hpp for the parity status.
 */
#include "orc_physics.hpp"
#include <cstdlib>

namespace orc {

// anumericalflux.cpp:317-472 (reference notes it "does not work"; kept for completeness)
void Flux::ausm_jac(const R* ul, const R* ur, const R* n, R* dfdl, R* dfdr) const
{
	R ML, MR;
	R vi[NDIM], vj[NDIM], vni, vnj, pi, pj, Hi, Hj;
	P.varsFromConserved(ul, n, vi, vni, pi, Hi);
	P.varsFromConserved(ur, n, vj, vnj, pj, Hj);
	const R ci = P.soundSpeed(ul[0],pi), cj = P.soundSpeed(ur[0],pj);
	const R Mni = vni/ci, Mnj = vnj/cj;
	R dpi[NVARS], dci[NVARS], dpj[NVARS], dcj[NVARS], dmni[NVARS], dmnj[NVARS];
	R dML[NVARS], dMR[NVARS], dpL[NVARS], dpR[NVARS];
	for(int i = 0; i < NVARS; i++) {
		dpi[i] = 0; dci[i] = 0; dpj[i] = 0; dcj[i] = 0; dmni[i] = 0; dmnj[i] = 0;
		dML[i] = dMR[i] = dpL[i] = dpR[i] = 0;
	}
	P.jacPressure(ul, dpi);
	P.jacPressure(ur, dpj);
	P.jacSoundSpeed(ul[0], pi, dpi, ci, dci);
	P.jacSoundSpeed(ur[0], pj, dpj, cj, dcj);

	dmni[0] = (-1.0/(ul[0]*ul[0])*(ul[1]*n[0]+ul[2]*n[1])*ci - vni*dci[0])/(ci*ci);
	dmni[1] = (n[0]/ul[0]*ci - vni*dci[1])/(ci*ci);
	dmni[2] = (n[1]/ul[0]*ci - vni*dci[2])/(ci*ci);
	dmni[3] = -vni*dci[3]/(ci*ci);
	dmnj[0] = (-1.0/(ur[0]*ur[0])*(ur[1]*n[0]+ur[2]*n[1])*cj - vnj*dcj[0])/(cj*cj);
	dmnj[1] = (n[0]/ur[0]*cj - vnj*dcj[1])/(cj*cj);
	dmnj[2] = (n[1]/ur[0]*cj - vnj*dcj[2])/(cj*cj);
	dmnj[3] = -vnj*dcj[3]/(cj*cj);

	if(std::fabs(Mni) <= 1.0) {
		ML = 0.25*(Mni+1)*(Mni+1);
		for(int k = 0; k < NVARS; k++) dML[k] = 0.5*(Mni+1)*dmni[k];
		for(int k = 0; k < NVARS; k++) dpL[k] = dML[k]*pi*(2.0-Mni) + ML*dpi[k]*(2.0-Mni) - ML*pi*dmni[k];
	}
	else if(Mni < -1.0) { ML = 0; }
	else {
		ML = Mni;
		for(int k = 0; k < NVARS; k++) { dML[k] = dmni[k]; dpL[k] = dpi[k]; }
	}
	if(std::fabs(Mnj) <= 1.0) {
		MR = -0.25*(Mnj-1)*(Mnj-1);
		for(int k = 0; k < NVARS; k++) dMR[k] = -0.5*(Mnj-1)*dmnj[k];
		for(int k = 0; k < NVARS; k++) dpR[k] = -dMR[k]*pj*(2.0+Mnj) - MR*dpj[k]*(2.0+Mnj) - MR*pj*dmnj[k];
	}
	else if(Mnj < -1.0) {
		MR = Mnj;
		for(int k = 0; k < NVARS; k++) { dMR[k] = dmnj[k]; dpR[k] = dpj[k]; }
	}
	else { MR = 0; }

	const R Mh = ML+MR;
	const R sg = (Mh>=0 ? 1.0 : -1.0);
	dfdl[0] = dML[0]/2.0*(ul[0]*ci+ur[0]*cj) + Mh/2.0*(ci+ul[0]*dci[0])
		-( sg*dML[0]/2.0*(ur[0]*cj-ul[0]*ci) + std::fabs(Mh)/2.0*(-ci-ul[0]*dci[0]) );
	dfdr[0] = dMR[0]/2.0*(ul[0]*ci+ur[0]*cj) + Mh/2.0*(cj+ur[0]*dcj[0])
		-( sg*dMR[0]/2.0*(ur[0]*cj-ul[0]*ci) + std::fabs(Mh)/2.0*(cj+ur[0]*dcj[0]) );
	for(int k = 1; k < NVARS; k++) {
		dfdl[k] = dML[k]/2.0*(ul[0]*ci+ur[0]*cj) + Mh/2.0*ul[0]*dci[k] -
			( (Mh>=0 ? 1.0:-1.0)*dML[k]/2.0*(ur[0]*cj-ul[0]*ci) - std::fabs(Mh)/2.0*ul[0]*dci[k] );
		dfdr[k] = dMR[k]/2.0*(ul[0]*ci+ur[0]*cj) + Mh/2.0*ur[0]*dcj[k] -
			( (Mh>=0 ? 1.0:-1.0)*dMR[k]/2.0*(ur[0]*cj-ul[0]*ci) + std::fabs(Mh)/2.0*ur[0]*dcj[k] );
	}
	for(int j = 1; j < NDIM+1; j++) {
		dfdl[j*NVARS+j] = dML[j]/2.0*(ul[j]*ci+ur[j]*cj) + Mh/2.0*(ci+ul[j]*dci[j]) -
			( (Mh>=0? 1.0:-1.0)*dML[j]/2.0*(ur[j]*cj-ul[j]*ci) + std::fabs(Mh)/2.0*(-ci-ul[j]*dci[j]) )
			+ dpL[j]*n[j-1];
		dfdr[j*NVARS+j] = dMR[j]/2.0*(ul[j]*ci+ur[j]*cj) + Mh/2.0*(cj+ur[j]*dcj[j]) -
			( (Mh>=0? 1.0:-1.0)*dMR[j]/2.0*(ur[j]*cj-ul[j]*ci) + std::fabs(Mh)/2.0*(cj+ur[j]*dcj[j]) )
			+ dpR[j]*n[j-1];
		for(int k = 0; k < NVARS; k++) {
			if(k == j) continue;
			dfdl[j*NVARS+k] = dML[k]/2.0*(ul[j]*ci+ur[j]*cj) + Mh/2.0*ul[j]*dci[k] -
				( (Mh>=0?1.0:-1.0)*dML[k]/2.0*(ur[j]*cj-ul[j]*ci) - std::fabs(Mh)/2.0*ul[j]*dci[k] )
				+ dpL[k]*n[j-1];
			dfdr[j*NVARS+k] = dMR[k]/2.0*(ul[j]*ci+ur[j]*cj) + Mh/2.0*ur[j]*dcj[k] -
				( (Mh>=0?1.0:-1.0)*dMR[k]/2.0*(ur[j]*cj-ul[j]*ci) + std::fabs(Mh)/2.0*ur[j]*dcj[k] )
				+ dpR[k]*n[j-1];
		}
	}
	dfdl[3*NVARS+3] =
		dML[3]/2.0*(ci*(ul[3]+pi)+cj*(ur[3]+pj)) + Mh/2.0*(dci[3]*(ul[3]+pi)+ci*(1.0+dpi[3])) -
		( (Mh>=0?1.0:-1.0)*dML[3]/2.0*(cj*(ur[3]+pj)-ci*(ul[3]+pi))
		  +std::fabs(Mh)/2.0*(-dci[3]*(ul[3]+pi)-ci*(1.0+dpi[3])) );
	dfdr[3*NVARS+3] =
		dMR[3]/2.0*(ci*(ul[3]+pi)+cj*(ur[3]+pj)) + Mh/2.0*(dcj[3]*(ur[3]+pj)+cj*(1.0+dpj[3])) -
		( (Mh>=0?1.0:-1.0)*dMR[3]/2.0*(cj*(ur[3]+pj)-ci*(ul[3]+pi))
		  +std::fabs(Mh)/2.0*(dcj[3]*(ur[3]+pj)+cj*(1.0+dpj[3])) );
	for(int k = 0; k < NVARS-1; k++) {
		dfdl[3*NVARS+k] =
		  dML[k]/2.0*(ci*(ul[3]+pi)+cj*(ur[3]+pj)) +Mh/2.0*(dci[k]*(ul[3]+pi)+ci*dpi[k]) -
		  ( (Mh>=0?1.0:-1.0)*dML[k]/2.0*(cj*(ur[3]+pj)-ci*(ul[3]+pi))
			+std::fabs(Mh)/2.0*(-dci[k]*(ul[3]+pi)-ci*dpi[k]) );
		dfdr[3*NVARS+k] =
		  dMR[k]/2.0*(ci*(ul[3]+pi)+cj*(ur[3]+pj)) +Mh/2.0*(dcj[k]*(ur[3]+pj)+cj*dpj[k]) -
		  ( (Mh>=0?1.0:-1.0)*dMR[k]/2.0*(cj*(ur[3]+pj)-ci*(ul[3]+pi))
			+std::fabs(Mh)/2.0*(dcj[k]*(ur[3]+pj)+cj*dpj[k]) );
	}
	for(int k = 0; k < NVARS*NVARS; k++) dfdl[k] = -dfdl[k];
}

// anumericalflux.cpp:567-660
void Flux::roeAvgJac(const R* ul, const R* ur, const R* n, R vxi, R vyi, R Hi, R vxj, R vyj, R Hj,
                     const R* dvxi, const R* dvyi, const R* dHi, const R* dvxj, const R* dvyj, const R* dHj,
                     R* dRiji, R* drhoiji, R* dvxiji, R* dvyiji, R* dvm2iji, R* dvniji, R* dHiji, R* dciji,
                     R* dRijj, R* drhoijj, R* dvxijj, R* dvyijj, R* dvm2ijj, R* dvnijj, R* dHijj, R* dcijj) const
{
	(void)dvxi; (void)dvyi; (void)dvxj; (void)dvyj;
	R Rij,rhoij,vm2ij,vnij,Hij,cij;
	R vi[NDIM] = {vxi, vyi}, vj[NDIM] = {vxj, vyj}, vij[NDIM];
	roeAverages(ul,ur,n,vi,Hi,vj,Hj, Rij,rhoij,vij,vm2ij,vnij,Hij,cij);
	const R vxij = vij[0], vyij = vij[1];

	dRiji[0] = 0.5/Rij * (-ur[0])/(ul[0]*ul[0]);
	dRijj[0] = 0.5/Rij / ul[0];
	for(int k = 1; k < NVARS; k++) { dRiji[k] = 0; dRijj[k] = 0; }
	const R rden2 = (Rij+1.0)*(Rij+1.0);

	dvxiji[0] = ((dRiji[0]*ur[1]/ur[0] -ul[1]/(ul[0]*ul[0]))*(Rij+1.0) -(Rij*vxj+vxi)*dRiji[0])/rden2;
	dvxiji[1] = ((dRiji[1]*ur[1]/ur[0] + 1.0/ul[0])*(Rij+1.0)-(Rij*vxj+vxi)*dRiji[1])/rden2;
	dvxiji[2] = (dRiji[2]*ur[1]/ur[0] *(Rij+1.0)- (Rij*vxj+vxi)*dRiji[2])/rden2;
	dvxiji[3] = (dRiji[3]*ur[1]/ur[0] *(Rij+1.0)- (Rij*vxj+vxi)*dRiji[3])/rden2;
	dvxijj[0] = ((dRijj[0]*ur[1]/ur[0] +Rij/(ur[0]*ur[0])*(-ur[1]))*(Rij+1.0) -(Rij*vxj+vxi)*dRijj[0]) / rden2;
	dvxijj[1] = ((dRijj[1]*ur[1]/ur[0] +Rij/ur[0])*(Rij+1.0)-(Rij*vxj+vxi)*dRijj[1]) / rden2;
	dvxijj[2] = (dRijj[2]*ur[1]/ur[0] *(Rij+1.0) - (Rij*vxj+vxi)*dRijj[2]) / rden2;
	dvxijj[3] = (dRijj[3]*ur[1]/ur[0] *(Rij+1.0) - (Rij*vxj+vxi)*dRijj[3]) / rden2;

	dvyiji[0] = ((ur[2]/ur[0]*dRiji[0] - ul[2]/(ul[0]*ul[0]))*(Rij+1.0) -(Rij*vyj+vyi)*dRiji[0]) / rden2;
	dvyiji[1] = (ur[2]/ur[0]*dRiji[1] *(Rij+1.0) - (Rij*vyj+vyi)*dRiji[1]) / rden2;
	dvyiji[2] = ((ur[2]/ur[0]*dRiji[2] + 1.0/ul[0])*(Rij+1.0) -(Rij*vyj+vyi)*dRiji[2]) / rden2;
	dvyiji[3] = (ur[2]/ur[0]*dRiji[3] *(Rij+1.0) -(Rij*vyj+vyi)*dRiji[3]) / rden2;
	dvyijj[0] = ((dRijj[0]*ur[2]/ur[0] + Rij/(ur[0]*ur[0])*(-ur[2]))*(Rij+1.0) -(Rij*vyj+vyi)*dRijj[0] ) / rden2;
	dvyijj[1] = (dRijj[1]*ur[2]/ur[0] *(Rij+1.0) -(Rij*vyj+vyi)*dRijj[1]) / rden2;
	dvyijj[2] = ((dRijj[2]*ur[2]/ur[0] + Rij/ur[0])*(Rij+1.0) -(Rij*vyj+vyi)*dRijj[2]) / rden2;
	dvyijj[3] = (dRijj[3]*ur[2]/ur[0] *(Rij+1.0) - (Rij*vyj+vyi)*dRijj[3]) / rden2;

	for(int k = 0; k < NVARS; k++) {
		dvniji[k] = dvxiji[k]*n[0] + dvyiji[k]*n[1];
		dvnijj[k] = dvxijj[k]*n[0] + dvyijj[k]*n[1];
		dvm2iji[k] = 2.0*( vxij*dvxiji[k] + vyij*dvyiji[k] );
		dvm2ijj[k] = 2.0*( vxij*dvxijj[k] + vyij*dvyijj[k] );
	}
	for(int k = 0; k < NVARS; k++) {
		dciji[k] = 0.5/cij*(g-1.0) * (((dRiji[k]*Hj+dHi[k])*(Rij+1)-(Rij*Hj+Hi)*dRiji[k])/rden2 - 0.5*dvm2iji[k]);
		dcijj[k] = 0.5/cij*(g-1.0) * (((dRijj[k]*Hj+Rij*dHj[k])*(Rij+1) - (Rij*Hj+Hi)*dRijj[k])/rden2 - 0.5*dvm2ijj[k] );
	}
	drhoiji[0] = dRiji[0]*ul[0] + Rij;
	drhoijj[0] = dRijj[0]*ul[0];
	for(int k = 1; k < NVARS; k++) { drhoiji[k] = 0; drhoijj[k] = 0; }
	for(int k = 0; k < NVARS; k++) {
		dHiji[k] = ((dRiji[k]*Hj+dHi[k])*(Rij+1.0)-(Rij*Hj+Hi)*dRiji[k])/rden2;
		dHijj[k] = ((dRijj[k]*Hj+Rij*dHj[k])*(Rij+1.0)-(Rij*Hj+Hi)*dRijj[k])/rden2;
	}
}

// anumericalflux.cpp:736-965
void Flux::roe_jac(const R* ul, const R* ur, const R* n, R* dfdl, R* dfdr) const
{
	R vi[NDIM], vj[NDIM], vni, vnj, pi, pj, Hi, Hj;
	P.varsFromConserved(ul, n, vi, vni, pi, Hi);
	P.varsFromConserved(ur, n, vj, vnj, pj, Hj);
	const R vxi = vi[0], vxj = vj[0], vyi = vi[1], vyj = vj[1];
	R Rij,rhoij,vm2ij,vnij,Hij,cij,vij[NDIM];
	roeAverages(ul,ur,n,vi,Hi,vj,Hj, Rij,rhoij,vij,vm2ij,vnij,Hij,cij);
	const R vxij = vij[0], vyij = vij[1];
	const R fixeps = 1.0e-4;

	R dpi[NVARS], dpj[NVARS], dvni[NVARS], dvnj[NVARS], dvi[NDIM*NVARS], dvj[NDIM*NVARS], dHi[NVARS], dHj[NVARS],
	  dRiji[NVARS], dRijj[NVARS], dvxiji[NVARS], dvyiji[NVARS], dvxijj[NVARS], dvyijj[NVARS],
	  dvniji[NVARS], dvnijj[NVARS], dvm2iji[NVARS], dvm2ijj[NVARS], dciji[NVARS], dcijj[NVARS],
	  drhoiji[NVARS], drhoijj[NVARS], dHiji[NVARS], dHijj[NVARS];
	for(int k = 0; k < NVARS; k++) {
		dpi[k] = dpj[k] = dHi[k] = dHj[k] = 0;
		dvni[k] = dvnj[k] = 0;
		for(int j = 0; j < NDIM; j++) { dvi[j*NVARS+k] = 0; dvj[j*NVARS+k] = 0; }
	}
	P.jacVars(ul,n,dvi,dvni,dpi,dHi);
	P.jacVars(ur,n,dvj,dvnj,dpj,dHj);
	R dvxj[NVARS], dvyj[NVARS], dvxi[NVARS], dvyi[NVARS];
	for(int k = 0; k < NVARS; k++) {
		dvxi[k] = dvi[k]; dvxj[k] = dvj[k]; dvyi[k] = dvi[NVARS+k]; dvyj[k] = dvj[NVARS+k];
	}
	roeAvgJac(ul,ur,n,vxi,vyi,Hi,vxj,vyj,Hj,dvxi,dvyi,dHi,dvxj,dvyj,dHj,
	          dRiji, drhoiji, dvxiji, dvyiji, dvm2iji, dvniji, dHiji, dciji,
	          dRijj, drhoijj, dvxijj, dvyijj, dvm2ijj, dvnijj, dHijj, dcijj);

	R l[NVARS];
	l[0] = std::fabs(vnij-cij); l[1] = std::fabs(vnij); l[2] = l[1]; l[3] = std::fabs(vnij+cij);
	R dli[NVARS][NVARS], dlj[NVARS][NVARS];
	for(int k = 0; k < NVARS; k++) {
		dli[0][k] = (vnij-cij >= 0 ? 1.0:-1.0)*(dvniji[k]-dciji[k]);
		dli[1][k] = (vnij>=0 ? 1.0:-1.0)*dvniji[k];
		dli[2][k] = dli[1][k];
		dli[3][k] = (vnij+cij >= 0 ? 1.0:-1.0)*(dvniji[k]+dciji[k]);
		dlj[0][k] = (vnij-cij >= 0 ? 1.0:-1.0)*(dvnijj[k]-dcijj[k]);
		dlj[1][k] = (vnij>=0 ? 1.0:-1.0)*dvnijj[k];
		dlj[2][k] = dlj[1][k];
		dlj[3][k] = (vnij+cij >= 0 ? 1.0:-1.0)*(dvnijj[k]+dcijj[k]);
	}
	const R delta = fixeps*cij;
	for(int iv = 0; iv < NVARS; iv++) {
		if(l[iv] < delta) {
			l[iv] = (l[iv]*l[iv] + delta*delta)/(2.0*delta);
			for(int k = 0; k < NVARS; k++) {
				dli[iv][k] = ((2.0*(l[iv]*dli[iv][k]+delta*fixeps*dciji[k])*2.0*delta)
					- (l[iv]*l[iv]+delta*delta)*2.0*fixeps*dciji[k]) / (4.0*delta*delta);
				dlj[iv][k] = ((2.0*(l[iv]*dlj[iv][k]+delta*fixeps*dcijj[k])*2.0*delta)
					- (l[iv]*l[iv]+delta*delta)*2.0*fixeps*dcijj[k]) / (4.0*delta*delta);
			}
		}
	}

	const R devn = vnj-vni, dep = pj-pi, derho = ur[0]-ul[0];
	R dderhoi[NVARS], dderhoj[NVARS];
	dderhoi[0] = -1.0; dderhoj[0] = 1.0;
	for(int k = 1; k < NVARS; k++) { dderhoi[k] = 0; dderhoj[k] = 0; }

	R la[NVARS], dlai[NVARS][NVARS], dlaj[NVARS][NVARS];
	const R cij4 = cij*cij*cij*cij;
	la[0] = l[0]*(dep-rhoij*cij*devn)/(2.0*cij*cij);
	for(int k = 0; k < NVARS; k++) {
		dlai[0][k] = (( dli[0][k]*(dep-rhoij*cij*devn) +l[0]*(-dpi[k] - drhoiji[k]*cij*devn
			-rhoij*dciji[k]*devn-rhoij*cij*(-dvni[k])))*2.0*cij*cij - l[0]*(dep-rhoij*cij*devn) *
			4.0*cij*dciji[k] ) / (4.0*cij4);
		dlaj[0][k] = (( dlj[0][k]*(dep-rhoij*cij*devn) +l[0]*(dpj[k] - drhoijj[k]*cij*devn
			-rhoij*dcijj[k]*devn-rhoij*cij*dvnj[k]))*2.0*cij*cij - l[0]*(dep-rhoij*cij*devn) *
			4.0*cij*dcijj[k] ) / (4.0*cij4);
	}
	la[1] = l[1]*(derho - dep/(cij*cij));
	for(int k = 0; k < NVARS; k++) {
		dlai[1][k] = dli[1][k]*(derho-dep/(cij*cij))+l[1]*(dderhoi[k] - ((-dpi[k])*cij*cij
			- dep*2.0*cij*dciji[k])/cij4);
		dlaj[1][k] = dlj[1][k]*(derho-dep/(cij*cij))+l[1]*(dderhoj[k] - (dpj[k]*cij*cij
			- dep*2.0*cij*dcijj[k])/cij4);
	}
	la[2] = l[1]*rhoij;
	for(int k = 0; k < NVARS; k++) {
		dlai[2][k] = dli[1][k]*rhoij + l[1]*drhoiji[k];
		dlaj[2][k] = dlj[1][k]*rhoij + l[1]*drhoijj[k];
	}
	la[3] = l[3]*(dep+rhoij*cij*devn)/(2.0*cij*cij);
	for(int k = 0; k < NVARS; k++) {
		dlai[3][k] = ((dli[3][k]*(dep+rhoij*cij*devn) + l[3]*(-dpi[k] +drhoiji[k]*cij*devn
			+rhoij*dciji[k]*devn+rhoij*cij*(-dvni[k])))*2.0*cij*cij - l[3]*(dep+rhoij*cij*devn)
			*4.0*cij*dciji[k]) / (4.0*cij4);
		dlaj[3][k] = ((dlj[3][k]*(dep+rhoij*cij*devn) + l[3]*(dpj[k] +drhoijj[k]*cij*devn
			+rhoij*dcijj[k]*devn +rhoij*cij*dvnj[k]))*2.0*cij*cij - l[3]*(dep+rhoij*cij*devn)
			*4.0*cij*dcijj[k]) / (4.0*cij4);
	}

	R dadui[NVARS][NVARS], daduj[NVARS][NVARS];
	for(int k = 0; k < NVARS; k++) {
		dadui[0][k] = dlai[0][k];
		dadui[1][k] = dlai[0][k]*(vxij-cij*n[0]) + la[0]*(dvxiji[k]-dciji[k]*n[0]);
		dadui[2][k] = dlai[0][k]*(vyij-cij*n[1]) + la[0]*(dvyiji[k]-dciji[k]*n[1]);
		dadui[3][k] = dlai[0][k]*(Hij-cij*vnij) + la[0]*(dHiji[k]-dciji[k]*vnij-cij*dvniji[k]);
		daduj[0][k] = dlaj[0][k];
		daduj[1][k] = dlaj[0][k]*(vxij-cij*n[0]) + la[0]*(dvxijj[k]-dcijj[k]*n[0]);
		daduj[2][k] = dlaj[0][k]*(vyij-cij*n[1]) + la[0]*(dvyijj[k]-dcijj[k]*n[1]);
		daduj[3][k] = dlaj[0][k]*(Hij-cij*vnij) + la[0]*(dHijj[k]-dcijj[k]*vnij-cij*dvnijj[k]);
	}
	for(int k = 0; k < NVARS; k++) {
		dadui[0][k] += dlai[1][k];
		dadui[1][k] += dlai[1][k]*vxij+la[1]*dvxiji[k]
			+dlai[2][k]*(vxj-vxi-devn*n[0]) +la[2]*(-dvxi[k]+dvni[k]*n[0]);
		dadui[2][k] += dlai[1][k]*vyij+la[1]*dvyiji[k]
			+dlai[2][k]*(vyj-vyi-devn*n[1]) +la[2]*(-dvyi[k]+dvni[k]*n[1]);
		dadui[3][k] += dlai[1][k]*vm2ij/2.0+la[1]*dvm2iji[k]/2.0
			+dlai[2][k]*(vxij*(vxj-vxi)+vyij*(vyj-vyi)-vnij*devn)
			+ la[2]*(dvxiji[k]*(vxj-vxi)+vxij*(-dvxi[k]) + dvyiji[k]*(vyj-vyi)+vyij*(-dvyi[k])
			-dvniji[k]*devn-vnij*(-dvni[k]));
		daduj[0][k] += dlaj[1][k];
		daduj[1][k] += dlaj[1][k]*vxij+la[1]*dvxijj[k]
			+dlaj[2][k]*(vxj-vxi-devn*n[0]) +la[2]*(dvxj[k]-dvnj[k]*n[0]);
		daduj[2][k] += dlaj[1][k]*vyij+la[1]*dvyijj[k]
			+dlaj[2][k]*(vyj-vyi-devn*n[1]) +la[2]*(dvyj[k]-dvnj[k]*n[1]);
		daduj[3][k] += dlaj[1][k]*vm2ij/2.0+la[1]*dvm2ijj[k]/2.0
			+dlaj[2][k]*(vxij*(vxj-vxi)+vyij*(vyj-vyi)-vnij*devn)
			+ la[2]*(dvxijj[k]*(vxj-vxi)+vxij*dvxj[k] + dvyijj[k]*(vyj-vyi)+vyij*dvyj[k]
			-dvnijj[k]*devn-vnij*dvnj[k]);
	}
	for(int k = 0; k < NVARS; k++) {
		dadui[0][k] += dlai[3][k];
		dadui[1][k] += dlai[3][k]*(vxij+cij*n[0]) + la[3]*(dvxiji[k]+dciji[k]*n[0]);
		dadui[2][k] += dlai[3][k]*(vyij+cij*n[1]) + la[3]*(dvyiji[k]+dciji[k]*n[1]);
		dadui[3][k] += dlai[3][k]*(Hij+cij*vnij) + la[3]*(dHiji[k]+dciji[k]*vnij+cij*dvniji[k]);
		daduj[0][k] += dlaj[3][k];
		daduj[1][k] += dlaj[3][k]*(vxij+cij*n[0]) + la[3]*(dvxijj[k]+dcijj[k]*n[0]);
		daduj[2][k] += dlaj[3][k]*(vyij+cij*n[1]) + la[3]*(dvyijj[k]+dcijj[k]*n[1]);
		daduj[3][k] += dlaj[3][k]*(Hij+cij*vnij) + la[3]*(dHijj[k]+dcijj[k]*vnij+cij*dvnijj[k]);
	}
	P.jacDirFlux(ul, n, dfdl);
	P.jacDirFlux(ur, n, dfdr);
	for(int iv = 0; iv < NVARS; iv++)
		for(int k = 0; k < NVARS; k++) {
			dfdl[iv*NVARS+k] = - 0.5*(dfdl[iv*NVARS+k] - dadui[iv][k]);
			dfdr[iv*NVARS+k] =   0.5*(dfdr[iv*NVARS+k] - daduj[iv][k]);
		}
}

// anumericalflux.cpp:1012-1061 (frozen signal speeds)
void Flux::hll_jac(const R* ul, const R* ur, const R* n, R* dfdl, R* dfdr) const
{
	R vi[NDIM], vj[NDIM], vni, vnj, pi, pj, Hi, Hj, ci, cj;
	P.varsFromConserved(ul, n, vi, vni, pi, Hi);
	P.varsFromConserved(ur, n, vj, vnj, pj, Hj);
	ci = P.soundSpeed(ul[0], pi);
	cj = P.soundSpeed(ur[0], pj);
	R Rij,rhoij,vm2ij,vnij,Hij,cij,vij[NDIM];
	roeAverages(ul,ur,n,vi,Hi,vj,Hj, Rij,rhoij,vij,vm2ij,vnij,Hij,cij);
	R sr, sl;
	sl = vni - ci;
	if (sl > vnij-cij) sl = vnij-cij;
	sr = vnj+cj;
	if(sr < vnij+cij) sr = vnij+cij;
	const R sr0 = sr > 0 ? 0 : sr;
	const R sl0 = sl > 0 ? 0 : sl;
	const R t1 = (sr0 - sl0)/(sr-sl);
	const R t2 = 1.0 - t1;
	const R t3 = 0.5*(sr*std::fabs(sl)-sl*std::fabs(sr))/(sr-sl);
	P.jacDirFlux(ul, n, dfdl);
	P.jacDirFlux(ur, n, dfdr);
	for(int i = 0; i < NVARS; i++)
		for(int j = 0; j < NVARS; j++) {
			dfdl[i*NVARS+j] = -t2*dfdl[i*NVARS+j];
			dfdr[i*NVARS+j] =  t1*dfdr[i*NVARS+j];
		}
	for(int i = 0; i < NVARS; i++) {
		dfdl[i*NVARS+i] = dfdl[i*NVARS+i] - t3;
		dfdr[i*NVARS+i] = dfdr[i*NVARS+i] - t3;
	}
}

// anumericalflux.cpp:1083-1171
void Flux::starStateJac(const R* u, const R* n, R vn, R p, R ss, R sm, const R* dvn, const R* dp,
                        const R* dssi, const R* dsmi, const R* dssj, const R* dsmj,
                        R* ustr, R dustri[NVARS][NVARS], R dustrj[NVARS][NVARS]) const
{
	const R pstar = u[0]*(vn-ss)*(vn-sm) + p;
	R dpsi[NVARS], dpsj[NVARS];
	dpsi[0] = (vn-ss)*(vn-sm) +u[0]*(dvn[0]-dssi[0])*(vn-sm) +u[0]*(vn-ss)*(dvn[0]-dsmi[0]) + dp[0];
	dpsj[0] = u[0]*((-dssj[0])*(vn-sm) + (vn-ss)*(-dsmj[0]));
	for(int k = 1; k < NVARS; k++) {
		dpsi[k] = u[0]*((dvn[k]-dssi[k])*(vn-sm)+(vn-ss)*(dvn[k]-dsmi[k])) + dp[k];
		dpsj[k] = u[0]*((-dssj[k])*(vn-sm)+(vn-ss)*(-dsmj[k]));
	}
	const R D = (ss-sm)*(ss-sm);
	ustr[0] = u[0] * (ss - vn)/(ss-sm);
	dustri[0][0]=u[0]*((dssi[0]-dvn[0])*(ss-sm)-(ss-vn)*(dssi[0]-dsmi[0]))/((ss-sm)*(ss-sm)) + (ss-vn)/(ss-sm);
	dustrj[0][0]=u[0]*(dssj[0]*(ss-sm)-(ss-vn)*(dssj[0]-dsmj[0])) / ((ss-sm)*(ss-sm));
	for(int k = 1; k < NVARS; k++) {
		dustri[0][k]=u[0]*((dssi[k]-dvn[k])*(ss-sm)-(ss-vn)*(dssi[k]-dsmi[k])) / ((ss-sm)*(ss-sm));
		dustrj[0][k]=u[0]*(dssj[k]*(ss-sm)-(ss-vn)*(dssj[k]-dsmj[k])) / ((ss-sm)*(ss-sm));
	}
	(void)D;
	ustr[1] = ( (ss-vn)*u[1] + (pstar-p)*n[0] )/(ss-sm);
	for(int k = 0; k < NVARS; k++) {
		if(k == 1) continue;
		dustri[1][k]= ( ((dssi[k]-dvn[k])*u[1] + (dpsi[k]-dp[k])*n[0])*(ss-sm)
			- ((ss-vn)*u[1]+(pstar-p)*n[0])*(dssi[k]-dsmi[k]) )/((ss-sm)*(ss-sm));
		dustrj[1][k]= ( (dssj[k]*u[1] + dpsj[k]*n[0])*(ss-sm)
			- ((ss-vn)*u[1]+(pstar-p)*n[0])*(dssj[k]-dsmj[k]) )/((ss-sm)*(ss-sm));
	}
	dustri[1][1]= ( ((dssi[1]-dvn[1])*u[1]+(ss-vn) + (dpsi[1]-dp[1])*n[0])*(ss-sm)
			- ((ss-vn)*u[1]+(pstar-p)*n[0])*(dssi[1]-dsmi[1]) )/((ss-sm)*(ss-sm));
	dustrj[1][1]= ( (dssj[1]*u[1] + dpsj[1]*n[0])*(ss-sm)
		- ((ss-vn)*u[1]+(pstar-p)*n[0])*(dssj[1]-dsmj[1]) )/((ss-sm)*(ss-sm));
	ustr[2] = ( (ss-vn)*u[2] + (pstar-p)*n[1] )/(ss-sm);
	for(int k = 0; k < NVARS; k++) {
		if(k == 2) continue;
		dustri[2][k]= ( ((dssi[k]-dvn[k])*u[2] + (dpsi[k]-dp[k])*n[1])*(ss-sm)
			- ((ss-vn)*u[2]+(pstar-p)*n[1])*(dssi[k]-dsmi[k]) )/((ss-sm)*(ss-sm));
		dustrj[2][k]= ( (dssj[k]*u[2] + dpsj[k]*n[1])*(ss-sm)
			- ((ss-vn)*u[2]+(pstar-p)*n[1])*(dssj[k]-dsmj[k]) )/((ss-sm)*(ss-sm));
	}
	dustri[2][2]= ( ((dssi[2]-dvn[2])*u[2]+(ss-vn) + (dpsi[2]-dp[2])*n[1])*(ss-sm)
			- ((ss-vn)*u[2]+(pstar-p)*n[1])*(dssi[2]-dsmi[2]) )/((ss-sm)*(ss-sm));
	dustrj[2][2]= ( (dssj[2]*u[2] + dpsj[2]*n[1])*(ss-sm)
		- ((ss-vn)*u[2]+(pstar-p)*n[1])*(dssj[2]-dsmj[2]) )/((ss-sm)*(ss-sm));
	ustr[3] = ( (ss-vn)*u[3] - p*vn + pstar*sm )/(ss-sm);
	for(int k = 0; k < NVARS-1; k++) {
		dustri[3][k]= ( ((dssi[k]-dvn[k])*u[3] -dp[k]*vn-p*dvn[k] +dpsi[k]*sm+pstar*dsmi[k]) * (ss-sm)
			- ((ss-vn)*u[3]-p*vn+pstar*sm)*(dssi[k]-dsmi[k]) )/((ss-sm)*(ss-sm));
		dustrj[3][k]= ( (dssj[k]*u[3] + dpsj[k]*sm+pstar*dsmj[k])*(ss-sm)
			- ((ss-vn)*u[3]-p*vn+pstar*sm)*(dssj[k]-dsmj[k]) )/((ss-sm)*(ss-sm));
	}
	dustri[3][3]= ( ((dssi[3]-dvn[3])*u[3]+(ss-vn) -dp[3]*vn-p*dvn[3] +dpsi[3]*sm+pstar*dsmi[3]) * (ss-sm)
		- ((ss-vn)*u[3]-p*vn+pstar*sm)*(dssi[3]-dsmi[3]) )/((ss-sm)*(ss-sm));
	dustrj[3][3]= ( (dssj[3]*u[3] + dpsj[3]*sm+pstar*dsmj[3])*(ss-sm)
		- ((ss-vn)*u[3]-p*vn+pstar*sm)*(dssj[3]-dsmj[3]) )/((ss-sm)*(ss-sm));
}

// anumericalflux.cpp:1230-1397
void Flux::hllc_jac(const R* ul, const R* ur, const R* n, R* dfdl, R* dfdr) const
{
	R vi[NDIM], vj[NDIM], vni, vnj, pi, pj, Hi, Hj, ci, cj;
	P.varsFromConserved(ul, n, vi, vni, pi, Hi);
	P.varsFromConserved(ur, n, vj, vnj, pj, Hj);
	ci = P.soundSpeed(ul[0], pi);
	cj = P.soundSpeed(ur[0], pj);
	const R vxi = vi[0], vxj = vj[0], vyi = vi[1], vyj = vj[1];
	R Rij,rhoij,vm2ij,vnij,Hij,cij,vij[NDIM];
	roeAverages(ul,ur,n,vi,Hi,vj,Hj, Rij,rhoij,vij,vm2ij,vnij,Hij,cij);

	R dpi[NVARS], dpj[NVARS], dvni[NVARS], dvnj[NVARS], dvi[NDIM*NVARS], dvj[NDIM*NVARS],
	  dHi[NVARS], dHj[NVARS], dci[NVARS], dcj[NVARS],
	  dRiji[NVARS], dRijj[NVARS], dvxiji[NVARS], dvyiji[NVARS], dvxijj[NVARS], dvyijj[NVARS],
	  dvniji[NVARS], dvnijj[NVARS], dvm2iji[NVARS], dvm2ijj[NVARS], dciji[NVARS], dcijj[NVARS],
	  drhoiji[NVARS], drhoijj[NVARS], dHiji[NVARS], dHijj[NVARS];
	for(int k = 0; k < NVARS; k++) {
		dpi[k] = dpj[k] = dHi[k] = dHj[k] = dci[k] = dcj[k] = 0;
		dvni[k] = dvnj[k] = 0;
		for(int j = 0; j < NDIM; j++) { dvi[j*NVARS+k] = 0; dvj[j*NVARS+k] = 0; }
	}
	P.jacVars(ul,n,dvi,dvni,dpi,dHi);
	P.jacVars(ur,n,dvj,dvnj,dpj,dHj);
	P.jacSoundSpeed(ul[0],pi,dpi,ci,dci);
	P.jacSoundSpeed(ur[0],pj,dpj,cj,dcj);
	R dvxi[NVARS], dvxj[NVARS], dvyi[NVARS], dvyj[NVARS];
	for(int k = 0; k < NVARS; k++) {
		dvxi[k] = dvi[k]; dvxj[k] = dvj[k]; dvyi[k] = dvi[NVARS+k]; dvyj[k] = dvj[NVARS+k];
	}
	roeAvgJac(ul,ur,n,vxi,vyi,Hi,vxj,vyj,Hj,dvxi,dvyi,dHi,dvxj,dvyj,dHj,
	          dRiji, drhoiji, dvxiji, dvyiji, dvm2iji, dvniji, dHiji, dciji,
	          dRijj, drhoijj, dvxijj, dvyijj, dvm2ijj, dvnijj, dHijj, dcijj);

	R sr, sl, dsli[NVARS], dslj[NVARS], dsri[NVARS], dsrj[NVARS];
	sl = vni - ci;
	for(int k = 0; k < NVARS; k++) { dsli[k] = dvni[k] - dci[k]; dslj[k] = 0; }
	if (sl > vnij-cij) {
		sl = vnij-cij;
		for(int k = 0; k < NVARS; k++) { dsli[k] = dvniji[k] - dciji[k]; dslj[k] = dvnijj[k] - dcijj[k]; }
	}
	sr = vnj+cj;
	for(int k = 0; k < NVARS; k++) { dsri[k] = 0; dsrj[k] = dvnj[k] + dcj[k]; }
	if(sr < vnij+cij) {
		sr = vnij+cij;
		for(int k = 0; k < NVARS; k++) { dsri[k] = dvniji[k] + dciji[k]; dsrj[k] = dvnijj[k] + dcijj[k]; }
	}
	const R num = ( ur[0]*vnj*(sr-vnj) - ul[0]*vni*(sl-vni) + pi-pj );
	const R denom = (ur[0]*(sr-vnj) - ul[0]*(sl-vni));
	const R sm = num / denom;
	R dsmi[NVARS], dsmj[NVARS];
	dsmi[0]= ( (ur[0]*vnj*dsri[0] -vni*(sl-vni)-ul[0]*dvni[0]*(sl-vni)-ul[0]*vni*(dsli[0]-dvni[0])
		+ dpi[0] )*denom
		-num*(ur[0]*dsri[0] - (sl-vni)-ul[0]*(dsli[0]-dvni[0])) ) / (denom*denom);
	dsmj[0]= ( (vnj*(sr-vnj)+ur[0]*dvnj[0]*(sr-vnj)+ur[0]*vnj*(dsrj[0]-dvnj[0]) -ul[0]*vni*dslj[0]
		- dpj[0])*denom
		-num*((sr-vnj)+ur[0]*(dsrj[0]-dvnj[0]) - ul[0]*dslj[0]) ) / (denom*denom);
	for(int k = 1; k < NVARS; k++) {
		dsmi[k]= ( (ur[0]*vnj*dsri[k] - ul[0]*(dvni[k]*(sl-vni)+vni*(dsli[k]-dvni[k])) +dpi[k])
		  * denom - num *(ur[0]*dsri[k] -ul[0]*(dsli[k]-dvni[k])) ) / (denom*denom);
		dsmj[k]= ( (ur[0]*(dvnj[k]*(sr-vnj)+vnj*(dsrj[k]-dvnj[k])) -ul[0]*vni*dslj[k] -dpj[k])
			* denom - num * (ur[0]*(dsrj[k]-dvnj[k]) - ul[0]*dslj[k]) ) / (denom*denom);
	}

	if(sl > 0) {
		P.jacDirFlux(ul,n,dfdl);
		for(int k = 0; k < NVARS*NVARS; k++) dfdr[k] = 0;
	}
	else if(sl <= 0 && sm > 0) {
		P.jacDirFlux(ul,n,dfdl);
		for(int k = 0; k < NVARS*NVARS; k++) dfdr[k] = 0;
		R us[NVARS], dusi[NVARS][NVARS], dusj[NVARS][NVARS];
		starStateJac(ul,n,vni,pi,sl,sm,dvni,dpi,dsli,dsmi,dslj,dsmj, us,dusi,dusj);
		for(int iv = 0; iv < NVARS; iv++)
			for(int k = 0; k < NVARS; k++) {
				dfdl[iv*NVARS+k] += dsli[k]*(us[iv]-ul[iv]) + sl*(dusi[iv][k] - (iv==k ? 1.0 : 0.0));
				dfdr[iv*NVARS+k] += dslj[k]*(us[iv]-ul[iv]) + sl*dusj[iv][k];
			}
	}
	else if(sm <= 0 && sr >= 0) {
		P.jacDirFlux(ur,n,dfdr);
		for(int k = 0; k < NVARS*NVARS; k++) dfdl[k] = 0;
		R us[NVARS], dusi[NVARS][NVARS], dusj[NVARS][NVARS];
		// reference passes (this=r, other=l) and receives (durstrj, durstri)
		starStateJac(ur,n,vnj,pj,sr,sm,dvnj,dpj,dsrj,dsmj,dsri,dsmi, us,dusj,dusi);
		for(int iv = 0; iv < NVARS; iv++)
			for(int k = 0; k < NVARS; k++) {
				dfdl[iv*NVARS+k] += dsri[k]*(us[iv]-ur[iv]) +sr*dusi[iv][k];
				dfdr[iv*NVARS+k] += dsrj[k]*(us[iv]-ur[iv]) + sr*(dusj[iv][k] - (iv==k ? 1.0:0.0));
			}
	}
	else {
		P.jacDirFlux(ur,n,dfdr);
		for(int k = 0; k < NVARS*NVARS; k++) dfdl[k] = 0;
	}
	for(int i = 0; i < NVARS*NVARS; i++) dfdl[i] *= -1.0;
}

// ------------------------------------------------------------------------------------------------
// Boundary conditions, abc.cpp:41-437 (the factory maps "adiabaticwall" to Adiabaticwall2D, :486)
// ------------------------------------------------------------------------------------------------

void BC::ghost(const Gas& P, const R* ins, const R* n, R* gs) const
{
	switch(type) {
	case BC_INOUTFLOW: {                                              // :46-81
		const R vni = dimDot(&ins[1],&n[0])/ins[0];
		const R ci = P.soundSpeedFromConserved(ins);
		const R Mni = vni/ci;
		const R pinf = P.freestreamPressure();
		if(Mni <= 0) { for(int i = 0; i < NVARS; i++) gs[i] = uinf[i]; }
		else if(Mni < 1) {
			gs[0] = ins[0];
			for(int i = 1; i < NDIM+1; i++) gs[i] = ins[i];
			gs[NDIM+1] = P.energyFromPressure(pinf, ins[0], dimDot(&ins[1],&ins[1])/(ins[0]*ins[0]));
		}
		else { for(int i = 0; i < NVARS; i++) gs[i] = ins[i]; }
		break;
	}
	case BC_SUBSONIC_INFLOW: {                                        // :145-175
		const R ptotal = vals[0], ttotal = vals[1];
		const R ci = P.soundSpeedFromConserved(ins);
		const R Rminus = dimDot(&ins[1],&n[0])/ins[0] - ci/(2*P.g - 1.0);
		const R co2 = ci*ci + (P.g-1.0)/2.0 * dimDot(&ins[1],&ins[1])/(ins[0]*ins[0]);
		const R q = std::sqrt((P.g+1)*co2/((P.g-1)*Rminus*Rminus) - (P.g-1)/2.0);
		const R cg = -Rminus*(P.g-1)/(P.g+1) * (1.0 + q);
		const R tg = ttotal*cg*cg/co2;
		const R pg = ptotal * std::pow(tg/ttotal, P.g/(P.g-1.0));
		gs[0] = P.densityFromPT(pg,tg);
		const R vgmag = std::sqrt(2.0/(P.g-1.0)*(co2 - cg*cg));
		// getComponentsCartesian (mathutils.hpp:39-59) in 2D: cosphi = 1
		R vg[NDIM];
		vg[0] = 0; vg[1] = 0;
		const R cosphi = 1.0;
		vg[0] = vgmag*cosphi*n[0];
		vg[1] = vgmag*cosphi*n[1];
		for(int i = 0; i < NDIM; i++) gs[i+1] = gs[0]*vg[i];
		gs[NDIM+1] = P.energyFromPressure(pg,gs[0],vgmag*vgmag);
		break;
	}
	case BC_FARFIELD:                                                 // :193-199
		for(int i = 0; i < NVARS; i++) gs[i] = uinf[i];
		break;
	case BC_SLIPWALL: {                                               // :219-229
		const R vni = dimDot(&ins[1],&n[0])/ins[0];
		gs[0] = ins[0];
		for(int i = 1; i < NDIM+1; i++) gs[i] = ins[i] - 2.0*vni*n[i-1]*ins[0];
		gs[NDIM+1] = ins[NDIM+1];
		break;
	}
	case BC_ADIABATIC_WALL: {                                         // Adiabaticwall2D :278-287
		const R tangvel = vals[0];
		const R tangMomentum = tangvel * ins[0];
		gs[0] = ins[0];
		gs[1] =  2.0*tangMomentum*n[1] - ins[1];
		gs[2] = -2.0*tangMomentum*n[0] - ins[2];
		gs[3] = ins[3];
		break;
	}
	case BC_ISOTHERMAL_WALL: {                                        // :349-366
		const R tangvel = vals[0], walltemperature = vals[1];
		const R p = P.pressureFromConserved(ins);
		const R gtemp = 2.0*walltemperature - P.temperature(ins[0],p);
		gs[0] = ins[0];
		gs[1] = gs[0]*( 2.0*tangvel*n[1] - ins[1]/ins[0]);
		gs[2] = gs[0]*(-2.0*tangvel*n[0] - ins[2]/ins[0]);
		const R vmag2 = dimDot(&gs[1],&gs[1])/(gs[0]*gs[0]);
		gs[3] = P.energyFromTemperature(gtemp, gs[0], vmag2);
		break;
	}
	case BC_EXTRAPOLATION:                                            // :414-420
		for(int k = 0; k < NVARS; k++) gs[k] = ins[k];
		break;
	default:
		throw std::runtime_error("BC type not implemented yet!");
	}
}

void BC::ghostJac(const Gas& P, const R* ins, const R* n, R* gs, R* dgs) const
{
	for(int k = 0; k < NVARS*NVARS; k++) dgs[k] = 0;
	switch(type) {
	case BC_INOUTFLOW: {                                              // :83-133
		const R vni = dimDot(&ins[1],&n[0])/ins[0];
		const R ci = P.soundSpeedFromConserved(ins);
		const R Mni = vni/ci;
		const R pinf = P.pressureFromConserved(&uinf[0]);
		if(Mni <= 0) { for(int i = 0; i < NVARS; i++) gs[i] = uinf[i]; }
		else if(Mni <= 1) {
			gs[0] = ins[0]; gs[1] = ins[1]; gs[2] = ins[2];
			for(int k = 0; k < NVARS-1; k++) dgs[k*NVARS+k] = 1.0;
			gs[NDIM+1] = P.energyFromPressure(pinf, ins[0], dimDot(&ins[1],&ins[1])/(ins[0]*ins[0]));
			dgs[(NDIM+1)*NVARS+0] = -0.5*dimDot(&ins[1],&ins[1])/(ins[0]*ins[0]);
			for(int j = 1; j < NDIM+1; j++) dgs[(NDIM+1)*NVARS+j] = ins[j]/ins[0];
			dgs[(NDIM+1)*NVARS+NDIM+1] = 0;
		}
		else { for(int i = 0; i < NVARS; i++) { gs[i] = ins[i]; dgs[i*NVARS+i] = 1.0; } }
		break;
	}
	case BC_FARFIELD:                                                 // :201-210
		for(int i = 0; i < NVARS; i++) gs[i] = uinf[i];
		break;
	case BC_SLIPWALL: {                                               // :231-261
		const R vni = dimDot(&ins[1],n)/ins[0];
		R dvni[NVARS];
		dvni[0] = -vni/ins[0];
		for(int i = 1; i < NDIM+1; i++) dvni[i] = n[i-1]/ins[0];
		dvni[NDIM+1] = 0;
		gs[0] = ins[0]; dgs[0] = 1.0;
		for(int i = 1; i < NDIM+1; i++) {
			gs[i] = ins[i] - 2.0*n[i-1]*vni*ins[0];
			dgs[i*NVARS] = -2.0*n[i-1]*(dvni[0]*ins[0] + vni);
			for(int j = 1; j < NDIM+1; j++) {
				if(i==j) dgs[i*NVARS+j] = 1.0 - 2.0*n[i-1]*dvni[i]*ins[0];
				else     dgs[i*NVARS+j] = -2.0*n[i-1]*dvni[j]*ins[0];
			}
		}
		gs[NDIM+1] = ins[NDIM+1];
		dgs[(NDIM+1)*NVARS+NDIM+1] = 1.0;
		break;
	}
	case BC_ADIABATIC_WALL: {                                         // :289-310
		const R tangvel = vals[0];
		const R tangMomentum = tangvel * ins[0];
		gs[0] = ins[0]; dgs[0] = 1.0;
		gs[1] =  2.0*tangMomentum*n[1] - ins[1];
		dgs[NVARS+0] = 2.0*tangvel*n[1]; dgs[NVARS+1] = -1.0;
		gs[2] = -2.0*tangMomentum*n[0] - ins[2];
		dgs[2*NVARS+0] = -2.0*tangvel*n[0]; dgs[2*NVARS+2] = -1.0;
		gs[3] = ins[3]; dgs[3*NVARS+3] = 1.0;
		break;
	}
	case BC_ISOTHERMAL_WALL: {                                        // :368-404 (FIXME upstream)
		const R tangvel = vals[0], walltemperature = vals[1];
		const R tangMomentum = tangvel * ins[0];
		gs[0] = ins[0]; dgs[0] = 1.0;
		gs[1] =  2.0*tangMomentum*n[1] - ins[1];
		dgs[NVARS+0] = 2.0*tangvel*n[1]; dgs[NVARS+1] = -1.0;
		gs[2] = -2.0*tangMomentum*n[0] - ins[2];
		dgs[2*NVARS+0] = -2.0*tangvel*n[0]; dgs[2*NVARS+2] = -1.0;
		const R vmag2 = dimDot(&gs[1],&gs[1])/(ins[0]*ins[0]);
		gs[3] = P.energyFromTemperature(walltemperature, ins[0], vmag2);
		R dvmag2[NVARS];
		dvmag2[0] = -2.0*dimDot(&gs[1],&gs[1])/(ins[0]*ins[0]*ins[0]);
		for(int i = 1; i < NDIM+1; i++) dvmag2[i] = 1.0/(ins[0]*ins[0]) * gs[i] * (-1.0);
		dvmag2[NDIM+1] = 0;
		R dT[NVARS] = {0,0,0,0};
		P.jacEnergyFromJacTV(walltemperature, ins[0], vmag2, dT, dvmag2, &dgs[3*NVARS]);
		break;
	}
	case BC_EXTRAPOLATION:                                            // :422-433
		for(int k = 0; k < NVARS; k++) { gs[k] = ins[k]; dgs[k*NVARS+k] = 1.0; }
		break;
	default:
		throw std::runtime_error("BC has no Jacobian in the reference (abc.cpp:178-185)");
	}
}

}
