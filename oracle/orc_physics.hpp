/** \file orc_physics.hpp
 * \brief ORACLE (test infrastructure only; never linked into the product): CPU restatement of
 *   FVENS's point-wise gas dynamics — ideal-gas physics, numerical inviscid fluxes and their
 *   Jacobians, and boundary-condition ghost states — in the reference's operation order.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this.
 * Parity status: pinned by the reference's own known-answer tests (wall-BC zero flux,
 * testwallbcs.cpp:9-66) and by consistency checks in tests/; the reference itself is
 * unbuildable here (needs Eigen/PETSc/Boost, absent from the image).
 *
 * Source lines restated (all under /root/reference/src):
 *   physics/aphysics_defs.hpp:13-487, physics/aphysics.cpp:16-215,
 *   spatial/anumericalflux.hpp:175-189, spatial/anumericalflux.cpp:40-1397,
 *   spatial/abc.cpp:41-437, physics/viscousphysics.cpp:14-246, mathutils.hpp:17-90.
 * Arithmetic is IEEE double with no contraction (built with -ffp-contract=off), matching the
 * reference's -O3 -msse4.2 Release build (CMakeLists.txt:52,206), which has no FMA.
 */
#ifndef ORC_PHYSICS_HPP
#define ORC_PHYSICS_HPP

#include <cmath>
#include <array>
#include <stdexcept>

namespace orc {

constexpr int NDIM = 2;
constexpr int NVARS = 4;
typedef double R;

/// mathutils.hpp:24-31
inline R dimDot(const R* u, const R* v) { R d = 0; for(int i = 0; i < NDIM; i++) d += u[i]*v[i]; return d; }

/// IdealGasPhysics (aphysics.hpp:48-336); constants as in the constructor aphysics.cpp:17-20
struct Gas
{
	R g, Minf, Tinf, Reinf, Pr, sC;
	Gas(R _g, R M, R T, R Re, R P) : g(_g), Minf(M), Tinf(T), Reinf(Re), Pr(P), sC(110.5) {}

	// aphysics_defs.hpp:13-23
	void dirFlux(const R* uc, const R* n, R vn, R p, R* flux) const {
		flux[0] = vn*uc[0];
		for(int i = 1; i < NDIM+1; i++) flux[i] = vn*uc[i] + p*n[i-1];
		flux[NDIM+1] = vn*(uc[NDIM+1] + p);
	}
	// :25-38
	void varsFromConserved(const R* uc, const R* n, R* v, R& vn, R& p, R& H) const {
		for(int j = 0; j < NDIM; j++) v[j] = uc[j+1]/uc[0];
		vn = dimDot(v,n);
		const R vmag2 = dimDot(v,v);
		p = (g-1.0)*(uc[3] - 0.5*uc[0]*vmag2);
		H = (uc[3]+p)/uc[0];
	}
	R pressure(R ie) const { return (g-1.0)*ie; }                                  // :51-55
	R pressureFromConserved(const R* uc) const {                                    // :58-63
		return pressure(uc[NDIM+1] - 0.5*dimDot(&uc[1],&uc[1])/uc[0]);
	}
	void jacPressure(const R* uc, R* dp) const {                                    // :93-102
		dp[0] = (g-1.0)*0.5*dimDot(&uc[1],&uc[1])/(uc[0]*uc[0]);
		for(int i = 1; i < NDIM+1; i++) dp[i] = -(g-1.0)*uc[i]/uc[0];
		dp[NDIM+1] = (g-1.0);
	}
	void jacPressure(const R* uc, R rho2vmag2, R* dp) const {                       // :104-114
		dp[0] = (g-1.0)*0.5*rho2vmag2/(uc[0]*uc[0]);
		for(int i = 1; i < NDIM+1; i++) dp[i] = -(g-1.0)*uc[i]/uc[0];
		dp[NDIM+1] = (g-1.0);
	}
	R temperature(R rho, R p) const { return p/rho * g*Minf*Minf; }               // :117-122
	void jacTemperature(R rho, R p, const R* dp, R* dT) const {                     // :125-135
		const R coef = g*Minf*Minf;
		dT[0] += coef*(dp[0]*rho - p)/(rho*rho);
		for(int i = 1; i < NVARS; i++) dT[i] += coef/rho * dp[i];
	}
	R soundSpeed(R rho, R p) const { return std::sqrt(g * p/rho); }               // :138-143
	void jacSoundSpeed(R rho, R p, const R* dp, R c, R* dc) const {                 // :145-154
		dc[0] += 0.5/c * g* (dp[0]*rho-p)/(rho*rho);
		for(int i = 1; i < NVARS; i++) dc[i] += 0.5/c * g*dp[i]/rho;
	}
	R soundSpeedFromConserved(const R* uc) const { return soundSpeed(uc[0],pressureFromConserved(uc)); }
	R energyFromPressure(R p, R d, R vmag2) const { return p/(g-1.0) + 0.5*d*vmag2; }   // :209-215
	R energyFromTemperature(R T, R d, R vmag2) const {                              // :217-223
		return d * (T/(g*(g-1.0)*Minf*Minf) + 0.5*vmag2);
	}
	void jacEnergyFromJacTV(R T, R d, R vmag2, const R* dT, const R* dvmag2, R* de) const { // :225-236
		const R coeff = 1.0/(g*(g-1.0)*Minf*Minf);
		de[0] += coeff * (T+d*dT[0]) + 0.5 * (vmag2+d*dvmag2[0]);
		for(int i = 1; i < NVARS; i++) de[i] += d * (coeff*dT[i] + 0.5*dvmag2[i]);
	}
	R energyFromPrimitive(const R* up) const {                                      // :239-244
		return energyFromPressure(up[NVARS-1], up[0], dimDot(&up[1],&up[1]));
	}
	void primFromCons(const R* uc, R* up) const {                                   // :257-267
		up[0] = uc[0];
		const R p = pressureFromConserved(uc);
		for(int i = 1; i < NDIM+1; i++) up[i] = uc[i]/uc[0];
		up[NDIM+1] = p;
	}
	void prim2FromCons(const R* uc, R* up) const {                                  // :271-281
		up[0] = uc[0];
		const R p = pressureFromConserved(uc);
		for(int i = 1; i < NDIM+1; i++) up[i] = uc[i]/uc[0];
		up[NVARS-1] = temperature(uc[0],p);
	}
	void consFromPrim(const R* up, R* uc) const {                                   // :285-295
		uc[0] = up[0];
		const R rhoE = energyFromPrimitive(up);
		for(int i = 1; i < NDIM+1; i++) uc[i] = up[0]*up[i];
		uc[NDIM+1] = rhoE;
	}
	R densityFromPT(R p, R T) const { return g*Minf*Minf*p/T; }                     // :297-303
	R temperatureFromConserved(const R* uc) const { return temperature(uc[0], pressureFromConserved(uc)); }
	void jacTemperatureWrtConserved(const R* uc, R* dT) const {                     // :326-337
		const R p = pressureFromConserved(uc);
		R dp[NVARS] = {0,0,0,0};
		jacPressure(uc,dp);
		jacTemperature(uc[0],p,dp,dT);
	}
	R gradTemperature(R rho, R gradrho, R p, R gradp) const {                        // :347-353
		return (gradp*rho - p*gradrho) / (rho*rho) * g*Minf*Minf;
	}
	R viscFromT(R T) const {                                                         // :408-413
		return (1.0+sC/Tinf)/(T+sC/Tinf) * std::pow(T,1.5) / Reinf;
	}
	R viscFromConserved(const R* uc) const { return viscFromT(temperatureFromConserved(uc)); }
	void jacSutherland(const R* uc, R* dmu) const {                                  // :423-439
		const R T = temperatureFromConserved(uc);
		R dT[NVARS] = {0,0,0,0};
		jacTemperatureWrtConserved(uc, dT);
		const R coef = (1.0+sC/Tinf)/Reinf;
		const R T15 = std::pow(T,1.5), Tm15 = std::pow(T,-1.5);
		const R denom = (T + sC/Tinf)*(T+sC/Tinf);
		for(int i = 0; i < NVARS; i++)
			dmu[i] += coef* (1.5*Tm15*dT[i]*(T+sC/Tinf) - T15*dT[i])/denom;
	}
	R constVisc() const { return 1.0/Reinf; }                                        // :441-445
	R thermCond(R muhat) const { return muhat / (Minf*Minf*(g-1.0)*Pr); }          // :447-451
	void jacThermCond(const R* dmuhat, R* dkhat) const {                             // :453-461
		for(int k = 0; k < NVARS; k++) dkhat[k] = dmuhat[k]/(Minf*Minf*(g-1.0)*Pr);
	}
	R freestreamPressure() const { return (1.0/(g*Minf*Minf)); }                   // :463-467
	void stressTensor(R mu, const R grad[NDIM][NVARS], R stress[NDIM][NDIM]) const { // :469-487
		R ldiv = 0;
		for(int j = 0; j < NDIM; j++) ldiv += grad[j][j+1];
		ldiv *= 2.0/3.0*mu;
		for(int i = 0; i < NDIM; i++) {
			for(int j = 0; j < NDIM; j++) stress[i][j] = mu*(grad[i][j+1] + grad[j][i+1]);
			stress[i][i] -= ldiv;
		}
	}
	// aphysics.cpp:28-35
	void dirFluxFromConserved(const R* u, const R* n, R* flux) const {
		const R vn = dimDot(&u[1],n)/u[0];
		const R p = pressure(u[NDIM+1] - 0.5*dimDot(&u[1],&u[1])/u[0]);
		dirFlux(u, n, vn, p, flux);
	}
	// aphysics.cpp:43-58 (angle-of-attack free stream, sideslip 0; mathutils.hpp:66-75)
	std::array<R,NVARS> freestream(R aoa) const {
		std::array<R,NVARS> u;
		const R beta = 0;
		u[0] = 1.0;
		u[1] = std::cos(aoa)*std::cos(beta);
		u[2] = std::sin(aoa)*std::cos(beta);
		u[3] = energyFromPressure(freestreamPressure(),1.0,1.0);
		return u;
	}
	// aphysics.cpp:60-127
	void jacDirFlux(const R* u, const R* n, R* dfdu) const {
		dfdu[0] = 0;
		for(int i = 1; i < NDIM+1; i++) dfdu[i] = n[i-1];
		dfdu[NDIM+1] = 0;
		const R p = pressureFromConserved(u);
		R dp[NVARS];
		jacPressure(u, dp);
		const R vn = dimDot(&u[1],n)/u[0];
		R dvn[NVARS];
		dvn[0] = -vn/u[0];
		for(int i = 1; i < NDIM+1; i++) dvn[i] = n[i-1]/u[0];
		dvn[NDIM+1] = 0;
		for(int i = 1; i < NDIM+1; i++) {
			dfdu[i*NVARS] = -vn*u[i]/u[0] + dp[0]*n[i-1];
			for(int j = 1; j < NDIM+1; j++) {
				if(i == j) dfdu[i*NVARS+j] = dvn[j]*u[i] + vn + dp[j]*n[i-1];
				else       dfdu[i*NVARS+j] = dvn[j]*u[i] + dp[j]*n[i-1];
			}
			dfdu[i*NVARS+NDIM+1] = dp[NDIM+1]*n[i-1];
		}
		dfdu[(NDIM+1)*NVARS] = -vn/u[0]*(u[NDIM+1]+p) + vn*dp[0];
		for(int j = 1; j < NDIM+1; j++) dfdu[(NDIM+1)*NVARS+j] = n[j-1]/u[0]*(u[NDIM+1]+p) + vn*dp[j];
		dfdu[(NDIM+1)*NVARS+NDIM+1] = vn*(1.0 + dp[NDIM+1]);
	}
	// aphysics.cpp:129-153 (outputs are added to)
	void jacVars(const R* uc, const R* n, R* dv, R* dvn, R* dp, R* dH) const {
		for(int j = 0; j < NDIM; j++) {
			dv[j*NVARS+0] += -uc[j+1]/(uc[0]*uc[0]);
			dv[j*NVARS+j+1] += 1.0/uc[0];
		}
		for(int j = 0; j < NDIM; j++) {
			dvn[0] += dv[j*NVARS]*n[j];
			dvn[j+1] += n[j]/uc[0];
		}
		const R p = pressureFromConserved(uc);
		jacPressure(uc, dp);
		dH[0] += (dp[0]*uc[0] - (uc[NDIM+1]+p))/(uc[0]*uc[0]);
		for(int j = 1; j < NDIM+1; j++) dH[j] += dp[j]/uc[0];
		dH[3] += (1.0+dp[NDIM+1])/uc[0];
	}
	// aphysics.cpp:155-175 (added to)
	void jacPrim2(const R* uc, R* jac) const {
		jac[0] += 1.0;
		const R rho2vmag2 = dimDot(&uc[1],&uc[1]);
		for(int i = 1; i < NDIM+1; i++) {
			jac[i*NVARS+0] += -uc[i]/(uc[0]*uc[0]);
			jac[i*NVARS+i] += 1.0/uc[0];
		}
		const R p = pressure(uc[NDIM+1] - 0.5*rho2vmag2/uc[0]);
		R dp[NVARS] = {0,0,0,0};
		jacPressure(uc, rho2vmag2, dp);
		jacTemperature(uc[0], p, dp, &jac[(NDIM+1)*NVARS]);
	}
	// aphysics.cpp:177-215
	void jacStress(R mu, const R* dmu, const R grad[NDIM][NVARS], const R dgrad[NDIM][NVARS][NVARS],
	               R stress[NDIM][NDIM], R dstress[NDIM][NDIM][NVARS]) const {
		R div = 0; R dldiv[NVARS] = {0,0,0,0};
		for(int j = 0; j < NDIM; j++) {
			div += grad[j][j+1];
			for(int k = 0; k < NVARS; k++) dldiv[k] += dgrad[j][j+1][k];
		}
		const R ldiv = 2.0/3.0*mu*div;
		for(int k = 0; k < NVARS; k++) dldiv[k] = 2.0/3.0 * (dmu[k]*div + mu*dldiv[k]);
		for(int i = 0; i < NDIM; i++) {
			for(int j = 0; j < NDIM; j++) {
				stress[i][j] = mu*(grad[i][j+1] + grad[j][i+1]);
				for(int k = 0; k < NVARS; k++)
					dstress[i][j][k] = dmu[k]*(grad[i][j+1] + grad[j][i+1]) + mu*(dgrad[i][j+1][k] + dgrad[j][i+1][k]);
			}
			stress[i][i] -= ldiv;
			for(int k = 0; k < NVARS; k++) dstress[i][i][k] -= dldiv[k];
		}
	}
};

enum FluxType { LLF = 0, VANLEER = 1, AUSM = 2, AUSMPLUS = 3, ROE = 4, HLL = 5, HLLC = 6 };

/// Numerical inviscid fluxes (anumericalflux.cpp). dfdl = -dF/dul, dfdr = +dF/dur (hpp:36-45).
struct Flux
{
	const Gas& P;
	int type;
	R g;
	Flux(const Gas& p, int t) : P(p), type(t), g(p.g) {}

	void roeAverages(const R* ul, const R* ur, const R* n, const R* vi, R Hi, const R* vj, R Hj,
	                 R& Rij, R& rhoij, R* vij, R& vm2ij, R& vnij, R& Hij, R& cij) const {  // hpp:175-189
		Rij = std::sqrt(ur[0]/ul[0]);
		rhoij = Rij*ul[0];
		for(int i = 0; i < NDIM; i++) vij[i] = (Rij*vj[i] + vi[i])/(Rij + 1.0);
		Hij = (Rij*Hj + Hi)/(Rij + 1.0);
		vm2ij = dimDot(vij,vij);
		vnij = dimDot(vij,n);
		cij = std::sqrt( (g-1.0)*(Hij - vm2ij*0.5) );
	}

	void flux(const R* ul, const R* ur, const R* n, R* f) const {
		switch(type) {
			case LLF: llf(ul,ur,n,f); break;
			case VANLEER: vanleer(ul,ur,n,f); break;
			case AUSM: ausm(ul,ur,n,f); break;
			case AUSMPLUS: ausmplus(ul,ur,n,f); break;
			case ROE: roe(ul,ur,n,f); break;
			case HLL: hll(ul,ur,n,f); break;
			case HLLC: hllc(ul,ur,n,f); break;
			default: throw std::invalid_argument("unknown flux");
		}
	}
	void jacobian(const R* ul, const R* ur, const R* n, R* dfdl, R* dfdr) const {
		switch(type) {
			case LLF: llf_jac(ul,ur,n,dfdl,dfdr); break;
			case AUSM: ausm_jac(ul,ur,n,dfdl,dfdr); break;
			case ROE: roe_jac(ul,ur,n,dfdl,dfdr); break;
			case HLL: hll_jac(ul,ur,n,dfdl,dfdr); break;
			case HLLC: hllc_jac(ul,ur,n,dfdl,dfdr); break;
			default: throw std::invalid_argument("flux has no Jacobian in the reference");
		}
	}

	// :40-61
	void llf(const R* ul, const R* ur, const R* n, R* flux) const {
		R vi[NDIM], vj[NDIM], vni, vnj, pi, pj, Hi, Hj, ci, cj;
		P.varsFromConserved(ul, n, vi, vni, pi, Hi);
		P.varsFromConserved(ur, n, vj, vnj, pj, Hj);
		ci = P.soundSpeed(ul[0],pi);
		cj = P.soundSpeed(ur[0],pj);
		const R eig = std::fabs(vni)+ci > std::fabs(vnj)+cj ? std::fabs(vni)+ci : std::fabs(vnj)+cj;
		P.dirFluxFromConserved(ul,n,flux);
		R fluxr[NVARS];
		P.dirFluxFromConserved(ur,n,fluxr);
		for(int i = 0; i < NVARS; i++) flux[i] = 0.5*( flux[i] + fluxr[i] - eig*(ur[i]-ul[i]) );
	}
	// :65-107 (frozen spectral radius)
	void llf_jac(const R* ul, const R* ur, const R* n, R* dfdl, R* dfdr) const {
		R vi[NDIM], vj[NDIM], vni, vnj, pi, pj, Hi, Hj, ci, cj, eig;
		P.varsFromConserved(ul, n, vi, vni, pi, Hi);
		P.varsFromConserved(ur, n, vj, vnj, pj, Hj);
		ci = P.soundSpeed(ul[0],pi);
		cj = P.soundSpeed(ur[0],pj);
		if(std::fabs(vni)+ci >= std::fabs(vnj)+cj) eig = std::fabs(vni)+ci;
		else eig = std::fabs(vnj)+cj;
		P.jacDirFlux(ul, n, dfdl);
		P.jacDirFlux(ur, n, dfdr);
		for(int i = 0; i < NVARS; i++) dfdl[i*NVARS+i] -= -eig;
		for(int i = 0; i < NVARS; i++) dfdr[i*NVARS+i] -= eig;
		for(int i = 0; i < NVARS; i++)
			for(int j = 0; j < NVARS; j++) {
				dfdl[i*NVARS+j] = -0.5*dfdl[i*NVARS+j];
				dfdr[i*NVARS+j] =  0.5*dfdr[i*NVARS+j];
			}
	}
	// :202-250
	void vanleer(const R* ul, const R* ur, const R* n, R* flux) const {
		R fiplus[NVARS], fjminus[NVARS];
		R vi[NDIM], vj[NDIM], vni, vnj, pi, pj, Hi, Hj, ci, cj;
		P.varsFromConserved(ul, n, vi, vni, pi, Hi);
		P.varsFromConserved(ur, n, vj, vnj, pj, Hj);
		ci = P.soundSpeed(ul[0],pi);
		cj = P.soundSpeed(ur[0],pj);
		const R Mni = vni/ci, Mnj = vnj/cj;
		if(Mni < -1.0) for(int i = 0; i < NVARS; i++) fiplus[i] = 0;
		else if(Mni > 1.0) P.dirFlux(ul,n,vni,pi,fiplus);
		else {
			const R vmags = std::pow(ul[1]/ul[0], 2) + std::pow(ul[2]/ul[0], 2);
			fiplus[0] = ul[0]*ci*std::pow(Mni+1, 2)/4.0;
			fiplus[1] = fiplus[0] * (ul[1]/ul[0] + n[0]*(2.0*ci - vni)/g);
			fiplus[2] = fiplus[0] * (ul[2]/ul[0] + n[1]*(2.0*ci - vni)/g);
			fiplus[3] = fiplus[0] * ( (vmags - vni*vni)/2.0 + std::pow((g-1)*vni+2*ci, 2)/(2*(g*g-1)) );
		}
		if(Mnj > 1.0) for(int i = 0; i < NVARS; i++) fjminus[i] = 0;
		else if(Mnj < -1.0) P.dirFlux(ur,n,vnj,pj,fjminus);
		else {
			const R vmags = std::pow(ur[1]/ur[0], 2) + std::pow(ur[2]/ur[0], 2);
			fjminus[0] = -ur[0]*cj*std::pow(Mnj-1, 2)/4.0;
			fjminus[1] = fjminus[0] * (ur[1]/ur[0] + n[0]*(-2.0*cj - vnj)/g);
			fjminus[2] = fjminus[0] * (ur[2]/ur[0] + n[1]*(-2.0*cj - vnj)/g);
			fjminus[3] = fjminus[0] * ( (vmags - vnj*vnj)/2.0 + std::pow((g-1)*vnj-2*cj, 2)/(2*(g*g-1)) );
		}
		for(int i = 0; i < NVARS; i++) flux[i] = fiplus[i] + fjminus[i];
	}
	// :264-315
	void ausm(const R* ul, const R* ur, const R* n, R* flux) const {
		R ML, MR, pL, pR;
		R vi[NDIM], vj[NDIM], vni, vnj, pi, pj, Hi, Hj;
		P.varsFromConserved(ul, n, vi, vni, pi, Hi);
		P.varsFromConserved(ur, n, vj, vnj, pj, Hj);
		const R ci = P.soundSpeed(ul[0],pi);
		const R cj = P.soundSpeed(ur[0],pj);
		const R Mni = vni/ci, Mnj = vnj/cj;
		if(std::fabs(Mni) <= 1.0) { ML = 0.25*(Mni+1)*(Mni+1); pL = ML*pi*(2.0-Mni); }
		else if(Mni < -1.0) { ML = 0; pL = 0; }
		else { ML = Mni; pL = pi; }
		if(std::fabs(Mnj) <= 1.0) { MR = -0.25*(Mnj-1)*(Mnj-1); pR = -MR*pj*(2.0+Mnj); }
		else if(Mnj < -1.0) { MR = Mnj; pR = pj; }
		else { MR = 0; pR = 0; }
		const R Mhalf = ML+MR;
		const R phalf = pL+pR;
		flux[0] = Mhalf/2.0*(ul[0]*ci+ur[0]*cj) -std::fabs(Mhalf)/2.0*(ur[0]*cj-ul[0]*ci);
		for(int j = 1; j < NDIM+1; j++)
			flux[j] = Mhalf/2.0*(ul[j]*ci+ur[j]*cj) -std::fabs(Mhalf)/2.0*(ur[j]*cj-ul[j]*ci) + phalf*n[j-1];
		flux[3] = Mhalf/2.0*(ci*(ul[3]+pi)+cj*(ur[3]+pj))
			-std::fabs(Mhalf)/2.0*(cj*(ur[3]+pj)-ci*(ul[3]+pi));
	}
	// :317-472
	void ausm_jac(const R* ul, const R* ur, const R* n, R* dfdl, R* dfdr) const;
	// :479-553
	void ausmplus(const R* ul, const R* ur, const R* n, R* flux) const {
		R ML, MR, pL, pR;
		R vi[NDIM], vj[NDIM], vni, vnj, pi, pj, Hi, Hj;
		P.varsFromConserved(ul, n, vi, vni, pi, Hi);
		P.varsFromConserved(ur, n, vj, vnj, pj, Hj);
		const R ci = P.soundSpeed(ul[0],pi);
		const R cj = P.soundSpeed(ur[0],pj);
		const R vmag2i = dimDot(vi,vi);
		const R vmag2j = dimDot(vj,vj);
		R csi = std::sqrt((ci*ci/(g-1.0)+0.5*vmag2i)*2.0*(g-1.0)/(g+1.0));
		R csj = std::sqrt((cj*cj/(g-1.0)+0.5*vmag2j)*2.0*(g-1.0)/(g+1.0));
		R corri, corrj;
		if(csi > vni) corri = csi; else corri = vni;
		if(csj > -vnj) corrj = csj; else corrj = -vnj;
		csi = csi*csi/corri;
		csj = csj*csj/corrj;
		const R chalf = (csi < csj) ? csi : csj;
		const R Mni = vni/chalf, Mnj = vnj/chalf;
		if(std::fabs(Mni) <= 1.0) {
			ML = 0.25*(Mni+1)*(Mni+1) + 1.0/8.0*(Mni*Mni-1.0)*(Mni*Mni-1.0);
			pL = pi*(0.25*(Mni+1)*(Mni+1)*(2.0-Mni) + 3.0/16*Mni*(Mni*Mni-1.0)*(Mni*Mni-1.0));
		}
		else if(Mni < -1.0) { ML = 0; pL = 0; }
		else { ML = Mni; pL = pi; }
		if(std::fabs(Mnj) <= 1.0) {
			MR = -0.25*(Mnj-1)*(Mnj-1) - 1.0/8.0*(Mnj*Mnj-1.0)*(Mnj*Mnj-1.0);
			pR = pj*(0.25*(Mnj-1)*(Mnj-1)*(2.0+Mnj) - 3.0/16*Mnj*(Mnj*Mnj-1.0)*(Mnj*Mnj-1.0));
		}
		else if(Mnj < -1.0) { MR = Mnj; pR = pj; }
		else { MR = 0; pR = 0; }
		const R Mhalf = ML+MR;
		const R phalf = pL+pR;
		flux[0] = chalf* (Mhalf/2.0*(ul[0]+ur[0]) -std::fabs(Mhalf)/2.0*(ur[0]-ul[0]));
		for(int j = 1; j < NDIM+1; j++)
			flux[j] = chalf* (Mhalf/2.0*(ul[j]+ur[j]) -std::fabs(Mhalf)/2.0*(ur[j]-ul[j])) + phalf*n[j-1];
		flux[3] = chalf* (Mhalf/2.0*(ul[3]+pi+ur[3]+pj) -std::fabs(Mhalf)/2.0*((ur[3]+pj)-(ul[3]+pi)));
	}
	// :667-732
	void roe(const R* ul, const R* ur, const R* n, R* flux) const {
		R vi[NDIM], vj[NDIM], vni, vnj, pi, pj, Hi, Hj;
		P.varsFromConserved(ul, n, vi, vni, pi, Hi);
		P.varsFromConserved(ur, n, vj, vnj, pj, Hj);
		R Rij,rhoij,vij[NDIM],vm2ij,vnij,Hij,cij;
		roeAverages(ul,ur,n,vi,Hi,vj,Hj, Rij,rhoij,vij,vm2ij,vnij,Hij,cij);
		const R fixeps = 1.0e-4;
		R l[NVARS];
		l[0] = std::fabs(vnij-cij);
		for(int j = 1; j < NDIM+1; j++) l[j] = std::fabs(vnij);
		l[NDIM+1] = std::fabs(vnij+cij);
		const R delta = fixeps*cij;
		for(int iv = 0; iv < NVARS; iv++)
			if(l[iv] < delta) l[iv] = (l[iv]*l[iv] + delta*delta)/(2.0*delta);
		const R devn = vnj-vni, dep = pj-pi, derho = ur[0]-ul[0];
		R adu[NVARS], la[NVARS];
		la[0] = l[0]*(dep-rhoij*cij*devn)/(2.0*cij*cij);
		la[1] = l[1]*(derho - dep/(cij*cij));
		la[2] = l[1]*rhoij;
		la[3] = l[3]*(dep+rhoij*cij*devn)/(2.0*cij*cij);
		adu[0] = la[0];
		adu[1] = la[0]*(vij[0]-cij*n[0]);
		adu[2] = la[0]*(vij[1]-cij*n[1]);
		adu[3] = la[0]*(Hij-cij*vnij);
		adu[0] += la[1];
		adu[1] += la[1]*vij[0] +      la[2]*(vj[0]-vi[0] - devn*n[0]);
		adu[2] += la[1]*vij[1] +      la[2]*(vj[1]-vi[1] - devn*n[1]);
		adu[3] += la[1]*vm2ij/2.0 + la[2] *(vij[0]*(vj[0]-vi[0]) +vij[1]*(vj[1]-vi[1]) -vnij*devn);
		adu[0] += la[3];
		adu[1] += la[3]*(vij[0]+cij*n[0]);
		adu[2] += la[3]*(vij[1]+cij*n[1]);
		adu[3] += la[3]*(Hij+cij*vnij);
		R fi[NVARS], fj[NVARS];
		P.dirFlux(ul,n,vni,pi,fi);
		P.dirFlux(ur,n,vnj,pj,fj);
		for(int iv = 0; iv < NVARS; iv++) flux[iv] = 0.5*(fi[iv]+fj[iv] - adu[iv]);
	}
	void roeAvgJac(const R* ul, const R* ur, const R* n, R vxi, R vyi, R Hi, R vxj, R vyj, R Hj,
	               const R* dvxi, const R* dvyi, const R* dHi, const R* dvxj, const R* dvyj, const R* dHj,
	               R* dRiji, R* drhoiji, R* dvxiji, R* dvyiji, R* dvm2iji, R* dvniji, R* dHiji, R* dciji,
	               R* dRijj, R* drhoijj, R* dvxijj, R* dvyijj, R* dvm2ijj, R* dvnijj, R* dHijj, R* dcijj) const;
	void roe_jac(const R* ul, const R* ur, const R* n, R* dfdl, R* dfdr) const;
	// :973-1007
	void hll(const R* ul, const R* ur, const R* n, R* flux) const {
		R vi[NDIM], vj[NDIM], vni, vnj, pi, pj, Hi, Hj, ci, cj;
		P.varsFromConserved(ul, n, vi, vni, pi, Hi);
		P.varsFromConserved(ur, n, vj, vnj, pj, Hj);
		ci = P.soundSpeed(ul[0], pi);
		cj = P.soundSpeed(ur[0], pj);
		R Rij,rhoij,vm2ij,vnij,Hij,cij,vij[NDIM];
		roeAverages(ul,ur,n,vi,Hi,vj,Hj, Rij,rhoij,vij,vm2ij,vnij,Hij,cij);
		R sl = vni - ci;
		if (sl > vnij-cij) sl = vnij-cij;
		R sr = vnj+cj;
		if(sr < vnij+cij) sr = vnij+cij;
		const R sr0 = sr > 0 ? 0 : sr;
		const R sl0 = sl > 0 ? 0 : sl;
		const R t1 = (sr0 - sl0)/(sr-sl); const R t2 = 1.0 - t1;
		const R t3 = 0.5*(sr*std::fabs(sl)-sl*std::fabs(sr))/(sr-sl);
		flux[0] = t1*vnj*ur[0] + t2*vni*ul[0]                     - t3*(ur[0]-ul[0]);
		flux[1] = t1*(vnj*ur[1]+pj*n[0]) + t2*(vni*ul[1]+pi*n[0]) - t3*(ur[1]-ul[1]);
		flux[2] = t1*(vnj*ur[2]+pj*n[1]) + t2*(vni*ul[2]+pi*n[1]) - t3*(ur[2]-ul[2]);
		flux[3] = t1*(vnj*ur[0]*Hj) + t2*(vni*ul[0]*Hi)           - t3*(ur[3]-ul[3]);
	}
	void hll_jac(const R* ul, const R* ur, const R* n, R* dfdl, R* dfdr) const;
	// :1069-1081
	void starState(const R* u, const R* n, R vn, R p, R ss, R sm, R* ustr) const {
		const R pstar = u[0]*(vn-ss)*(vn-sm) + p;
		ustr[0] = u[0] * (ss - vn)/(ss-sm);
		ustr[1] = ( (ss-vn)*u[1] + (pstar-p)*n[0] )/(ss-sm);
		ustr[2] = ( (ss-vn)*u[2] + (pstar-p)*n[1] )/(ss-sm);
		ustr[3] = ( (ss-vn)*u[3] - p*vn + pstar*sm )/(ss-sm);
	}
	// :1173-1228
	void hllc(const R* ul, const R* ur, const R* n, R* flux) const {
		R vi[NDIM], vj[NDIM], vni, vnj, pi, pj, Hi, Hj, ci, cj;
		P.varsFromConserved(ul, n, vi, vni, pi, Hi);
		P.varsFromConserved(ur, n, vj, vnj, pj, Hj);
		ci = P.soundSpeed(ul[0], pi);
		cj = P.soundSpeed(ur[0], pj);
		R Rij,rhoij,vij[NDIM],vm2ij,vnij,Hij,cij;
		roeAverages(ul,ur,n,vi,Hi,vj,Hj, Rij,rhoij,vij,vm2ij,vnij,Hij,cij);
		R sr, sl;
		sl = vni - ci;
		if (sl > vnij-cij) sl = vnij-cij;
		sr = vnj+cj;
		if(sr < vnij+cij) sr = vnij+cij;
		const R sm = ( ur[0]*vnj*(sr-vnj) - ul[0]*vni*(sl-vni) + pi-pj )
			/ ( ur[0]*(sr-vnj) - ul[0]*(sl-vni) );
		if(sl > 0)
			P.dirFlux(ul,n,vni,pi,flux);
		else if(sl <= 0 && sm > 0) {
			P.dirFlux(ul,n,vni,pi,flux);
			R ulstr[NVARS];
			starState(ul,n,vni,pi,sl,sm,ulstr);
			for(int iv = 0; iv < NVARS; iv++) flux[iv] += sl * ( ulstr[iv] - ul[iv]);
		}
		else if(sm <= 0 && sr >= 0) {
			P.dirFlux(ur,n,vnj,pj,flux);
			R urstr[NVARS];
			starState(ur,n,vnj,pj,sr,sm,urstr);
			for(int iv = 0; iv < NVARS; iv++) flux[iv] += sr * ( urstr[iv] - ur[iv]);
		}
		else
			P.dirFlux(ur,n,vnj,pj,flux);
	}
	void starStateJac(const R* u, const R* n, R vn, R p, R ss, R sm, const R* dvn, const R* dp,
	                  const R* dssi, const R* dsmi, const R* dssj, const R* dsmj,
	                  R* ustr, R dustri[NVARS][NVARS], R dustrj[NVARS][NVARS]) const;
	void hllc_jac(const R* ul, const R* ur, const R* n, R* dfdl, R* dfdr) const;
};

/// BC types (abctypes.hpp) and their ghost states (abc.cpp:41-437)
enum BCType { BC_SLIPWALL = 0, BC_FARFIELD = 1, BC_INOUTFLOW = 2, BC_SUBSONIC_INFLOW = 3,
              BC_EXTRAPOLATION = 4, BC_PERIODIC = 5, BC_ISOTHERMAL_WALL = 6,
              BC_ADIABATIC_WALL = 7 };

struct BC
{
	int type = -1, tag = -1;
	R vals[2] = {0,0};
	std::array<R,NVARS> uinf;
	void ghost(const Gas& P, const R* ins, const R* n, R* gs) const;
	void ghostJac(const Gas& P, const R* ins, const R* n, R* gs, R* dgs) const;
};

}
#endif
