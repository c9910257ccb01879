/** \file orc_spatial.cpp
 * \brief ORACLE (test infrastructure only): restatement of the FVENS sweep. See orc_spatial.hpp.
 */
#include "orc_spatial.hpp"
#include <cstring>
#include <cmath>
#include <stdexcept>
#include <map>

namespace orc {

static inline const double* G(const double* grads, int cell) { return grads + 8*static_cast<size_t>(cell); }
// GradBlock_t is Eigen::Array<scalar,2,4,ColMajor> (aconstants.hpp:89-90): (dim,var) at var*2+dim
static inline double gat(const double* g, int dim, int var) { return g[var*2+dim]; }

Spatial::Spatial(const OMesh& mesh, const Config& c)
	: m(mesh), cfg(c), phy(c.gamma, c.Minf, c.Tinf, c.Reinf, c.Pr),
	  invf(phy, c.flux), jacf(phy, c.jacflux)
{
	uinf = phy.freestream(c.aoa);
	for(auto b : c.bcs) { b.uinf = uinf; bcmap[b.tag] = b; }
	const int N = m.nelem;
	const double* rc = m.rc.data(); const double* rcbp = m.rcbp.data();

	if(cfg.grad == GRAD_LEASTSQUARES) {
		// WeightedLeastSquaresGradients ctor (agradientschemes.cpp:218-317); V(i,j) row-major 2x2
		V.assign(4*static_cast<size_t>(N), 0.0);
		for(int f = 0; f < m.nbface; f++) {
			const int ie = m.L(f);
			double w2 = 0, dr[2];
			for(int d = 0; d < 2; d++) {
				w2 += (rc[2*ie+d]-rcbp[2*f+d])*(rc[2*ie+d]-rcbp[2*f+d]);
				dr[d] = rc[2*ie+d]-rcbp[2*f+d];
			}
			w2 = 1.0/(w2);
			for(int i = 0; i < 2; i++) for(int j = 0; j < 2; j++) V[4*ie+2*i+j] += w2*dr[i]*dr[j];
		}
		for(int f = m.nbface; f < m.nbface+m.ninface; f++) {
			const int ie = m.L(f), je = m.Rt(f);
			double w2 = 0, dr[2];
			for(int d = 0; d < 2; d++) {
				w2 += (rc[2*ie+d]-rc[2*je+d])*(rc[2*ie+d]-rc[2*je+d]);
				dr[d] = rc[2*ie+d]-rc[2*je+d];
			}
			w2 = 1.0/(w2);
			for(int i = 0; i < 2; i++) for(int j = 0; j < 2; j++) {
				V[4*ie+2*i+j] += w2*dr[i]*dr[j];
				V[4*je+2*i+j] += w2*dr[i]*dr[j];
			}
		}
		// connectivity faces: the subdomain cell only (agradientschemes.cpp:292-310)
		for(int f = m.nbface+m.ninface; f < m.naface; f++) {
			const int ie = m.L(f), je = m.Rt(f);
			double w2 = 0, dr[2];
			for(int d = 0; d < 2; d++) {
				w2 += (rc[2*ie+d]-rc[2*je+d])*(rc[2*ie+d]-rc[2*je+d]);
				dr[d] = rc[2*ie+d]-rc[2*je+d];
			}
			w2 = 1.0/(w2);
			for(int i = 0; i < 2; i++) for(int j = 0; j < 2; j++) V[4*ie+2*i+j] += w2*dr[i]*dr[j];
		}
		// Eigen 2x2 inverse: det = m00*m11 - m10*m01; invdet = 1/det (InverseImpl.h size-2 helper)
		for(int e = 0; e < N; e++) {
			double* v = &V[4*e];
			const double det = v[0]*v[3] - v[2]*v[1];
			const double invdet = 1.0/det;
			const double t = v[0];
			v[0] = v[3]*invdet;
			v[2] = -v[2]*invdet;
			v[1] = -v[1]*invdet;
			v[3] = t*invdet;
		}
	}
	if(cfg.recon == REC_VENKATAKRISHNAN) {
		// limitedlinearreconstruction.cpp:186-205
		clength.assign(N, 0.0);
		for(int e = 0; e < N; e++) {
			for(int ifa = 0; ifa < m.nnode[e]; ifa++) {
				double llen = 0;
				const int in0 = ifa, jn = (ifa+1) % m.nnode[e];
				for(int d = 0; d < 2; d++)
					llen += std::pow(m.coords[2*m.in(e,in0)+d] - m.coords[2*m.in(e,jn)+d], 2);
				if(clength[e] < llen) clength[e] = llen;
			}
			clength[e] = std::sqrt(clength[e]);
		}
	}
}

// flow_spatial.cpp:85-93
void Spatial::boundary_state(int iface, const double* ins, double* gs) const
{
	const double n[2] = {m.nx(iface), m.ny(iface)};
	bcmap.at(m.btag(iface)).ghost(phy, ins, n, gs);
}

// flow_spatial.cpp:73-83
void Spatial::compute_boundary_states(const double* ins, double* gs) const
{
	for(int f = 0; f < m.nbface; f++) boundary_state(f, ins + 4*f, gs + 4*f);
}

void Spatial::compute_gradients(const double* u, const double* ug, double* grads) const
{
	const int N = m.nelem;
	const double* rc = m.rc.data(); const double* rcbp = m.rcbp.data();
	auto GR = [&](int cell, int dim, int var) -> double& { return grads[8*static_cast<size_t>(cell)+var*2+dim]; };
	if(cfg.grad == GRAD_ZERO) {                                    // agradientschemes.cpp:36-50
		for(int e = 0; e < N; e++) for(int j = 0; j < 2; j++) for(int i = 0; i < 4; i++) GR(e,j,i) = 0;
	}
	else if(cfg.grad == GRAD_GREENGAUSS) {                          // :61-214
		for(int e = 0; e < N; e++) for(int j = 0; j < 2; j++) for(int i = 0; i < 4; i++) GR(e,j,i) = 0;
		auto mid = [&](int f, double* md) {
			md[0] = 0; md[1] = 0;
			for(int k = 2; k < 4; k++) {
				const int ip = m.intfac[4*f+k];
				for(int d = 0; d < 2; d++) md[d] += m.coords[2*ip+d];
			}
			for(int d = 0; d < 2; d++) md[d] /= 2;
		};
#pragma omp parallel for default(shared)
		for(int f = 0; f < m.nbface; f++) {
			const int ie = m.L(f);
			double md[2]; mid(f, md);
			double dL = 0, dR = 0;
			for(int d = 0; d < 2; d++) {
				dL += (md[d]-rc[2*ie+d])*(md[d]-rc[2*ie+d]);
				dR += (md[d]-rcbp[2*f+d])*(md[d]-rcbp[2*f+d]);
			}
			dL = 1.0/std::sqrt(dL); dR = 1.0/std::sqrt(dR);
			const double ai = 1.0/m.area[ie];
			for(int iv = 0; iv < 4; iv++) {
				const double ut = (u[4*ie+iv]*dL + ug[4*f+iv]*dR)/(dL+dR) * m.len(f);
				for(int d = 0; d < 2; d++) {
#pragma omp atomic update
					GR(ie,d,iv) += (ut * m.facemetric[3*f+d])*ai;
				}
			}
		}
#pragma omp parallel for default(shared)
		for(int f = m.nbface; f < m.nbface+m.ninface; f++) {
			const int ie = m.L(f), je = m.Rt(f);
			double md[2]; mid(f, md);
			double dL = 0, dR = 0;
			for(int d = 0; d < 2; d++) {
				dL += (md[d]-rc[2*ie+d])*(md[d]-rc[2*ie+d]);
				dR += (md[d]-rc[2*je+d])*(md[d]-rc[2*je+d]);
			}
			dL = 1.0/std::sqrt(dL); dR = 1.0/std::sqrt(dR);
			const double a1 = 1.0/m.area[ie], a2 = 1.0/m.area[je];
			for(int iv = 0; iv < 4; iv++) {
				const double ut = (u[4*ie+iv]*dL + u[4*je+iv]*dR)/(dL+dR) * m.len(f);
				for(int d = 0; d < 2; d++) {
#pragma omp atomic update
					GR(ie,d,iv) += (ut * m.facemetric[3*f+d])*a1;
#pragma omp atomic update
					GR(je,d,iv) -= (ut * m.facemetric[3*f+d])*a2;
				}
			}
		}
		// connectivity faces: the subdomain cell only (:173-212)
		for(int f = m.nbface+m.ninface; f < m.naface; f++) {
			const int ie = m.L(f), je = m.Rt(f);
			double md[2]; mid(f, md);
			double dL = 0, dR = 0;
			for(int d = 0; d < 2; d++) {
				dL += (md[d]-rc[2*ie+d])*(md[d]-rc[2*ie+d]);
				dR += (md[d]-rc[2*je+d])*(md[d]-rc[2*je+d]);
			}
			dL = 1.0/std::sqrt(dL); dR = 1.0/std::sqrt(dR);
			const double a1 = 1.0/m.area[ie];
			for(int iv = 0; iv < 4; iv++) {
				const double ut = (u[4*ie+iv]*dL + u[4*je+iv]*dR)/(dL+dR) * m.len(f);
				for(int d = 0; d < 2; d++) GR(ie,d,iv) += (ut * m.facemetric[3*f+d])*a1;
			}
		}
	}
	else if(cfg.grad == GRAD_LEASTSQUARES) {                       // :322-440
		std::vector<double> fr(8*static_cast<size_t>(N), 0.0);   // f(jdim,ivar) at ivar*2+jdim
#pragma omp parallel for default(shared)
		for(int f = 0; f < m.nbface; f++) {
			const int ie = m.L(f);
			double w2 = 0, dr[2], du[4];
			for(int d = 0; d < 2; d++) {
				w2 += (rc[2*ie+d]-rcbp[2*f+d])*(rc[2*ie+d]-rcbp[2*f+d]);
				dr[d] = rc[2*ie+d]-rcbp[2*f+d];
			}
			w2 = 1.0/(w2);
			for(int iv = 0; iv < 4; iv++) du[iv] = u[4*ie+iv] - ug[4*f+iv];
			for(int iv = 0; iv < 4; iv++) for(int d = 0; d < 2; d++) {
#pragma omp atomic update
				fr[8*ie+iv*2+d] += w2*dr[d]*du[iv];
			}
		}
#pragma omp parallel for default(shared)
		for(int f = m.nbface; f < m.nbface+m.ninface; f++) {
			const int ie = m.L(f), je = m.Rt(f);
			double w2 = 0, dr[2], du[4];
			for(int d = 0; d < 2; d++) {
				w2 += (rc[2*ie+d]-rc[2*je+d])*(rc[2*ie+d]-rc[2*je+d]);
				dr[d] = rc[2*ie+d]-rc[2*je+d];
			}
			w2 = 1.0/(w2);
			for(int iv = 0; iv < 4; iv++) du[iv] = u[4*ie+iv] - u[4*je+iv];
			for(int iv = 0; iv < 4; iv++) for(int d = 0; d < 2; d++) {
#pragma omp atomic update
				fr[8*ie+iv*2+d] += w2*dr[d]*du[iv];
#pragma omp atomic update
				fr[8*je+iv*2+d] += w2*dr[d]*du[iv];
			}
		}
		// connectivity faces: the subdomain cell only (:404-427)
		for(int f = m.nbface+m.ninface; f < m.naface; f++) {
			const int ie = m.L(f), je = m.Rt(f);
			double w2 = 0, dr[2], du[4];
			for(int d = 0; d < 2; d++) {
				w2 += (rc[2*ie+d]-rc[2*je+d])*(rc[2*ie+d]-rc[2*je+d]);
				dr[d] = rc[2*ie+d]-rc[2*je+d];
			}
			w2 = 1.0/(w2);
			for(int iv = 0; iv < 4; iv++) du[iv] = u[4*ie+iv] - u[4*je+iv];
			for(int iv = 0; iv < 4; iv++) for(int d = 0; d < 2; d++) fr[8*ie+iv*2+d] += w2*dr[d]*du[iv];
		}
		// d = V*f (Eigen lazy 2x2 * 2x4 product: d(i,j) = V(i,0) f(0,j) + V(i,1) f(1,j))
#pragma omp parallel for default(shared)
		for(int e = 0; e < N; e++) {
			const double* v = &V[4*e];
			for(int iv = 0; iv < 4; iv++)
				for(int d = 0; d < 2; d++)
					GR(e,d,iv) = v[2*d+0]*fr[8*e+iv*2+0] + v[2*d+1]*fr[8*e+iv*2+1];
		}
	}
	else throw std::invalid_argument("gradient scheme");
}

void Spatial::compute_face_values(const double* up, const double* ug, const double* grads,
                                  double* ufl, double* ufr) const
{
	const int N = m.nelem, nb = m.nbface, F = m.naface;
	const double* ri = m.rc.data(); const double* ribp = m.rcbp.data(); const double* gr = m.gr.data();
	// u(jel,ivar) with the boundary-ghost deviation documented in the header
	auto U = [&](int cell, int iv) -> double {
		return cell < N + m.nconnface ? up[4*static_cast<size_t>(cell)+iv] : ug[4*static_cast<size_t>(cell-N-m.nconnface)+iv];
	};
	// reconstruction_utils.hpp:17-32
	auto linex = [&](double uc, const double* g, int iv, double lim, const double* gp, const double* rc) {
		double uf = uc;
		for(int d = 0; d < 2; d++) uf += lim*gat(g,d,iv)*(gp[d] - rc[d]);
		return uf;
	};
	switch(cfg.recon) {
	case REC_NONE: {                                               // areconstruction.cpp:51-103
		for(int f = nb+m.ninface; f < F; f++) {                    // connectivity faces: left only
			const int ie = m.L(f);
			for(int i = 0; i < 4; i++) ufl[4*f+i] = linex(up[4*ie+i], G(grads,ie), i, 1.0, gr+2*f, ri+2*ie);
		}
#pragma omp parallel for default(shared)
		for(int f = nb; f < nb+m.ninface; f++) {
			const int ie = m.L(f), je = m.Rt(f);
			for(int i = 0; i < 4; i++) {
				ufl[4*f+i] = linex(up[4*ie+i], G(grads,ie), i, 1.0, gr+2*f, ri+2*ie);
				ufr[4*f+i] = linex(up[4*je+i], G(grads,je), i, 1.0, gr+2*f, ri+2*je);
			}
		}
		for(int f = 0; f < nb; f++) {
			const int ie = m.L(f);
			for(int i = 0; i < 4; i++) ufl[4*f+i] = linex(up[4*ie+i], G(grads,ie), i, 1.0, gr+2*f, ri+2*ie);
		}
		break;
	}
	case REC_VANALBADA: {                                          // musclreconstruction.cpp:24-130
		const double eps = 1e-8, k = 1.0/3.0;
		auto bdiff = [&](const double* rI, const double* rJ, double uI, double uJ, const double* g, int iv) {
			double del = 0;
			for(int d = 0; d < 2; d++) del += gat(g,d,iv)*(rJ[d]-rI[d]);
			return 2.0*del - (uJ-uI);
		};
		auto recL = [&](double ui, double uj, double dm, double phi) {
			return ui + phi/4.0*( (1.0-k*phi)*dm + (1.0+k*phi)*(uj - ui) ); };
		auto recR = [&](double ui, double uj, double dp, double phi) {
			return uj - phi/4.0*( (1.0-k*phi)*dp + (1.0+k*phi)*(uj - ui) ); };
		for(int f = 0; f < nb; f++) {
			const int ie = m.L(f);
			for(int i = 0; i < 4; i++) {
				const double dm = bdiff(ri+2*ie, ribp+2*f, up[4*ie+i], ug[4*f+i], G(grads,ie), i);
				double phi = (2.0*dm * (ug[4*f+i] - up[4*ie+i]) + eps)
					/ (dm*dm + (ug[4*f+i] - up[4*ie+i])*(ug[4*f+i] - up[4*ie+i]) + eps);
				if(phi < 0.0) phi = 0.0;
				ufl[4*f+i] = recL(up[4*ie+i], ug[4*f+i], dm, phi);
			}
		}
#pragma omp parallel for default(shared)
		for(int f = nb; f < F; f++) {
			const int ie = m.L(f), je = m.Rt(f);
			for(int i = 0; i < 4; i++) {
				const double uI = up[4*ie+i], uJ = up[4*je+i];
				const double dm = bdiff(ri+2*ie, ri+2*je, uI, uJ, G(grads,ie), i);
				const double dp = bdiff(ri+2*ie, ri+2*je, uI, uJ, G(grads,je), i);
				double phl = (2.0*dm * (uJ - uI) + eps) / (dm*dm + (uJ - uI)*(uJ - uI) + eps);
				if(phl < 0.0) phl = 0.0;
				double phr = (2*dp * (uJ - uI) + eps) / (dp*dp + (uJ - uI)*(uJ - uI) + eps);
				if(phr < 0.0) phr = 0.0;
				ufl[4*f+i] = recL(uI, uJ, dm, phl);
				ufr[4*f+i] = recR(uI, uJ, dp, phr);
			}
		}
		break;
	}
	case REC_BARTHJESPERSEN:                                       // limitedlinearreconstruction.cpp:118-176
	case REC_VENKATAKRISHNAN: {                                    // :207-268
		const bool venk = cfg.recon == REC_VENKATAKRISHNAN;
#pragma omp parallel for default(shared)
		for(int e = 0; e < N; e++) {
			const double eps2 = venk ? std::pow(cfg.limiter_param*clength[e], 3) : 0.0;
			for(int iv = 0; iv < 4; iv++) {
				double dmin = 0, dmax = 0;
				for(int j = 0; j < m.nfael[e]; j++) {
					const int jel = m.gesuel(e,j);
					const double dui = U(jel,iv)-up[4*e+iv];
					if(dui > dmax) dmax = dui;
					if(dui < dmin) dmin = dui;
				}
				double lim = 1.0;
				for(int j = 0; j < m.nfael[e]; j++) {
					const int face = m.gelemface(e,j);
					const double uface = linex(up[4*e+iv], G(grads,e), iv, 1.0, gr+2*face, ri+2*e);
					double phiik;
					if(venk) {
						const double dm = uface - up[4*e+iv];
						const double dp = dm < 0 ? dmin : dmax;
						phiik = (dp*dp + 2*dp*dm + eps2)/(dp*dp + dp*dm + 2*dm*dm + eps2);
					} else {
						const double diff = uface - up[4*e+iv];
						if(diff>0) phiik = 1 < dmax/diff ? 1 : dmax/diff;
						else if(diff < 0) phiik = 1 < dmin/diff ? 1 : dmin/diff;
						else phiik = 1;
					}
					if(phiik < lim) lim = phiik;
				}
				for(int j = 0; j < m.nfael[e]; j++) {
					const int face = m.gelemface(e,j);
					const int jel = m.gesuel(e,j);
					if(e < jel) ufl[4*face+iv] = linex(up[4*e+iv], G(grads,e), iv, lim, gr+2*face, ri+2*e);
					else        ufr[4*face+iv] = linex(up[4*e+iv], G(grads,e), iv, lim, gr+2*face, ri+2*e);
				}
			}
		}
		break;
	}
	case REC_WENO: {                                               // :27-105
		const double gamma = 4.0, lambda = cfg.limiter_param, epsilon = 1.0e-5;
		auto gm2 = [&](const double* g, int iv) { double r = 0; for(int j = 0; j < 2; j++) r += gat(g,j,iv)*gat(g,j,iv); return r; };
#pragma omp parallel for default(shared)
		for(int e = 0; e < N; e++) {
			for(int iv = 0; iv < 4; iv++) {
				double wsum = 0, lg[2] = {0,0};
				{
					const double denom = std::pow(gm2(G(grads,e),iv) + epsilon, gamma);
					const double w = lambda / denom;
					wsum += w;
					for(int j = 0; j < 2; j++) lg[j] += w*gat(G(grads,e),j,iv);
				}
				for(int jl = 0; jl < m.nfael[e]; jl++) {
					const int je = m.gesuel(e,jl);
					if(je >= N+m.nconnface) continue;
					const double denom = std::pow(gm2(G(grads,je),iv) + epsilon, gamma);
					const double w = 1.0 / denom;
					wsum += w;
					for(int j = 0; j < 2; j++) lg[j] += w*gat(G(grads,je),j,iv);
				}
				for(int j = 0; j < 2; j++) lg[j] /= wsum;
				for(int jf = 0; jf < m.nfael[e]; jf++) {
					const int face = m.gelemface(e,jf);
					const int je = m.gesuel(e,jf);
					double* dst = e < je ? &ufl[4*face+iv] : &ufr[4*face+iv];
					*dst = up[4*e+iv];
					for(int j = 0; j < 2; j++) *dst += lg[j]*(gr[2*face+j] - ri[2*e+j]);
				}
			}
		}
		break;
	}
	default: throw std::invalid_argument("reconstruction");
	}
}

// flow_spatial.cpp:348-395 + aspatial.cpp:172-205 + viscousphysics.cpp:14-122
void Spatial::viscous_flux(const double* n, const double* rcl, const double* rcr, const double* ucl,
                           const double* ucr, const double* gradsl, const double* gradsr,
                           const double* ul, const double* ur, double* vflux) const
{
	double uctl[4], uctr[4], gradl[8], gradr[8];     // dim-major [dim][var]
	if(cfg.order2) {
		for(int i = 0; i < 2; i++) for(int j = 0; j < 4; j++) {
			gradl[i*4+j] = gat(gradsl,i,j); gradr[i*4+j] = gat(gradsr,i,j);
		}
		phy.primFromCons(ucl, uctl);
		phy.primFromCons(ucr, uctr);
		for(int j = 0; j < 2; j++) {
			gradl[j*4+3] = phy.gradTemperature(uctl[0], gradl[j*4], uctl[3], gradl[j*4+3]);
			gradr[j*4+3] = phy.gradTemperature(uctr[0], gradr[j*4], uctr[3], gradr[j*4+3]);
		}
		uctl[3] = phy.temperature(uctl[0], uctl[3]);
		uctr[3] = phy.temperature(uctr[0], uctr[3]);
	} else {
		phy.prim2FromCons(ucl, uctl);
		phy.prim2FromCons(ucr, uctr);
		for(int i = 0; i < 8; i++) { gradl[i] = 0; gradr[i] = 0; }
	}
	// getFaceGradient_modifiedAverage (aspatial.cpp:172-205)
	double grad[2][4];
	{
		double dr[2], dist = 0;
		for(int i = 0; i < 2; i++) { dr[i] = rcr[i]-rcl[i]; dist += dr[i]*dr[i]; }
		dist = std::sqrt(dist);
		for(int i = 0; i < 2; i++) dr[i] /= dist;
		for(int i = 0; i < 4; i++) {
			double davg[2];
			for(int j = 0; j < 2; j++) davg[j] = 0.5*(gradl[j*4+i] + gradr[j*4+i]);
			const double corr = (uctr[i]-uctl[i])/dist;
			const double ddr = dimDot(davg,dr);
			for(int j = 0; j < 2; j++) grad[j][i] = davg[j] - ddr*dr[j] + corr*dr[j];
		}
	}
	// computeViscousFlux (viscousphysics.cpp:70-122)
	const double muRe = cfg.constvisc ? phy.constVisc()
		: 0.5*( phy.viscFromConserved(ul) + phy.viscFromConserved(ur) );
	const double kdiff = phy.thermCond(muRe);
	double stress[2][2] = {{0,0},{0,0}};
	phy.stressTensor(muRe, grad, stress);
	vflux[0] = 0;
	for(int i = 0; i < 2; i++) {
		vflux[i+1] = 0;
		for(int j = 0; j < 2; j++) vflux[i+1] -= stress[i][j] * n[j];
	}
	double vavg[2];
	for(int j = 0; j < 2; j++) vavg[j] = 0.5*( ul[j+1]/ul[0] + ur[j+1]/ur[0] );
	vflux[3] = 0;
	for(int i = 0; i < 2; i++) {
		double comp = 0;
		for(int j = 0; j < 2; j++) comp += stress[i][j]*vavg[j];
		comp += kdiff*grad[i][3];
		vflux[3] -= comp * n[i];
	}
}

// flow_spatial.cpp:488-563
void Spatial::compute_fluxes(const double* u, const double* grads, const double* ul, const double* ur,
                             const double* ug, double* res) const
{
	const int N = m.nelem;
	static const double zg[8] = {0,0,0,0,0,0,0,0};
#pragma omp parallel for default(shared)
	for(int f = 0; f < m.naface; f++) {
		const double n[2] = {m.nx(f), m.ny(f)};
		const double len = m.len(f);
		const int le = m.L(f), re = m.Rt(f);
		double fl[4];
		invf.flux(&ul[4*f], &ur[4*f], n, fl);
		for(int iv = 0; iv < 4; iv++) fl[iv] *= len;
		if(cfg.viscous) {
			const bool isb = f < m.nbface;
			const double* rcr = isb ? &m.rcbp[2*f] : &m.rc[2*re];
			const double* ucr = isb ? &ug[4*f] : &u[4*re];
			const double* gl = cfg.order2 ? G(grads,le) : zg;
			const double* grr = cfg.order2 ? (isb ? G(grads,le) : G(grads,re)) : zg;
			double vf[4];
			viscous_flux(n, &m.rc[2*le], rcr, &u[4*le], ucr, gl, grr, &ul[4*f], &ur[4*f], vf);
			for(int iv = 0; iv < 4; iv++) fl[iv] += vf[iv]*len;
		}
		for(int iv = 0; iv < 4; iv++) {
#pragma omp atomic update
			res[4*le+iv] -= fl[iv];
		}
		if(re < N) for(int iv = 0; iv < 4; iv++) {
#pragma omp atomic update
			res[4*re+iv] += fl[iv];
		}
	}
}

// flow_spatial.cpp:565-634
void Spatial::compute_max_timestep(const double* ul, const double* ur, double* dtm) const
{
	const int N = m.nelem;
	std::vector<double> integ(N, 0.0);
#pragma omp parallel for default(shared)
	for(int f = 0; f < m.naface; f++) {
		const double n[2] = {m.nx(f), m.ny(f)};
		const double len = m.len(f);
		const int le = m.L(f), re = m.Rt(f);
		const double ci = phy.soundSpeedFromConserved(&ul[4*f]);
		const double cj = phy.soundSpeedFromConserved(&ur[4*f]);
		const double vni = dimDot(&ul[4*f+1],n)/ul[4*f];
		const double vnj = dimDot(&ur[4*f+1],n)/ur[4*f];
		double sri = (std::fabs(vni)+ci)*len;
		double srj = (std::fabs(vnj)+cj)*len;
		if(cfg.viscous) {
			double mui, muj;
			if(cfg.constvisc) { mui = phy.constVisc(); muj = phy.constVisc(); }
			else { mui = phy.viscFromConserved(&ul[4*f]); muj = phy.viscFromConserved(&ur[4*f]); }
			const double coi = std::max(4.0/(3*ul[4*f]), phy.g/ul[4*f]);
			const double coj = std::max(4.0/(3*ur[4*f]), phy.g/ur[4*f]);
			sri += coi*mui/phy.Pr * len*len/m.area[le];
			if(re < N) srj += coj*muj/phy.Pr * len*len/m.area[re];
		}
#pragma omp atomic update
		integ[le] += sri;
		if(re < N) {
#pragma omp atomic update
			integ[re] += srj;
		}
	}
#pragma omp parallel for default(shared)
	for(int e = 0; e < N; e++) dtm[e] = m.area[e]/integ[e];
}

// flow_spatial.cpp:636-816 (single domain: no connectivity faces)
void Spatial::compute_residual(const double* u, double* res, bool gettimesteps, double* dtm) const
{
	if(m.nconnface) throw std::invalid_argument("per-rank mesh: use compute_residual_ranks");
	const int N = m.nelem, nb = m.nbface, F = m.naface;
	std::vector<double> ul(4*static_cast<size_t>(F), 0.0), ur(4*static_cast<size_t>(F), 0.0);
	for(int f = 0; f < nb; f++) for(int iv = 0; iv < 4; iv++) ul[4*f+iv] = u[4*m.L(f)+iv];
	std::vector<double> ubcell(4*static_cast<size_t>(nb));
	std::vector<double> grads;
	if(cfg.order2) {
		compute_boundary_states(ul.data(), ur.data());
		std::vector<double> up(4*static_cast<size_t>(N));
		for(int f = 0; f < nb; f++) {
			for(int j = 0; j < 4; j++) ubcell[4*f+j] = ur[4*f+j];
			phy.primFromCons(&ur[4*f], &ur[4*f]);
		}
#pragma omp parallel for default(shared)
		for(int e = 0; e < N; e++) phy.primFromCons(&u[4*e], &up[4*e]);
		const double* ug = ur.data();
		grads.assign(8*static_cast<size_t>(N), 0.0);
		compute_gradients(up.data(), ug, grads.data());
		// the ghost primitive states are read by the reconstruction while uright is written,
		// exactly like the reference (ug aliases uright of the boundary faces)
		std::vector<double> ugcopy(ur.begin(), ur.begin()+4*nb);
		compute_face_values(up.data(), ugcopy.data(), grads.data(), ul.data(), ur.data());
#pragma omp parallel for default(shared)
		for(int f = nb; f < F; f++) {
			phy.consFromPrim(&ul[4*f], &ul[4*f]);
			phy.consFromPrim(&ur[4*f], &ur[4*f]);
		}
		for(int f = 0; f < nb; f++) phy.consFromPrim(&ul[4*f], &ul[4*f]);
	} else {
		for(int f = nb; f < F; f++) for(int iv = 0; iv < 4; iv++) {
			ul[4*f+iv] = u[4*m.L(f)+iv]; ur[4*f+iv] = u[4*m.Rt(f)+iv];
		}
	}
	compute_boundary_states(ul.data(), ur.data());
	const double* ugpb = cfg.order2 ? ubcell.data() : ur.data();
	compute_fluxes(u, cfg.order2 ? grads.data() : nullptr, ul.data(), ur.data(), ugpb, res);
	if(gettimesteps) compute_max_timestep(ul.data(), ur.data(), dtm);
}

// flow_spatial.cpp:95-112
void Spatial::getGradients(const double* u, double* grads) const
{
	std::vector<double> ug(4*static_cast<size_t>(m.nbface));
	for(int f = 0; f < m.nbface; f++) boundary_state(f, &u[4*m.L(f)], &ug[4*f]);
	compute_gradients(u, ug.data(), grads);
}

// flow_spatial.cpp:397-446 + aspatial.cpp:207-240 + viscousphysics.cpp:124-246
void Spatial::viscous_flux_jacobian(int iface, const double* ul, const double* ur, double* dvfi, double* dvfj) const
{
	double upr[4], upl[4], dupr[16], dupl[16];
	for(int k = 0; k < 16; k++) { dupr[k] = 0; dupl[k] = 0; }
	phy.prim2FromCons(ul, upl);
	phy.prim2FromCons(ur, upr);
	phy.jacPrim2(ul, dupl);
	phy.jacPrim2(ur, dupr);
	double grad[2][4], dgradl[2][4][4], dgradr[2][4][4];
	const int le = m.L(iface), re = m.Rt(iface);
	const double* cl = &m.rc[2*le];
	const double* cr = iface < m.nbface ? &m.rcbp[2*iface] : &m.rc[2*re];
	{
		double dr[2], dist = 0;
		for(int i = 0; i < 2; i++) { dr[i] = cr[i]-cl[i]; dist += dr[i]*dr[i]; }
		dist = std::sqrt(dist);
		for(int i = 0; i < 2; i++) dr[i] /= dist;
		for(int i = 0; i < 4; i++) {
			const double corr = (upr[i]-upl[i])/dist;
			for(int j = 0; j < 2; j++) {
				grad[j][i] = corr*dr[j];
				for(int k = 0; k < 4; k++) {
					dgradl[j][i][k] = -dupl[i*4+k]/dist * dr[j];
					dgradr[j][i][k] = dupr[i*4+k]/dist * dr[j];
				}
			}
		}
	}
	const double n[2] = {m.nx(iface), m.ny(iface)};
	const double muRe = cfg.constvisc ? phy.constVisc()
		: 0.5*( phy.viscFromConserved(ul) + phy.viscFromConserved(ur) );
	const double kdiff = phy.thermCond(muRe);
	double dmul[4] = {0,0,0,0}, dmur[4] = {0,0,0,0}, dkdl[4] = {0,0,0,0}, dkdr[4] = {0,0,0,0};
	if(!cfg.constvisc) {
		phy.jacSutherland(ul, dmul);
		phy.jacSutherland(ur, dmur);
		for(int k = 0; k < 4; k++) { dmul[k] *= 0.5; dmur[k] *= 0.5; }
		phy.jacThermCond(dmul, dkdl);
		phy.jacThermCond(dmur, dkdr);
	}
	double stress[2][2], dsl[2][2][4], dsr[2][2][4];
	for(int i = 0; i < 2; i++) for(int j = 0; j < 2; j++) {
		stress[i][j] = 0;
		for(int k = 0; k < 4; k++) { dsl[i][j][k] = 0; dsr[i][j][k] = 0; }
	}
	phy.jacStress(muRe, dmul, grad, dgradl, stress, dsl);
	phy.jacStress(muRe, dmur, grad, dgradr, stress, dsr);
	for(int i = 0; i < 2; i++)
		for(int j = 0; j < 2; j++)
			for(int k = 0; k < 4; k++) {
				dvfi[(i+1)*4+k] += dsl[i][j][k] * n[j];
				dvfj[(i+1)*4+k] -= dsr[i][j][k] * n[j];
			}
	double vavg[2], dvavgl[2][4], dvavgr[2][4];
	for(int j = 0; j < 2; j++) {
		vavg[j] = 0.5*( ul[j+1]/ul[0] + ur[j+1]/ur[0] );
		for(int k = 0; k < 4; k++) { dvavgl[j][k] = 0; dvavgr[j][k] = 0; }
		dvavgl[j][0] = -0.5*ul[j+1]/(ul[0]*ul[0]);
		dvavgr[j][0] = -0.5*ur[j+1]/(ur[0]*ur[0]);
		dvavgl[j][j+1] = 0.5/ul[0];
		dvavgr[j][j+1] = 0.5/ur[0];
	}
	for(int i = 0; i < 2; i++) {
		double dcl[4] = {0,0,0,0}, dcr[4] = {0,0,0,0};
		for(int j = 0; j < 2; j++)
			for(int k = 0; k < 4; k++) {
				dcl[k] += dsl[i][j][k]*vavg[j] + stress[i][j]*dvavgl[j][k];
				dcr[k] += dsr[i][j][k]*vavg[j] + stress[i][j]*dvavgr[j][k];
			}
		for(int k = 0; k < 4; k++) {
			dcl[k] += dkdl[k]*grad[i][3] + kdiff*dgradl[i][3][k];
			dcr[k] += dkdr[k]*grad[i][3] + kdiff*dgradr[i][3][k];
		}
		for(int k = 0; k < 4; k++) {
			dvfi[3*4+k] += dcl[k] * n[i];
			dvfj[3*4+k] -= dcr[k] * n[i];
		}
	}
}

// flow_spatial.cpp:818-839
void Spatial::local_jacobian_interior(int iface, const double* ul, const double* ur, double* L, double* U) const
{
	const double n[2] = {m.nx(iface), m.ny(iface)};
	const double len = m.len(iface);
	jacf.jacobian(ul, ur, n, L, U);
	if(cfg.viscous) viscous_flux_jacobian(iface, ul, ur, L, U);
	for(int k = 0; k < 16; k++) { L[k] *= len; U[k] *= len; }
}

// flow_spatial.cpp:841-875
void Spatial::local_jacobian_boundary(int iface, const double* ul, double* left) const
{
	const double n[2] = {m.nx(iface), m.ny(iface)};
	const double len = m.len(iface);
	double uface[4], drdl[16], right[16];
	bcmap.at(m.btag(iface)).ghostJac(phy, ul, n, uface, drdl);
	jacf.jacobian(ul, uface, n, left, right);
	if(cfg.viscous) viscous_flux_jacobian(iface, ul, uface, left, right);
	double tmp[16];
	for(int i = 0; i < 4; i++)
		for(int j = 0; j < 4; j++) {
			double s = right[i*4+0]*drdl[0*4+j];
			for(int k = 1; k < 4; k++) s += right[i*4+k]*drdl[k*4+j];
			tmp[i*4+j] = s;
		}
	for(int k = 0; k < 16; k++) left[k] = len*(left[k] - tmp[k]);
}

// aspatial.cpp:242-340 (single domain; PETSc ADD_VALUES in face order)
void Spatial::assemble_jacobian(const double* u, double* diag, double* lower, double* upper) const
{
	for(int f = 0; f < m.nbface; f++) {
		const int le = m.L(f);
		double left[16];
		local_jacobian_boundary(f, &u[4*le], left);
		for(int k = 0; k < 16; k++) diag[16*le+k] += -1.0*left[k];
	}
	for(int f = m.nbface; f < m.nbface+m.ninface; f++) {
		const int le = m.L(f), re = m.Rt(f);
		double L[16], U[16];
		local_jacobian_interior(f, &u[4*le], &u[4*re], L, U);
		const size_t fi = static_cast<size_t>(f - m.nbface);
		for(int k = 0; k < 16; k++) { lower[16*fi+k] += L[k]; upper[16*fi+k] += U[k]; }
		for(int k = 0; k < 16; k++) { diag[16*le+k] += -1.0*L[k]; }
		for(int k = 0; k < 16; k++) { diag[16*re+k] += -1.0*U[k]; }
	}
}

// alinalg.cpp:142-233 (ghost rows zeroed explicitly)
void Spatial::matfree_apply(const double* u, const double* res, const double* mdt, double eps,
                            const double* x, double* y) const
{
	const size_t n = 4*static_cast<size_t>(m.nelem);
	double s = 0;
	for(size_t i = 0; i < n; i++) s += x[i]*x[i];
	const double xnorm = std::sqrt(s);
	const double pertmag = eps/xnorm;
	std::vector<double> aux(n), yg(n, 0.0);
	for(size_t i = 0; i < n; i++) aux[i] = u[i] + pertmag * x[i];
	compute_residual(aux.data(), yg.data(), false, nullptr);
	for(int e = 0; e < m.nelem; e++)
		for(int i = 0; i < 4; i++)
			y[4*e+i] = mdt[e]*x[4*e+i] + (-yg[4*e+i] + res[4*e+i])/pertmag;
}

int steady_forward_euler(const Spatial& s, double* u, double cfl, double tol, int maxiter, double* resratio)
{
	const int N = s.m.nelem;
	std::vector<double> r(4*static_cast<size_t>(N)), dtm(N);
	double resi = 1.0, initres = 1.0;
	int step = 0;
	while(resi/initres > tol && step < maxiter) {
		std::fill(r.begin(), r.end(), 0.0);
		s.compute_residual(u, r.data(), true, dtm.data());
		for(int e = 0; e < N; e++)
			for(int i = 0; i < 4; i++)
				u[4*e+i] += cfl*dtm[e] * 1.0/s.m.area[e]*r[4*e+i];
		double locres = 0;
		for(int e = 0; e < N; e++) locres += r[4*e+3]*r[4*e+3]*s.m.area[e];
		resi = std::sqrt(locres);
		if(step == 0) initres = resi;
		step++;
		if(!std::isfinite(resi)) throw std::runtime_error("forward Euler diverged");
	}
	if(resratio) *resratio = resi/initres;
	return step;
}

std::array<double,3> surface_functionals(const Spatial& s, const double* u, const double* grads, int iwbcm)
{
	const OMesh& m = s.m;
	const double aoa = s.cfg.aoa;
	const double wind[2] = {std::cos(aoa)*std::cos(0.0), std::sin(aoa)*std::cos(0.0)};
	double totalarea = 0, Cdf = 0, Cdp = 0, Cl = 0;
	const double pinf = s.phy.freestreamPressure();
	const double flownormal[2] = {-wind[1], wind[0]};
	for(int f = 0; f < m.nbface; f++) {
		if(m.btag(f) != iwbcm) continue;
		const int le = m.L(f);
		const double n[2] = {m.nx(f), m.ny(f)};
		const double area = m.len(f);
		const double tangf[2] = {n[1], -n[0]};
		double urec[4];
		for(int i = 0; i < 4; i++) urec[i] = u[4*le+i];
		const double cp = (s.phy.pressureFromConserved(urec) - pinf)*2.0;
		const double muhat = s.phy.viscFromConserved(urec);
		double gradu[2][2];
		const double* g = G(grads, le);
		for(int i = 0; i < 2; i++)
			for(int j = 0; j < 2; j++)
				gradu[i][j] = (gat(g,j,i+1)*urec[0] - urec[i+1]*gat(g,j,0)) / (urec[0]*urec[0]);
		double force[2];
		for(int i = 0; i < 2; i++) {
			force[i] = 0;
			for(int j = 0; j < 2; j++) force[i] += (gradu[i][j] + gradu[j][i])*n[j];
		}
		const double tauw = muhat*dimDot(force,tangf);
		const double cf = 2*tauw;
		const double ndotw = dimDot(n,wind), ndotnw = dimDot(n,flownormal), tdotw = dimDot(tangf,wind);
		totalarea += area;
		Cl += cp*ndotnw*area;
		Cdp += cp*ndotw*area;
		Cdf += cf*tdotw*area;
	}
	Cdp /= totalarea; Cdf /= totalarea; Cl /= totalarea;
	return {Cl, Cdp, Cdf};
}

// flow_spatial.cpp:636-816 on every rank of a partition (per-rank meshes with connectivity faces),
// with the exchanges the reference makes over MPI in between: the ghost gradients (VecGhostUpdate on
// gradvec, :711-729 and :784-787) and the face traces (L2TraceVector::updateSharedFaces, :738 and
// :782, tracevector.cpp:213-340); the ghost rows of u come in filled (the driver's VecGhostUpdate)
void compute_residual_ranks(const std::vector<const Spatial*>& S, const std::vector<const double*>& u,
                            const std::vector<double*>& res, bool gettimesteps, const std::vector<double*>& dtm)
{
	const size_t P = S.size();
	const Config& cfg = S[0]->cfg;
	struct St { std::vector<double> ul, ur, ubcell, up, grads; };
	std::vector<St> st(P);
	// owner-local index of a global cell
	std::map<int, std::pair<int,int>> owner;
	for(size_t r = 0; r < P; r++)
		for(int e = 0; e < S[r]->m.nelem; e++) owner[S[r]->m.globalElemIndex[e]] = {static_cast<int>(r), e};
	auto ghostGradients = [&]() {
		for(size_t r = 0; r < P; r++) {
			const OMesh& m = S[r]->m;
			for(int ic = 0; ic < m.nconnface; ic++) {
				const auto o = owner.at(m.gconnface(ic,3));
				for(int k = 0; k < 8; k++)
					st[r].grads[8*(static_cast<size_t>(m.nelem)+ic)+k] = st[o.first].grads[8*static_cast<size_t>(o.second)+k];
			}
		}
	};
	for(size_t r = 0; r < P; r++) {
		const Spatial& s = *S[r];
		const OMesh& m = s.m;
		const int N = m.nelem, nb = m.nbface, F = m.naface;
		St& a = st[r];
		a.ul.assign(4*static_cast<size_t>(F), 0.0); a.ur.assign(4*static_cast<size_t>(F), 0.0);
		for(int f = 0; f < nb; f++) for(int iv = 0; iv < 4; iv++) a.ul[4*f+iv] = u[r][4*m.L(f)+iv];
		a.ubcell.assign(4*static_cast<size_t>(nb), 0.0);
		if(cfg.order2) {
			s.compute_boundary_states(a.ul.data(), a.ur.data());
			a.up.assign(4*static_cast<size_t>(N+m.nconnface), 0.0);
			for(int f = 0; f < nb; f++) {
				for(int j = 0; j < 4; j++) a.ubcell[4*f+j] = a.ur[4*f+j];
				s.phy.primFromCons(&a.ur[4*f], &a.ur[4*f]);
			}
			for(int e = 0; e < N+m.nconnface; e++) s.phy.primFromCons(&u[r][4*e], &a.up[4*e]);
			a.grads.assign(8*static_cast<size_t>(N+m.nconnface), 0.0);
			s.compute_gradients(a.up.data(), a.ur.data(), a.grads.data());
		}
	}
	if(cfg.order2) {
		if(cfg.recon == REC_WENO) ghostGradients();
		for(size_t r = 0; r < P; r++) {
			const Spatial& s = *S[r];
			const OMesh& m = s.m;
			const int nb = m.nbface, F = m.naface, cs = nb + m.ninface;
			St& a = st[r];
			std::vector<double> ugcopy(a.ur.begin(), a.ur.begin()+4*nb);
			s.compute_face_values(a.up.data(), ugcopy.data(), a.grads.data(), a.ul.data(), a.ur.data());
			for(int f = cs; f < F; f++) s.phy.consFromPrim(&a.ul[4*f], &a.ul[4*f]);
			for(int f = nb; f < cs; f++) {
				s.phy.consFromPrim(&a.ul[4*f], &a.ul[4*f]);
				s.phy.consFromPrim(&a.ur[4*f], &a.ur[4*f]);
			}
			for(int f = 0; f < nb; f++) s.phy.consFromPrim(&a.ul[4*f], &a.ul[4*f]);
		}
		// trace exchange: a connectivity face's right state is the neighbour's left state of the
		// same global face
		for(size_t r = 0; r < P; r++) {
			const OMesh& m = S[r]->m;
			const int cs = m.nbface + m.ninface;
			for(int ic = 0; ic < m.nconnface; ic++) {
				const int q = m.gconnface(ic,2), gf = m.gconnface(ic,4);
				const OMesh& mq = S[q]->m;
				const int csq = mq.nbface + mq.ninface;
				int jc = 0;
				while(jc < mq.nconnface && mq.gconnface(jc,4) != gf) jc++;
				if(jc == mq.nconnface) throw std::logic_error("connectivity face without a partner");
				for(int iv = 0; iv < 4; iv++) st[r].ur[4*(cs+ic)+iv] = st[q].ul[4*(csq+jc)+iv];
			}
		}
		if(cfg.recon != REC_WENO) ghostGradients();
	} else {
		for(size_t r = 0; r < P; r++) {
			const OMesh& m = S[r]->m;
			for(int f = m.nbface; f < m.naface; f++) for(int iv = 0; iv < 4; iv++) {
				st[r].ul[4*f+iv] = u[r][4*m.L(f)+iv]; st[r].ur[4*f+iv] = u[r][4*m.Rt(f)+iv];
			}
		}
	}
	for(size_t r = 0; r < P; r++) {
		const Spatial& s = *S[r];
		St& a = st[r];
		s.compute_boundary_states(a.ul.data(), a.ur.data());
		const double* ugpb = cfg.order2 ? a.ubcell.data() : a.ur.data();
		s.compute_fluxes(u[r], cfg.order2 ? a.grads.data() : nullptr, a.ul.data(), a.ur.data(), ugpb, res[r]);
		if(gettimesteps) s.compute_max_timestep(a.ul.data(), a.ur.data(), dtm[r]);
	}
}

}
