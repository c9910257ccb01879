/** \file orc_api.cpp
 * \brief ORACLE (test infrastructure only): flat C entry points over the restated reference, for
 *   tests/ (ctypes), __graft_entry__.smoke() and bench.py's cpu_baseline leg. Nothing in the
 *   product links or loads this library.
 */
#include "orc_spatial.hpp"
#include <cstring>
#include <string>
#include <stdexcept>
#include <chrono>
#include <algorithm>
#include <cmath>
#ifdef _OPENMP
#include <omp.h>
#endif

using namespace orc;

static thread_local std::string g_err;

#define ORC_TRY(body) try { body; return 0; } catch(const std::exception& e) { g_err = e.what(); return -1; }

extern "C" {

const char* orc_last_error() { return g_err.c_str(); }

void* orc_mesh_read(const char* path)
{
	try { OMesh* m = new OMesh(orc_readGmsh2(path)); orc_preprocess(*m); return m; }
	catch(const std::exception& e) { g_err = e.what(); return nullptr; }
}

void* orc_mesh_from_raw(int npoin, const double* coords, int nelem, int maxnnode, const int* inpoel,
                        const int* nnode, int nbface, int nbtag, const int* bface)
{
	try {
		OMesh* m = new OMesh(orc_fromRaw(npoin, coords, nelem, maxnnode, inpoel, nnode, nbface, nbtag, bface));
		orc_preprocess(*m);
		return m;
	} catch(const std::exception& e) { g_err = e.what(); return nullptr; }
}

void orc_mesh_free(void* h) { delete static_cast<OMesh*>(h); }

/// subdomain `rank` of a preprocessed global mesh under elemdist (meshpartitioning.cpp:24-159)
void* orc_mesh_restrict(void* gm, const int* elemdist, int rank)
{
	try {
		const OMesh& g = *static_cast<OMesh*>(gm);
		return new OMesh(orc_restrict(g, std::vector<int>(elemdist, elemdist + g.nelem), rank));
	} catch(const std::exception& e) { g_err = e.what(); return nullptr; }
}

int orc_partition_trivial(int nelem, int nranks, int* elemdist)
{
	ORC_TRY(const std::vector<int> d = orc_partition_trivial(nelem, nranks); std::memcpy(elemdist, d.data(), d.size()*sizeof(int)))
}

/// compute_residual on all ranks of a partition (handles of Spatials over per-rank meshes)
int orc_residual_ranks(int n, void** spatials, const double** u, double** res, int gettimesteps, double** dtm)
{
	ORC_TRY(
		std::vector<const Spatial*> S;
		for(int i = 0; i < n; i++) S.push_back(static_cast<const Spatial*>(spatials[i]));
		compute_residual_ranks(S, std::vector<const double*>(u, u+n), std::vector<double*>(res, res+n),
		                       gettimesteps != 0, gettimesteps ? std::vector<double*>(dtm, dtm+n) : std::vector<double*>(n, nullptr))
	)
}

/// info: npoin, nelem, nbface, naface, ninface, maxnnode, maxnfael, nbtag, nconnface
void orc_mesh_info(void* h, int* info)
{
	const OMesh& m = *static_cast<OMesh*>(h);
	info[0] = m.npoin; info[1] = m.nelem; info[2] = m.nbface; info[3] = m.naface;
	info[4] = m.ninface; info[5] = m.maxnnode; info[6] = m.maxnfael; info[7] = m.nbtag;
	info[8] = m.nconnface;
}

/// Copies a named mesh array out. Names: coords inpoel bface esuel elemface intfac btags
/// facemetric area rc gr rcbp
int orc_mesh_get(void* h, const char* name, void* out)
{
	const OMesh& m = *static_cast<OMesh*>(h);
	const std::string s(name);
	auto cpi = [&](const std::vector<int>& v) { std::memcpy(out, v.data(), v.size()*sizeof(int)); };
	auto cpd = [&](const std::vector<double>& v) { std::memcpy(out, v.data(), v.size()*sizeof(double)); };
	if(s == "coords") cpd(m.coords); else if(s == "inpoel") cpi(m.inpoel); else if(s == "bface") cpi(m.bface);
	else if(s == "esuel") cpi(m.esuel); else if(s == "elemface") cpi(m.elemface);
	else if(s == "intfac") cpi(m.intfac); else if(s == "btags") cpi(m.btags);
	else if(s == "facemetric") cpd(m.facemetric); else if(s == "area") cpd(m.area);
	else if(s == "rc") cpd(m.rc); else if(s == "gr") cpd(m.gr); else if(s == "rcbp") cpd(m.rcbp);
	else if(s == "connface") cpi(m.connface); else if(s == "globalElemIndex") cpi(m.globalElemIndex);
	else { g_err = "unknown array " + s; return -1; }
	return 0;
}

/// dparams: gamma Minf Tinf Reinf Pr aoa limiter_param
/// iparams: viscous constvisc order2 flux jacflux grad recon nbc
void* orc_spatial_create(void* mesh, const double* dp, const int* ip, const int* bctype,
                         const int* bctag, const double* bcvals)
{
	try {
		Config c;
		c.gamma = dp[0]; c.Minf = dp[1]; c.Tinf = dp[2]; c.Reinf = dp[3]; c.Pr = dp[4]; c.aoa = dp[5];
		c.limiter_param = dp[6];
		c.viscous = ip[0]; c.constvisc = ip[1]; c.order2 = ip[2]; c.flux = ip[3]; c.jacflux = ip[4];
		c.grad = ip[5]; c.recon = ip[6];
		for(int i = 0; i < ip[7]; i++) {
			BC b; b.type = bctype[i]; b.tag = bctag[i]; b.vals[0] = bcvals[2*i]; b.vals[1] = bcvals[2*i+1];
			c.bcs.push_back(b);
		}
		return new Spatial(*static_cast<OMesh*>(mesh), c);
	} catch(const std::exception& e) { g_err = e.what(); return nullptr; }
}

void orc_spatial_free(void* h) { delete static_cast<Spatial*>(h); }

int orc_residual(void* h, const double* u, double* res, int gettimesteps, double* dtm)
{ ORC_TRY(static_cast<Spatial*>(h)->compute_residual(u, res, gettimesteps != 0, dtm)) }

int orc_gradients(void* h, const double* u, double* grads)
{ ORC_TRY(static_cast<Spatial*>(h)->getGradients(u, grads)) }

int orc_compute_gradients(void* h, const double* u, const double* ug, double* grads)
{ ORC_TRY(static_cast<Spatial*>(h)->compute_gradients(u, ug, grads)) }

int orc_face_values(void* h, const double* up, const double* ug, const double* grads, double* ufl, double* ufr)
{ ORC_TRY(static_cast<Spatial*>(h)->compute_face_values(up, ug, grads, ufl, ufr)) }

int orc_boundary_states(void* h, const double* ins, double* gs)
{ ORC_TRY(static_cast<Spatial*>(h)->compute_boundary_states(ins, gs)) }

int orc_jacobian(void* h, const double* u, double* diag, double* lower, double* upper)
{ ORC_TRY(static_cast<Spatial*>(h)->assemble_jacobian(u, diag, lower, upper)) }

int orc_matfree(void* h, const double* u, const double* res, const double* mdt, double eps,
                const double* x, double* y)
{ ORC_TRY(static_cast<Spatial*>(h)->matfree_apply(u, res, mdt, eps, x, y)) }

int orc_forward_euler(void* h, double* u, double cfl, double tol, int maxiter, int* steps, double* ratio)
{ ORC_TRY(*steps = steady_forward_euler(*static_cast<Spatial*>(h), u, cfl, tol, maxiter, ratio)) }

int orc_surface(void* h, const double* u, const double* grads, int marker, double* out3)
{
	ORC_TRY(auto r = surface_functionals(*static_cast<Spatial*>(h), u, grads, marker);
	        out3[0] = r[0]; out3[1] = r[1]; out3[2] = r[2])
}

/// FlowOutput::compute_entropy_cell (aoutput.cpp:28-62), single rank, serial order
int orc_entropy(void* h, const double* u, double* err)
{
	ORC_TRY(
		const Spatial& s = *static_cast<Spatial*>(h);
		const double sinf = s.phy.pressureFromConserved(s.uinf.data())/std::pow(s.uinf[0], s.phy.g);
		double e = 0;
		for(int iel = 0; iel < s.m.nelem; iel++) {
			const double serr = (s.phy.pressureFromConserved(&u[4*static_cast<size_t>(iel)])
			                     /std::pow(u[4*static_cast<size_t>(iel)], s.phy.g) - sinf) / sinf;
			e += serr*serr*s.m.area[iel];
		}
		*err = std::sqrt(e)
	)
}

/// point-wise flux: gas = {gamma, Minf, Tinf, Reinf, Pr}
int orc_flux(int type, const double* gas, const double* ul, const double* ur, const double* n, double* f)
{
	ORC_TRY(Gas p(gas[0], gas[1], gas[2], gas[3], gas[4]); Flux fl(p, type); fl.flux(ul, ur, n, f))
}

int orc_flux_jacobian(int type, const double* gas, const double* ul, const double* ur, const double* n,
                      double* dfdl, double* dfdr)
{
	ORC_TRY(Gas p(gas[0], gas[1], gas[2], gas[3], gas[4]); Flux fl(p, type); fl.jacobian(ul, ur, n, dfdl, dfdr))
}

/// point-wise BC ghost state; aoa for the free stream
int orc_bc_ghost(int type, const double* gas, double aoa, const double* vals, const double* ins,
                 const double* n, double* gs, double* dgs)
{
	ORC_TRY(Gas p(gas[0], gas[1], gas[2], gas[3], gas[4]); BC b; b.type = type;
	        b.vals[0] = vals[0]; b.vals[1] = vals[1]; b.uinf = p.freestream(aoa);
	        if(dgs) b.ghostJac(p, ins, n, gs, dgs); else b.ghost(p, ins, n, gs))
}

/// OpenMP threads of the restatement (1 by default: the reference's single-thread order)
static struct OmpOne { OmpOne() { omp_set_num_threads(1); } } g_omp_one;
int orc_set_threads(int n) { omp_set_num_threads(n < 1 ? 1 : n); return omp_get_max_threads(); }

/// CPU baseline timing: nwarm untimed sweeps, then nrep sweeps of compute_residual
/// each timed with std::chrono::steady_clock; times[nrep] receives the seconds of each sweep and the
/// median is returned
double orc_time_residual(void* h, const double* u, int nwarm, int nrep, int gettimesteps, double* times)
{
	Spatial& s = *static_cast<Spatial*>(h);
	std::vector<double> r(4*static_cast<size_t>(s.m.nelem)), dtm(s.m.nelem), t(std::max(nrep, 1));
	for(int i = 0; i < nwarm; i++) {
		std::fill(r.begin(), r.end(), 0.0);
		s.compute_residual(u, r.data(), gettimesteps != 0, dtm.data());
	}
	for(int i = 0; i < nrep; i++) {
		std::fill(r.begin(), r.end(), 0.0);
		const auto t0 = std::chrono::steady_clock::now();
		s.compute_residual(u, r.data(), gettimesteps != 0, dtm.data());
		const auto t1 = std::chrono::steady_clock::now();
		t[i] = std::chrono::duration<double>(t1-t0).count();
		if(times) times[i] = t[i];
	}
	std::sort(t.begin(), t.begin() + nrep);
	return nrep % 2 ? t[nrep/2] : 0.5*(t[nrep/2-1] + t[nrep/2]);
}

}
