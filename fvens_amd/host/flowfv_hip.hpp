/** \file flowfv_hip.hpp
 * \brief C++ host face of libfvhip.so mirroring FVENS's flow spatial-discretisation API.
 *
 * Header-only; depends only on include/fvhip.h and the C++ standard library (no PETSc, no Eigen),
 * so it can be compiled into the reference tree or any other driver. Names, argument meaning and
 * error behaviour follow the reference:
 *   FlowBCConfig        spatial/abc.hpp:34-40        (bc_tag, bc_type, bc_vals)
 *   FlowPhysicsConfig   spatial/flow_spatial.hpp:33-44
 *   FlowNumericsConfig  spatial/flow_spatial.hpp:47-55 (strings as the control file gives them)
 *   FlowFV_HIP          FlowFV<scalar,order2,constVisc> spatial/flow_spatial.hpp:174-320 behind the
 *                       Spatial<freal,NVARS> interface (aspatial.hpp:62-92)
 *   InviscidFlux_HIP    InviscidFlux::get_flux / get_jacobian (anumericalflux.hpp:19-57), batched
 *   MatrixFreeSpatialJacobian_HIP  linalg/alinalg.hpp MatrixFreeSpatialJacobian (set_state/apply)
 * Strings are mapped exactly as the reference's factories map them (afactory.cpp:38-81, 111-127,
 * 178-211): an unknown flux name is an error, an unknown gradient scheme means "zero gradients".
 * Methods return StatusCode 0 like the reference and throw std::runtime_error (the reference's
 * fvens_throw) when the library reports an error.
 */
#ifndef FVENS_HIP_FLOWFV_HIP_HPP
#define FVENS_HIP_FLOWFV_HIP_HPP

#include "../../include/fvhip.h"

#include <stdexcept>
#include <string>
#include <vector>
#include <map>

namespace fvens_hip {

typedef int StatusCode;

/// spatial/abctypes.hpp:12-21, same enumerator order
enum BCType {
	SLIP_WALL_BC = FVHIP_BC_SLIPWALL, FARFIELD_BC = FVHIP_BC_FARFIELD,
	INFLOW_OUTFLOW_BC = FVHIP_BC_INFLOW_OUTFLOW, SUBSONIC_INFLOW_BC = FVHIP_BC_SUBSONIC_INFLOW,
	EXTRAPOLATION_BC = FVHIP_BC_EXTRAPOLATION, PERIODIC_BC = FVHIP_BC_PERIODIC,
	ISOTHERMAL_WALL_BC = FVHIP_BC_ISOTHERMAL_WALL, ADIABATIC_WALL_BC = FVHIP_BC_ADIABATIC_WALL
};

struct FlowBCConfig {
	int bc_tag;
	BCType bc_type;
	std::vector<double> bc_vals;
	std::vector<int> bc_opts;
};

struct FlowPhysicsConfig {
	double gamma, Minf, Tinf, Reinf, Pr, aoa;
	bool viscous_sim, const_visc;
	std::vector<FlowBCConfig> bcconf;
};

struct FlowNumericsConfig {
	std::string conv_numflux, conv_numflux_jac, gradientscheme, reconstruction;
	double limiter_param;
	bool order2;
	bool fast_math = false;    ///< not a reference option (include/fvhip.h)
};

inline void check(int rc) {
	if(rc != 0) throw std::runtime_error(std::string("fvhip: ") + fvhip_last_error());
}

/// afactory.cpp:38-81
inline int fluxFromName(const std::string& s) {
	static const std::map<std::string,int> m = {
		{"VANLEER", FVHIP_FLUX_VANLEER}, {"ROE", FVHIP_FLUX_ROE}, {"HLL", FVHIP_FLUX_HLL},
		{"HLLC", FVHIP_FLUX_HLLC}, {"LLF", FVHIP_FLUX_LLF}, {"AUSM", FVHIP_FLUX_AUSM},
		{"AUSMPLUS", FVHIP_FLUX_AUSMPLUS}};
	const auto it = m.find(s);
	if(it == m.end()) throw std::invalid_argument("Inviscid flux not available!");
	return it->second;
}
/// afactory.cpp:111-127: anything else is the zero-gradient scheme
inline int gradientFromName(const std::string& s) {
	if(s == "LEASTSQUARES") return FVHIP_GRAD_LEASTSQUARES;
	if(s == "GREENGAUSS") return FVHIP_GRAD_GREENGAUSS;
	return FVHIP_GRAD_ZERO;
}
/// afactory.cpp:178-211
inline int reconstructionFromName(const std::string& s) {
	static const std::map<std::string,int> m = {
		{"NONE", FVHIP_REC_NONE}, {"WENO", FVHIP_REC_WENO}, {"VANALBADA", FVHIP_REC_VANALBADA},
		{"BARTHJESPERSEN", FVHIP_REC_BARTHJESPERSEN}, {"VENKATAKRISHNAN", FVHIP_REC_VENKATAKRISHNAN}};
	const auto it = m.find(s);
	if(it == m.end()) throw std::invalid_argument("Reconstruction scheme not available!");
	return it->second;
}

/// Device-resident FlowFV. u is the ghosted state [nelem+nconnface][4] in the mesh's numbering.
class FlowFV_HIP
{
public:
	FlowFV_HIP(const fvhip_mesh& mesh, const FlowPhysicsConfig& pconf, const FlowNumericsConfig& nconf,
	           int device = 0)
		: m(mesh), pc(pconf), nc(nconf)
	{
		for(const FlowBCConfig& b : pc.bcconf) {
			bctype.push_back(b.bc_type);
			bctag.push_back(b.bc_tag);
			bcvals.push_back(b.bc_vals.size() > 0 ? b.bc_vals[0] : 0.0);
			bcvals.push_back(b.bc_vals.size() > 1 ? b.bc_vals[1] : 0.0);
		}
		fvhip_flow_config c{};
		c.gamma = pc.gamma; c.Minf = pc.Minf; c.Tinf = pc.Tinf; c.Reinf = pc.Reinf; c.Pr = pc.Pr;
		c.aoa = pc.aoa; c.viscous_sim = pc.viscous_sim; c.const_visc = pc.const_visc;
		c.conv_numflux = fluxFromName(nc.conv_numflux);
		c.conv_numflux_jac = fluxFromName(nc.conv_numflux_jac);
		c.gradientscheme = gradientFromName(nc.gradientscheme);
		c.reconstruction = reconstructionFromName(nc.reconstruction);
		c.limiter_param = nc.limiter_param;
		c.order2 = nc.order2 ? 1 : 0;   // FlowFV<., order2, .> template choice, afactory.cpp:251-267
		c.nbc = static_cast<int>(bctype.size());
		c.bc_type = bctype.data(); c.bc_tag = bctag.data(); c.bc_vals = bcvals.data();
		c.fast_math = nc.fast_math ? 1 : 0;
		check(fvhip_create(&m, &c, device, &h));
	}
	~FlowFV_HIP() { if(h) fvhip_destroy(h); }
	FlowFV_HIP(const FlowFV_HIP&) = delete;
	FlowFV_HIP& operator=(const FlowFV_HIP&) = delete;

	const fvhip_mesh& mesh() const { return m; }
	fvhip_handle handle() const { return h; }

	/// Adds -r(u) into residual; computes local time steps if asked (flow_spatial.hpp:186-197)
	StatusCode compute_residual(const double* u, double* residual, bool gettimesteps, double* dtm) const {
		check(fvhip_compute_residual(h, u, residual, gettimesteps ? 1 : 0, dtm));
		return 0;
	}
	/// Same on device arrays in the library's internal cell order (asynchronous)
	StatusCode compute_residual_device(const double* d_u, double* d_r, bool gettimesteps, double* d_dtm,
	                                   bool zeroed = true) const {
		check(fvhip_compute_residual_device(h, d_u, d_r, gettimesteps ? 1 : 0, d_dtm,
		                                    zeroed ? FVHIP_RES_OVERWRITE : 0));
		return 0;
	}
	/// FlowFV_base::getGradients (GradBlock_t array, [nelem][4 vars][2 dims])
	void getGradients(const double* u, double* grads) const { check(fvhip_get_gradients(h, u, grads)); }

	/// Spatial::assemble_jacobian in face-block form: diag [nelem][16], lower/upper [ninface][16]
	StatusCode assemble_jacobian(const double* u, double* diag, double* lower, double* upper) const {
		check(fvhip_assemble_jacobian(h, u, diag, lower, upper));
		return 0;
	}
	/// Block-CSR (BAIJ, bs = 4) pattern and values, as setJacobianPreallocation + assemble_jacobian
	void jacobian_pattern(std::vector<int>& rowptr, std::vector<int>& colind) const {
		const int ninface = m.naface - m.nbface - m.nconnface;
		rowptr.assign(m.nelem + 1, 0);
		colind.assign(static_cast<size_t>(m.nelem) + 2*static_cast<size_t>(ninface), 0);
		check(fvhip_jacobian_pattern(h, rowptr.data(), colind.data()));
	}
	StatusCode assemble_jacobian_bsr(const double* u, const std::vector<int>& rowptr,
	                                 const std::vector<int>& colind, double* vals) const {
		check(fvhip_assemble_jacobian_bsr(h, u, rowptr.data(), colind.data(), vals));
		return 0;
	}

	/// permutation: perm[internal] = reference cell
	std::vector<int> permutation() const {
		std::vector<int> p(m.nelem);
		check(fvhip_get_permutation(h, p.data()));
		return p;
	}
	void synchronize() const { check(fvhip_synchronize(h)); }

private:
	fvhip_mesh m;
	FlowPhysicsConfig pc;
	FlowNumericsConfig nc;
	std::vector<int> bctype, bctag;
	std::vector<double> bcvals;
	fvhip_handle h = nullptr;
};

/// MatrixFreeSpatialJacobian (alinalg.hpp): y = (V/dt) x + [r(u) - r(u + eps x/|x|)] |x| / eps
class MatrixFreeSpatialJacobian_HIP
{
public:
	explicit MatrixFreeSpatialJacobian_HIP(const FlowFV_HIP* s, double eps = 1e-7) : spatial(s) {
		check(fvhip_matfree_set_eps(spatial->handle(), eps));
	}
	/// u: state, r: -r(u) as stored by the caller, mdt: area/(CFL dt) (alinalg.cpp:131-140)
	int set_state(const double* u, const double* r, const double* mdt) {
		check(fvhip_matfree_set_state(spatial->handle(), u, r, mdt));
		return 0;
	}
	StatusCode apply(const double* x, double* y) const {
		check(fvhip_matfree_apply(spatial->handle(), x, y));
		return 0;
	}
private:
	const FlowFV_HIP* spatial;
};

/// SteadyForwardEulerSolver (aodesolver.hpp:113-131) with the state kept on the device
class SteadyForwardEulerSolver_HIP
{
public:
	SteadyForwardEulerSolver_HIP(const FlowFV_HIP* s, double cflinit, double tol, int maxiter)
		: spatial(s), cfl(cflinit), tol(tol), maxiter(maxiter) { }
	/// d_u: device state in the library's internal cell order; throws like the reference's
	/// Tolerance_error when the tolerance is not reached (aodesolver.cpp:263-268)
	StatusCode solve(double* d_u) {
		hist.assign(maxiter > 0 ? maxiter : 1, 0.0);
		check(fvhip_steady_forward_euler_device(spatial->handle(), d_u, cfl, tol, maxiter, &steps, &ratio, hist.data()));
		hist.resize(steps);
		if(steps == maxiter)     // the reference's test, even if the last step reached tol
			throw std::runtime_error("Steady forward Euler did not converge to specified tolerance!");
		return 0;
	}
	int steps = 0;
	double ratio = 1.0;
	std::vector<double> hist;     ///< energy-residual norm per step
private:
	const FlowFV_HIP* spatial;
	double cfl, tol;
	int maxiter;
};

/// SteadyBackwardEulerSolver (aodesolver.hpp:133-189) with the linear systems solved on the device
/// (GMRES + block-Jacobi instead of PETSc's KSP; fvhip_implicit_config holds SteadySolverConfig and
/// the -ksp_* / -matrix_free_* options)
class SteadyBackwardEulerSolver_HIP
{
public:
	SteadyBackwardEulerSolver_HIP(const FlowFV_HIP* s, const fvhip_implicit_config& c) : spatial(s), conf(c) { }
	/// d_u: device state (internal order); throws like Tolerance_error / Numerical_error
	/// (aodesolver.cpp:618-632) when the solve does not converge
	StatusCode solve(double* d_u) {
		hist.assign(conf.maxiter > 0 ? conf.maxiter : 1, 0.0);
		check(fvhip_steady_backward_euler_device(spatial->handle(), d_u, &conf, &stats, hist.data()));
		hist.resize(stats.steps);
		if(!stats.converged)
			throw std::runtime_error("Steady backward Euler did not converge to specified tolerance!");
		return 0;
	}
	fvhip_solve_stats stats{};
	std::vector<double> hist;     ///< energy-residual norm per step
private:
	const FlowFV_HIP* spatial;
	fvhip_implicit_config conf;
};

/// TVDRKSolver (aodesolver.hpp: UnsteadySolver / TVDRKSolver; aodesolver.cpp:646-758) on the device:
/// constructed with the reference's (temporal order, physical CFL), solve(finaltime) advances d_u
class TVDRKSolver_HIP
{
public:
	TVDRKSolver_HIP(const FlowFV_HIP* s, int temporal_order, double cfl_num, int max_steps = 1 << 30)
		: spatial(s), order(temporal_order), cfl(cfl_num), maxsteps(max_steps) { }
	StatusCode solve(double* d_u, double finaltime) {
		check(fvhip_tvdrk_device(spatial->handle(), d_u, order, cfl, finaltime, maxsteps, &steps, &time));
		return 0;
	}
	int steps = 0;
	double time = 0;              ///< physical time reached
private:
	const FlowFV_HIP* spatial;
	int order;
	double cfl;
	int maxsteps;
};

/// Batched InviscidFlux::get_flux / get_jacobian on the device (anumericalflux.hpp:32-45)
class InviscidFlux_HIP
{
public:
	InviscidFlux_HIP(const std::string& name, double gamma, double Minf, double Tinf, double Reinf, double Pr)
		: type(fluxFromName(name)), gas{gamma, Minf, Tinf, Reinf, Pr} { }
	void get_flux(int nf, const double* ul, const double* ur, const double* n, double* flux) const {
		check(fvhip_local_flux(type, gas, nf, ul, ur, n, flux));
	}
	void get_jacobian(int nf, const double* ul, const double* ur, const double* n, double* dfdl,
	                  double* dfdr) const {
		check(fvhip_local_flux_jacobian(type, gas, nf, ul, ur, n, dfdl, dfdr));
	}
private:
	int type;
	double gas[5];
};

}
#endif
