/** \file orc_spatial.hpp
 * \brief ORACLE (test infrastructure only): CPU restatement of FVENS's spatial discretisation
 *   for one (unpartitioned) domain: gradients, reconstruction, residual, local time steps,
 *   Jacobian assembly and the matrix-free operator, in the reference's single-thread loop order.
 *
 * Restated (under /root/reference/src): flow_spatial.cpp:73-93, 348-395, 397-446, 488-875;
 * aspatial.cpp:172-340; agradientschemes.cpp:29-440; areconstruction.cpp:51-103;
 * musclreconstruction.cpp:24-130; limitedlinearreconstruction.cpp:27-268;
 * reconstruction_utils.hpp:17-47; viscousphysics.cpp:14-246; alinalg.cpp:142-233;
 * aodesolver.cpp:135-282, 300-329.
 *
 * Documented deviations (same in the product): Barth-Jespersen/Venkatakrishnan read
 * u(jel) for a physical-boundary neighbour jel = N+nc+iface past the end of the primitive array
 * (limitedlinearreconstruction.cpp:134-137, 229-232): here the ghost primitive state ug is used.
 * limiter_param is passed explicitly (the reference never parses it, controlparser.cpp:178-182).
 */
#ifndef ORC_SPATIAL_HPP
#define ORC_SPATIAL_HPP

#include "orc_physics.hpp"
#include "orc_mesh.hpp"
#include <vector>
#include <map>

namespace orc {

enum GradType { GRAD_ZERO = 0, GRAD_GREENGAUSS = 1, GRAD_LEASTSQUARES = 2 };
enum ReconType { REC_NONE = 0, REC_WENO = 1, REC_VANALBADA = 2, REC_BARTHJESPERSEN = 3,
                 REC_VENKATAKRISHNAN = 4 };

struct Config
{
	double gamma = 1.4, Minf = 0.5, Tinf = 298.0, Reinf = 1.0/0.0, Pr = 0.0/0.0, aoa = 0.0;
	bool viscous = false, constvisc = false, order2 = true;
	int flux = ROE, jacflux = ROE, grad = GRAD_LEASTSQUARES, recon = REC_VANALBADA;
	double limiter_param = 20.0;
	std::vector<BC> bcs;     // type, tag, vals
};

class Spatial
{
public:
	Spatial(const OMesh& m, const Config& c);

	/// FlowFV::compute_residual: ADDS -r(u) into res (nelem x 4); dtm (nelem) if gettimesteps
	void compute_residual(const double* u, double* res, bool gettimesteps, double* dtm) const;
	/// FlowFV_base::getGradients (flow_spatial.cpp:95-112): conserved-variable gradients
	void getGradients(const double* u, double* grads) const;
	/// gradient scheme on arbitrary cell/ghost values (nvars = 4), GradBlock layout [cell][var][dim]
	void compute_gradients(const double* u, const double* ug, double* grads) const;
	/// reconstruction on primitive arrays: writes ufl/ufr (naface x 4)
	void compute_face_values(const double* up, const double* ug, const double* grads,
	                         double* ufl, double* ufr) const;
	/// Spatial::assemble_jacobian into BSR blocks: diag[nelem][16], lower/upper per interior face
	/// (A[R][L] += L -> lower[iface-nbface], A[L][R] += U -> upper[iface-nbface]); values added
	void assemble_jacobian(const double* u, double* diag, double* lower, double* upper) const;
	/// MatrixFreeSpatialJacobian::apply with state u, res = -r(u), mdt = Vol/(CFL dt)
	void matfree_apply(const double* u, const double* res, const double* mdt, double eps,
	                   const double* x, double* y) const;
	/// local Jacobian blocks (flow_spatial.cpp:818-875), exposed for tests
	void local_jacobian_interior(int iface, const double* ul, const double* ur, double* L, double* U) const;
	void local_jacobian_boundary(int iface, const double* ul, double* L) const;

	const OMesh& m;
	Config cfg;
	Gas phy;
	Flux invf, jacf;
	std::array<double,NVARS> uinf;
	std::map<int,BC> bcmap;
	std::vector<double> V;         ///< WLS inverse normal matrices [nelem][2][2] (row-major)
	std::vector<double> clength;   ///< Venkatakrishnan characteristic length

	void boundary_state(int iface, const double* ins, double* gs) const;
	void compute_boundary_states(const double* ins, double* gs) const;
	void compute_fluxes(const double* u, const double* grads, const double* ul, const double* ur,
	                    const double* ug, double* res) const;
	void compute_max_timestep(const double* ul, const double* ur, double* dtm) const;
	void viscous_flux(const double* n, const double* rcl, const double* rcr, const double* ucl,
	                  const double* ucr, const double* gradsl, const double* gradsr,
	                  const double* ul, const double* ur, double* vflux) const;
	void viscous_flux_jacobian(int iface, const double* ul, const double* ur, double* dvfi, double* dvfj) const;
};

/// Explicit forward-Euler pseudo-time steady solve (aodesolver.cpp:135-282) on one domain.
/// Returns the number of steps taken; writes the final energy-residual norm ratio to *resratio.
int steady_forward_euler(const Spatial& s, double* u, double cfl, double tol, int maxiter,
                         double* resratio);

/// FlowFV::compute_residual on every rank of a partition (per-rank meshes from orc_restrict), with
/// the ghost-gradient and face-trace exchanges in between; u[r] has nelem+nconnface rows (ghost rows
/// filled as the driver's VecGhostUpdate leaves them)
void compute_residual_ranks(const std::vector<const Spatial*>& S, const std::vector<const double*>& u,
                            const std::vector<double*>& res, bool gettimesteps, const std::vector<double*>& dtm);

/// computeSurfaceData (flow_spatial.cpp:130-310): returns {CL, CDp, CDsf} on marker iwbcm
std::array<double,3> surface_functionals(const Spatial& s, const double* u, const double* grads, int iwbcm);

}
#endif
