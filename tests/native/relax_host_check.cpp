// Host build of the device nonlinear-update source (fvens_amd/csrc/krylov.hpp relaxation_factor)
// for tests/test_krylov_host.py, which compares it with the restatement in tests/_oracle.py.
#include "../../fvens_amd/csrc/krylov.hpp"

extern "C" void relaxed_update_host(int n, double gamma, double minfactor, const double* du, const double* u,
                                    double* out)
{
	const fvhip::gd::Gas G = fvhip::gd::make_gas(gamma, 0.8, 298.0, 1e300, 0.72);
	for(int c = 0; c < n; c++) {
		const double om = fvhip::relaxation_factor(G, minfactor, du + 4*c, u + 4*c);
		for(int i = 0; i < 4; i++) out[4*c+i] = u[4*c+i] + om*du[4*c+i];
	}
}
