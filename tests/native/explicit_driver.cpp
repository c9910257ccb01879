// Test driver: the reference's explicit pseudo-time loop (SteadyForwardEulerSolver::solve,
// aodesolver.cpp:170-240) written against the C++ host wrapper fvens_amd/host/flowfv_hip.hpp,
// i.e. exactly what a C++ caller of the drop-in sees. It generates a mesh with the library's mesh
// builder, takes `nsteps` forward-Euler steps and writes the final state (reference cell order)
// and the residual-norm history as raw doubles, for tests/test_gpu_driver.py to compare with the
// oracle's forward Euler.
// usage: explicit_driver <out.bin> <ntheta> <nquad> <ntri> <nsteps> <cfl> <fast 0|1>
#include "../../fvens_amd/host/flowfv_hip.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace fvens_hip;

int main(int argc, char** argv)
{
	if(argc < 8) { std::fprintf(stderr, "usage: %s out nt nq ntri nsteps cfl fast\n", argv[0]); return 2; }
	const int nt = std::atoi(argv[2]), nq = std::atoi(argv[3]), ntri = std::atoi(argv[4]);
	const int nsteps = std::atoi(argv[5]);
	const double cfl = std::atof(argv[6]);
	const bool fast = std::atoi(argv[7]) != 0;
	try {
		fvmesh_handle mh;
		check(fvmesh_generate(0, nt, nq, ntri, 20.0, 1e-4, 0.0, &mh));
		fvhip_mesh m;
		check(fvmesh_view(mh, &m));

		// testcases/naca0012/transonic-sanity-test-muscl.ctrl
		FlowPhysicsConfig pc;
		pc.gamma = 1.4; pc.Minf = 0.8; pc.Tinf = 298.0; pc.Reinf = INFINITY; pc.Pr = NAN;
		pc.aoa = 1.25*M_PI/180.0; pc.viscous_sim = false; pc.const_visc = false;
		pc.bcconf = {FlowBCConfig{2, SLIP_WALL_BC, {}, {}}, FlowBCConfig{4, FARFIELD_BC, {}, {}}};
		FlowNumericsConfig nc;
		nc.conv_numflux = "ROE"; nc.conv_numflux_jac = "ROE"; nc.gradientscheme = "LEASTSQUARES";
		nc.reconstruction = "VANALBADA"; nc.limiter_param = 20.0; nc.order2 = true; nc.fast_math = fast;
		FlowFV_HIP spatial(m, pc, nc);

		// free-stream initial condition (aphysics.cpp:43-58)
		const int N = m.nelem;
		std::vector<double> u(4*static_cast<size_t>(N)), r(u.size()), dtm(N);
		const double pinf = 1.0/(pc.gamma*pc.Minf*pc.Minf);
		for(int e = 0; e < N; e++) {
			u[4*e+0] = 1.0; u[4*e+1] = std::cos(pc.aoa); u[4*e+2] = std::sin(pc.aoa);
			u[4*e+3] = pinf/(pc.gamma-1.0) + 0.5*1.0*1.0;
		}
		std::vector<double> hist;
		for(int step = 0; step < nsteps; step++) {
			std::fill(r.begin(), r.end(), 0.0);
			spatial.compute_residual(u.data(), r.data(), true, dtm.data());
			for(int e = 0; e < N; e++)
				for(int i = 0; i < 4; i++)
					u[4*e+i] += cfl*dtm[e] * 1.0/m.area[e]*r[4*e+i];
			double locres = 0;
			for(int e = 0; e < N; e++) locres += r[4*e+3]*r[4*e+3]*m.area[e];
			hist.push_back(std::sqrt(locres));
		}
		FILE* f = std::fopen(argv[1], "wb");
		if(!f) { std::perror("fopen"); return 3; }
		std::fwrite(&N, sizeof(int), 1, f);
		std::fwrite(u.data(), sizeof(double), u.size(), f);
		std::fwrite(hist.data(), sizeof(double), hist.size(), f);
		std::fclose(f);
		check(fvmesh_destroy(mh));
		std::printf("ok %d cells, %d steps, residual %.6e -> %.6e\n", N, nsteps, hist.front(), hist.back());
	} catch(const std::exception& e) {
		std::fprintf(stderr, "error: %s\n", e.what());
		return 1;
	}
	return 0;
}
