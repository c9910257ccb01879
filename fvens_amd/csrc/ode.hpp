/** \file ode.hpp
 * \brief Device pseudo-time stepping helpers (ode.hip).
 */
#ifndef FVHIP_ODE_HPP
#define FVHIP_ODE_HPP

#include <hip/hip_runtime.h>

namespace fvhip {

/// u[e] += cfl*dtm[e] * 1.0/area[e] * r[e]   (aodesolver.cpp:204-214)
void launch_fe_update(int n, const double* r, const double* dtm, const double* area, double cfl, double* u, hipStream_t s);
/// out[0] = sqrt(sum_e r[e][3]^2 area[e])   (aodesolver.cpp:216-223), fixed reduction order
void launch_resnorm(int n, const double* r, const double* area, double* part, double* out, hipStream_t s);
int resnorm_partials();
/// us = c0*u + c1*us - (sc/area)*r per cell, sc = c2*dtmin*cfl (TVDRKSolver::solve, aodesolver.cpp:735-744)
void launch_tvdrk_stage(int n, double c0, double c1, double sc, const double* area, const double* r, const double* u,
                        double* us, hipStream_t s);
/// out[0] = min_e x[e] (part: resnorm_partials() doubles of scratch)
void launch_min(int n, const double* x, double* part, double* out, hipStream_t s);

}
#endif
