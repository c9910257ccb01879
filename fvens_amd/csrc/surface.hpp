/** \file surface.hpp
 * \brief Launch interface of the surface-functional kernels (surface.hip).
 */
#ifndef FVHIP_SURFACE_HPP
#define FVHIP_SURFACE_HPP

#include "kernels.hpp"

namespace fvhip {

/// the boundary faces of one marker, in reference face order
struct SurfaceFaces
{
	int n;
	const int* L;          ///< [n] internal id of the face's cell
	const double* geo;     ///< [n][5]: nx, ny, length, face centre x, y
};

/// faceout [n][4] = (x, y, Cp, Cf); contrib [n][4] scratch; sums[4] = (Cl, Cdp, Cdf, total length)
/// before normalisation (flow_spatial.cpp:130-310)
void launch_surface(const SurfaceFaces& S, const double* u, const double* grad, const gd::Gas& G, double pinf,
                    double wx, double wy, double* faceout, double* contrib, double* sums, hipStream_t s);

/// sum over the owned cells of ((s - sinf)/sinf)^2 area into out[0] (FlowOutput::compute_entropy_cell
/// before the rank sum and the square root); part has entropy_partials(N) entries
int entropy_partials(int N);
void launch_entropy(int N, const double* u, const double* area, const gd::Gas& G, double sinf, double* part,
                    double* out, hipStream_t s);

}
#endif
