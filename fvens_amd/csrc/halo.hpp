/** \file halo.hpp
 * \brief Device helpers of the ghost-cell exchange (halo.hip).
 */
#ifndef FVHIP_HALO_HPP
#define FVHIP_HALO_HPP

#include <hip/hip_runtime.h>
#include "gasdyn.hpp"

namespace fvhip {

/// dst[i*width + k] = src[idx[i]*width + k] for i < n (rows of owned cells a neighbour needs)
void launch_pack_rows(const int* idx, int n, const double* src, int width, double* dst, hipStream_t s);
/// dst[idx[r]][k] = src[r][k] (the inverse of launch_pack_rows)
void launch_unpack_rows(const int* idx, int n, const double* src, int width, double* dst, hipStream_t s);
/// primitive state of rows [first, first+count) (ghost cells), same arithmetic as k_prep_cells
void launch_cons2prim_rows(const gd::Gas& G, const double* u, double* up, int first, int count, hipStream_t s);

}
#endif
