/** \file partition.hpp
 * \brief Cell partitioning and per-rank local meshes with one ghost-cell layer.
 *
 * Replaces, for the hot path, the reference's partitioned-mesh construction
 * (mesh/meshpartitioning.cpp:24-159, Scotch graph partition :376-458) with:
 *  - recursive coordinate bisection of cell centres (Scotch is not available in this image; the
 *    reference's own default is a trivial block partition, ameshutils.cpp:122-123);
 *  - a local topology per rank: owned cells, one layer of ghost cells (grouped by owner rank,
 *    ascending global id), and every global face touching an owned cell in ascending GLOBAL face
 *    index with its GLOBAL orientation. Unlike the reference's connectivity faces (local outward
 *    normal, faces appended last), this makes each owned cell's residual the same sequence of
 *    floating-point operations as on one GPU, so the N-GPU residual is bitwise the 1-GPU one.
 */
#ifndef FVHIP_PARTITION_HPP
#define FVHIP_PARTITION_HPP

#include <vector>
#include "../../include/fvhip.h"

namespace fvhip {

/// Mesh topology in the form the layout builder consumes. Cells [0,nown) are owned, [nown,ncell)
/// ghosts; a face's R >= ncell denotes physical boundary face R - ncell. Faces are sorted by global
/// index, physical boundary faces first.
struct MeshTopo
{
	int nown = 0, nghost = 0, nbface = 0, naface = 0;
	int ncell() const { return nown + nghost; }
	std::vector<int> cell_global;      ///< [ncell]
	std::vector<int> nfael;            ///< [nown]
	std::vector<int> cell_faces;       ///< [nown][4] local faces in the cell's own (elemface) order
	std::vector<int> cell_esuel;       ///< [nown][4] neighbour across each: local cell or ncell+bface
	std::vector<double> rc;            ///< [ncell][2]
	std::vector<double> area;          ///< [nown]
	std::vector<double> clength;       ///< [nown] longest edge (Venkatakrishnan), as the reference computes it
	std::vector<int> face_global;      ///< [naface]
	std::vector<int> L, R;             ///< [naface]
	std::vector<double> facemetric;    ///< [naface][3]
	std::vector<double> gr;            ///< [naface][2]
	std::vector<int> btag;             ///< [nbface]
	std::vector<double> rcbp;          ///< [nbface][2]
	// halo
	std::vector<int> nbr_rank;         ///< neighbour ranks, ascending
	std::vector<int> ghost_start;      ///< [nnbr+1] ghosts owned by nbr_rank[k] are local cells
	                                   ///<  nown+ghost_start[k] .. nown+ghost_start[k+1]-1
	std::vector<int> send_start;       ///< [nnbr+1] ranges into send_cells
	std::vector<int> send_cells;       ///< local owned cells each neighbour holds as ghosts (ascending global id)
	std::vector<int> ghost_row;        ///< [nghost] per-rank meshes: reference row (nelem+icface) of each ghost
	// two-layer halo (extractPartition): each neighbour's ghost block and send block hold its layer-1
	// cells (across a face of an owned cell) first, then its layer-2 cells (across a face of a layer-1
	// ghost); one exchange of u fills both, and the layer-1 ghosts' gradients are then computed
	// locally from the g1_* lists instead of being exchanged
	int halo_layers = 1;
	std::vector<int> ghost_l1_end;     ///< [nnbr] end of neighbour k's layer-1 ghosts (same base as ghost_start)
	std::vector<int> send_l1_end;      ///< [nnbr] end of neighbour k's layer-1 sends (same base as send_start)
	std::vector<int> g1_cells;         ///< local ids of the layer-1 ghosts
	std::vector<int> g1_nbr;           ///< [n1][4] their neighbours in ascending GLOBAL face order: local
	                                   ///<  cell, -2-j (extra boundary face j), -1 none
	std::vector<double> g1_gr;         ///< [n1][4][2] centres of those faces (same order; 0 padding), for
	                                   ///<  the layer-1 ghosts' limiter values (limited reconstructions)
	std::vector<double> g1_clength;    ///< [n1] their longest edges (Venkatakrishnan's eps)
	std::vector<int> xb_btag;         ///< extra boundary faces (touching a layer-1 ghost only): marker,
	std::vector<double> xb_n;          ///<  unit normal [2] (facemetric),
	std::vector<double> xb_rcbp;       ///<  ghost-cell centre [2]
};

/// Whole mesh as one rank (no ghosts)
MeshTopo topoFromMesh(const fvhip_mesh& m);

/// One rank's subdomain as the reference's multi-rank driver holds it (restrictMeshToPartitions,
/// meshpartitioning.cpp:24-159): mesh.connface [nconnface][5] lists its connectivity faces, which
/// come last in face order with the local outward normal and R = nelem + icface (mesh.cpp:744-757).
/// Each connectivity face gets a ghost cell of its own (the reference's ghost row nelem+icface),
/// grouped by neighbour rank and ordered by GLOBAL face index (connface(.,4)) within a rank; each
/// rank sends the rows of its connectivity-face cells in that same order, so both sides of every
/// exchange agree without the index handshake of L2TraceVector::update_comm_pattern
/// (tracevector.cpp:31-184). The result is the reference's per-rank residual: faces, orientation
/// and accumulation order are the subdomain's own.
MeshTopo topoFromRankMesh(const fvhip_mesh& m);

/// Rank `rank`'s piece of a single-domain mesh partitioned by `part` (part[cell] in [0,nparts)),
/// with a two-layer halo (layers = 2, the default) or the one-layer halo of round 1 (layers = 1)
MeshTopo extractPartition(const fvhip_mesh& m, const int* part, int rank, int layers = 2);

/// Recursive coordinate bisection of cell centres into nparts parts with sizes differing by at
/// most one cell per bisection level; deterministic (ties broken by cell index)
std::vector<int> partitionRCB(const double* rc, int ncell, int nparts);
/// the reference's line finder for its line orderings (mesh/meshordering.cpp:143-264, computeWeights +
/// findLines): lines of cells (reference numbering) in discovery order, each of at least two cells
std::vector<std::vector<int>> findLinesReference(const fvhip_mesh& m, double threshold);

/// Graph partition of the cell dual graph (the reference's Scotch SCOTCH_graphPart on the same graph,
/// meshpartitioning.cpp:376-458; Scotch is absent from the image): recursive bisection, each grown
/// breadth-first from a pseudo-peripheral cell and refined by balanced Kernighan-Lin boundary swaps.
/// Part sizes as RCB's (exact split per level); deterministic. weight (optional, [nelem], 1..4096):
/// cell weights -- each bisection then splits the weight instead of the cell count, to within the
/// largest weight (the hot path's cost per cell grows with its face count: weight = nfael balances the
/// fused residual's time across ranks of a mixed triangle/quad mesh)
std::vector<int> partitionGraph(const fvhip_mesh& m, int nparts, const int* weight = nullptr);

/// interior faces whose two cells lie in different parts
long long edgeCut(const fvhip_mesh& m, const int* part);

}
#endif
