/** \file mesh.hpp
 * \brief Host-side mesh for the MI355X face sweep: Gmsh-2 ingest, the reference's face-indexing
 *   contract, geometry, synthetic generators and the locality ordering used on the device.
 *
 * Everything exported (cell, face and boundary-face indices, normals, lengths, areas, centres)
 * follows FVENS's UMesh contract bit for bit:
 *  - readGmsh2               /root/reference/src/mesh/meshreaders.cpp:66-265
 *  - correctBoundaryFaceOrientation  mesh.cpp:55-82
 *  - compute_faceConnectivity        mesh.cpp:659-762 (face order, ghost index rule mesh.hpp:84-96)
 *  - compute_face_data               mesh.cpp:346-365
 *  - compute_areas / cell centres    mesh.cpp:290-328
 *  - face centres, ghost centres     aspatial.cpp:50-61, 97-119
 * The topology is found with a per-node incidence scan (O(N)), not the reference's nested loops,
 * but the loop that NUMBERS faces is the reference's, so indices are identical.
 */
#ifndef FVHIP_MESH_HPP
#define FVHIP_MESH_HPP

#include <vector>
#include <string>
#include <cstdint>

namespace fvhip {

/// Raw mesh as read from a file or generated; mirrors fvens::MeshData (meshreaders.hpp)
struct MeshData
{
	int npoin = 0, nelem = 0, nbface = 0;
	int nnofa = 2;           ///< nodes per face (linear only)
	int nbtag = 0, ndtag = 0;
	int maxnnode = 0, maxnfael = 0;
	std::vector<double> coords;    ///< [npoin][2]
	std::vector<int> inpoel;       ///< [nelem][maxnnode], -1 padded
	std::vector<int> nnode, nfael; ///< [nelem]
	std::vector<int> bface;        ///< [nbface][nnofa+nbtag]: nodes then tags
	std::vector<int> vol_regions;  ///< [nelem][ndtag]
};

/// A single-domain mesh with the reference's connectivity and geometry.
struct Mesh
{
	MeshData md;
	int naface = 0, ninface = 0, nconnface = 0;
	std::vector<int> esuel;        ///< [nelem][maxnfael]
	std::vector<int> elemface;     ///< [nelem][maxnfael]
	std::vector<int> intfac;       ///< [naface][4] = {L, R, node0, node1}
	std::vector<int> btags;        ///< [nbface][nbtag]
	std::vector<double> facemetric;///< [naface][3] = {nx, ny, len}
	std::vector<double> area;      ///< [nelem]
	std::vector<double> rc;        ///< [nelem+nconnface][2] cell centres (vertex average)
	std::vector<double> gr;        ///< [naface][2] face centres
	std::vector<double> rcbp;      ///< [nbface][2] ghost cell centres about face midpoints
	// one rank's subdomain (restrictMesh): connectivity faces and the global cell of each local cell
	std::vector<int> connface;     ///< [nconnface][5] = {cell, local face, owner rank of the neighbour,
	                               ///<  global neighbour cell, global face} (mesh.hpp:60-70)
	std::vector<int> globalElemIndex; ///< [nelem] (empty on a single domain)
};

/// Reads a Gmsh 2.2 ASCII mesh exactly as readGmsh2 does (boundary edges must precede cells).
MeshData readGmsh2(const std::string& path);

/// Writes a MeshData in Gmsh 2.2 ASCII format (boundary edges first, as readGmsh2 expects).
void writeGmsh2(const MeshData& m, const std::string& path);

/// Full reference preprocessing for one rank: orientation fix, topology, areas, face data,
/// centres. (constructMesh ameshutils.cpp:102-153 with a trivial 1-rank partition)
Mesh buildMesh(MeshData md);

/// preprocessMesh's topology + geometry for one rank's mesh whose connectivity faces are given
/// (connface [nconnface][5]); ghost-row centres rc[nelem..] are left zero for the caller to fill
void buildTopology(MeshData md, Mesh& M, const std::vector<int>& connface);

/// TrivialReplicatedGlobalMeshPartitioner::compute_partition (meshpartitioning.cpp:354-367):
/// nelem/nranks cells per rank in index order, the remainder to the last rank
std::vector<int> partitionTrivial(int nelem, int nranks);

/// ReplicatedGlobalMeshPartitioner::restrictMeshToPartitions (meshpartitioning.cpp:24-159) followed
/// by preprocessMesh (ameshutils.cpp:40-99): rank `rank`'s subdomain of the (preprocessed) global
/// mesh gm under the cell distribution elemdist, with its connectivity faces; the ghost rows of rc
/// hold the centres of the neighbouring cells (what the Spatial ctor's ghost scatter puts there)
Mesh restrictMesh(const Mesh& gm, const int* elemdist, int rank);

/// Synthetic hybrid O-grid around a NACA 0012 aerofoil (chord 1, LE at origin).
/// ntheta points around the surface, nquad quad layers at the wall, ntri triangle-split layers
/// outside them, outer circle radius rfar about (0.5,0). Wall marker 2, farfield marker 4.
/// Cells: ntheta*(nquad + 2*ntri).
MeshData generateNacaOgrid(int ntheta, int nquad, int ntri, double rfar, double wallspacing, int farmap = 0);
MeshData generateNacaCgrid(int nsurf, int nwake, int nquad, int ntri, double rfar, double wallspacing);
/// Hybrid mesh of the reference's visc-naca0012 topology (naca0012nasa-blcirc.geo: a quadrangle block
/// round the body, triangles outside it): generateNacaCgrid's points with nrows rows; quadrangles in the
/// body's first nquad rows (the boundary layer) and in the two wake blocks, near-isotropic triangles above
/// the body's quadrangles: each row there resampled to its distance from the row below (over 0.87, the
/// equilateral triangle's height), within a factor 1.25 of the row below's spacing, and zipped to it.
MeshData generateNacaHybrid(int nsurf, int nwake, int nquad, int nrows, double rfar, double wallspacing);

/// Synthetic O-grid annulus about a cylinder of radius r0 out to r1, all quads split into
/// triangles (2dcylinder-like). Inner marker 2, outer marker 4. Cells 2*ntheta*nr.
MeshData generateCylinderOgrid(int ntheta, int nr, double r0, double r1);

/// Structured flat-plate channel of nx*ny quads on [-xlead, 1]x[0, h] with wall clustering.
/// Markers: 3 = symmetry (slipwall, y=0 x<0), 2 = plate (adiabatic wall, y=0 x>=0),
/// 4 = top farfield, 5 = inflow/outflow (left and right).
MeshData generateFlatPlate(int nx, int ny, double xlead, double h, double wallspacing);

}

#endif
