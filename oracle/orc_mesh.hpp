/** \file orc_mesh.hpp
 * \brief ORACLE (test infrastructure only): literal CPU restatement of FVENS's mesh ingest and
 *   face-indexing contract, used to check the product mesh builder index-for-index.
 *
 * Restated: meshreaders.cpp:66-265 (readGmsh2), mesh.cpp:55-82 (boundary orientation),
 * mesh.cpp:290-328 (areas, centres), mesh.cpp:346-365 (face metric), mesh.cpp:425-541 (esup,
 * esuel, with the reference's nested searches), mesh.cpp:560-762 (face connectivity),
 * aspatial.cpp:50-61 and 97-119 (face centres, ghost centres), meshpartitioning.cpp:24-159 and
 * 354-367 (subdomain restriction, trivial partition).
 */
#ifndef ORC_MESH_HPP
#define ORC_MESH_HPP

#include <vector>
#include <string>

namespace orc {

struct OMesh
{
	int npoin = 0, nelem = 0, nbface = 0, nnofa = 2, nbtag = 0, ndtag = 0, maxnnode = 0, maxnfael = 0;
	int naface = 0, ninface = 0, nconnface = 0;
	std::vector<double> coords;        // [npoin][2]
	std::vector<int> inpoel;           // [nelem][maxnnode]
	std::vector<int> nnode, nfael;
	std::vector<int> bface;            // [nbface][nnofa+nbtag]
	std::vector<int> esup_p, esup;
	std::vector<int> esuel, elemface;  // [nelem][maxnfael]
	std::vector<int> intfac;           // [naface][4]
	std::vector<int> btags;            // [nbface][nbtag]
	std::vector<double> facemetric;    // [naface][3]
	std::vector<double> area;          // [nelem]
	std::vector<double> rc;            // [nelem+nconnface][2]
	std::vector<double> gr;            // [naface][2]
	std::vector<double> rcbp;          // [nbface][2]
	std::vector<int> connface;         // [nconnface][5] (mesh.hpp:60-70), per-rank meshes
	std::vector<int> globalElemIndex;  // [nelem], per-rank meshes

	int in(int e, int j) const { return inpoel[static_cast<size_t>(e)*maxnnode+j]; }
	int gesuel(int e, int j) const { return esuel[static_cast<size_t>(e)*maxnfael+j]; }
	int gelemface(int e, int j) const { return elemface[static_cast<size_t>(e)*maxnfael+j]; }
	int L(int f) const { return intfac[4*f]; }
	int Rt(int f) const { return intfac[4*f+1]; }
	double nx(int f) const { return facemetric[3*f]; }
	double ny(int f) const { return facemetric[3*f+1]; }
	double len(int f) const { return facemetric[3*f+2]; }
	int btag(int f) const { return btags[static_cast<size_t>(f)*nbtag]; }
	int gconnface(int ic, int k) const { return connface[5*static_cast<size_t>(ic)+k]; }
};

/// readGmsh2 restated with std::ifstream >> like the reference
OMesh orc_readGmsh2(const std::string& file);
/// Builds an OMesh from raw arrays (as the product generator produces them)
OMesh orc_fromRaw(int npoin, const double* coords, int nelem, int maxnnode, const int* inpoel,
                  const int* nnode, int nbface, int nbtag, const int* bface);
/// correctBoundaryFaceOrientation + compute_topological + areas + face data + centres
void orc_preprocess(OMesh& m);
/// preprocessMesh of one rank's mesh (compute_topological with m.connface, areas, face data, centres;
/// ghost-row centres left zero)
void orc_preprocess_rank(OMesh& m);
/// TrivialReplicatedGlobalMeshPartitioner::compute_partition (meshpartitioning.cpp:354-367)
std::vector<int> orc_partition_trivial(int nelem, int nranks);
/// restrictMeshToPartitions (meshpartitioning.cpp:24-159) + preprocessMesh of a preprocessed global mesh
OMesh orc_restrict(const OMesh& gm, const std::vector<int>& elemdist, int rank);

}
#endif
