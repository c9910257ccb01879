/** \file mesh.cpp
 * \brief Host mesh ingest, the reference face-indexing contract, geometry and generators.
 * See mesh.hpp for the reference lines each routine reproduces.
 */
#include "mesh.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <algorithm>
#include <numeric>

namespace fvhip {

// ------------------------------------------------------------------------------------------------
// Gmsh 2.2 ASCII (meshreaders.cpp:66-265)
// ------------------------------------------------------------------------------------------------

namespace {

/// Minimal fast tokenizer over a whole file; numbers parsed with strtol/strtod, which is what
/// std::istream's num_get reduces to, so coordinates round identically to the reference reader.
struct Tok
{
	std::vector<char> buf;
	size_t pos = 0;
	explicit Tok(const std::string& path) {
		std::ifstream f(path, std::ios::binary);
		if(!f) throw std::runtime_error("readGmsh2: cannot open " + path);
		f.seekg(0, std::ios::end);
		const size_t n = static_cast<size_t>(f.tellg());
		f.seekg(0);
		buf.resize(n+1);
		f.read(buf.data(), static_cast<std::streamsize>(n));
		buf[n] = '\0';
	}
	void skipLine() {
		while(pos < buf.size() && buf[pos] != '\n') pos++;
		if(pos < buf.size()) pos++;
	}
	void skipWs() { while(buf[pos] && isspace(static_cast<unsigned char>(buf[pos]))) pos++; }
	long getInt() {
		skipWs(); char* e; const long v = strtol(&buf[pos], &e, 10);
		if(e == &buf[pos]) throw std::runtime_error("readGmsh2: expected integer");
		pos = static_cast<size_t>(e - buf.data()); return v;
	}
	double getDouble() {
		skipWs(); char* e; const double v = strtod(&buf[pos], &e);
		if(e == &buf[pos]) throw std::runtime_error("readGmsh2: expected real");
		pos = static_cast<size_t>(e - buf.data()); return v;
	}
	std::string getWord() {
		skipWs(); const size_t s = pos;
		while(buf[pos] && !isspace(static_cast<unsigned char>(buf[pos]))) pos++;
		return std::string(&buf[s], pos-s);
	}
};

}

MeshData readGmsh2(const std::string& path)
{
	Tok t(path);
	MeshData m;
	for(int i = 0; i < 4; i++) t.skipLine();           // meshreaders.cpp:74-77

	m.npoin = static_cast<int>(t.getInt());
	m.coords.resize(static_cast<size_t>(m.npoin)*2);
	for(int i = 0; i < m.npoin; i++) {
		t.getInt();
		m.coords[2*i] = t.getDouble();
		m.coords[2*i+1] = t.getDouble();
		t.getDouble();                                  // z dropped (NDIM < 3)
	}
	t.getWord(); t.getWord();                           // $EndNodes $Elements

	const int nelm = static_cast<int>(t.getInt());
	constexpr int width = 25;
	std::vector<int> elms(static_cast<size_t>(nelm)*width, 0);
	std::vector<int> nnodes(nelm, 0), nfaels(nelm, 0);
	m.ndtag = 0; m.nbtag = 0; m.nbface = 0; m.nelem = 0;
	for(int i = 0; i < nelm; i++)
	{
		int* e = &elms[static_cast<size_t>(i)*width];
		t.getInt();
		const int type = static_cast<int>(t.getInt());
		int nn = 0, nfa = 0; bool isface = false;
		switch(type) {
			case 1: m.nnofa = 2; isface = true; break;
			case 8: m.nnofa = 3; isface = true; break;
			case 2: nn = 3; nfa = 3; m.nnofa = 2; break;
			case 3: nn = 4; nfa = 4; m.nnofa = 2; break;
			case 9: nn = 6; nfa = 3; m.nnofa = 3; break;
			case 16: nn = 8; nfa = 4; m.nnofa = 3; break;
			case 10: nn = 9; nfa = 4; m.nnofa = 3; break;
			default: nn = 3; nfa = 3; m.nnofa = 2;       // meshreaders.cpp:197-209
		}
		const int ntags = static_cast<int>(t.getInt());
		if(isface) {
			if(ntags > m.nbtag) m.nbtag = ntags;
			for(int j = 0; j < ntags; j++) e[j+m.nnofa] = static_cast<int>(t.getInt());
			for(int j = 0; j < m.nnofa; j++) e[j] = static_cast<int>(t.getInt());
			m.nbface++;
		} else {
			nnodes[i] = nn; nfaels[i] = nfa;
			if(ntags > m.ndtag) m.ndtag = ntags;
			for(int j = 0; j < ntags; j++) e[j+nn] = static_cast<int>(t.getInt());
			for(int j = 0; j < nn; j++) e[j] = static_cast<int>(t.getInt());
			m.nelem++;
		}
	}
	if(m.nnofa != 2)
		throw std::runtime_error("readGmsh2: only linear meshes are supported by the device path");

	m.maxnnode = nnodes[m.nbface]; m.maxnfael = nfaels[m.nbface];   // meshreaders.cpp:218-226
	for(int i = 0; i < nelm; i++) {
		m.maxnnode = std::max(m.maxnnode, nnodes[i]);
		m.maxnfael = std::max(m.maxnfael, nfaels[i]);
	}

	const int bw = m.nnofa + m.nbtag;
	m.bface.assign(static_cast<size_t>(m.nbface)*bw, 0);
	for(int i = 0; i < m.nbface; i++) {
		const int* e = &elms[static_cast<size_t>(i)*width];
		for(int j = 0; j < m.nnofa; j++) m.bface[i*bw+j] = e[j]-1;
		for(int j = m.nnofa; j < bw; j++) m.bface[i*bw+j] = e[j];
	}
	m.inpoel.assign(static_cast<size_t>(m.nelem)*m.maxnnode, -1);
	m.vol_regions.assign(static_cast<size_t>(m.nelem)*m.ndtag, 0);
	m.nnode.resize(m.nelem); m.nfael.resize(m.nelem);
	for(int i = 0; i < m.nelem; i++) {
		const int k = i + m.nbface;
		const int* e = &elms[static_cast<size_t>(k)*width];
		for(int j = 0; j < nnodes[k]; j++) m.inpoel[static_cast<size_t>(i)*m.maxnnode+j] = e[j]-1;
		for(int j = 0; j < m.ndtag; j++) m.vol_regions[static_cast<size_t>(i)*m.ndtag+j] = e[j+nnodes[k]];
		m.nnode[i] = nnodes[k]; m.nfael[i] = nfaels[k];
	}
	return m;
}

void writeGmsh2(const MeshData& m, const std::string& path)
{
	FILE* f = fopen(path.c_str(), "w");
	if(!f) throw std::runtime_error("writeGmsh2: cannot open " + path);
	fprintf(f, "$MeshFormat\n2.2 0 8\n$EndMeshFormat\n$Nodes\n%d\n", m.npoin);
	for(int i = 0; i < m.npoin; i++)
		fprintf(f, "%d %.17g %.17g 0\n", i+1, m.coords[2*i], m.coords[2*i+1]);
	fprintf(f, "$EndNodes\n$Elements\n%d\n", m.nbface + m.nelem);
	const int bw = m.nnofa + m.nbtag;
	int id = 1;
	for(int i = 0; i < m.nbface; i++) {
		fprintf(f, "%d 1 %d", id++, m.nbtag);
		for(int j = 0; j < m.nbtag; j++) fprintf(f, " %d", m.bface[i*bw+m.nnofa+j]);
		for(int j = 0; j < m.nnofa; j++) fprintf(f, " %d", m.bface[i*bw+j]+1);
		fprintf(f, "\n");
	}
	for(int i = 0; i < m.nelem; i++) {
		fprintf(f, "%d %d %d", id++, m.nnode[i] == 3 ? 2 : 3, m.ndtag);
		for(int j = 0; j < m.ndtag; j++) fprintf(f, " %d", m.vol_regions[static_cast<size_t>(i)*m.ndtag+j]);
		for(int j = 0; j < m.nnode[i]; j++) fprintf(f, " %d", m.inpoel[static_cast<size_t>(i)*m.maxnnode+j]+1);
		fprintf(f, "\n");
	}
	fprintf(f, "$EndElements\n");
	fclose(f);
}

// ------------------------------------------------------------------------------------------------
// Topology
// ------------------------------------------------------------------------------------------------

namespace {

/// CSR elements-surrounding-points (mesh.cpp:425-465); elements listed in increasing order.
void buildEsup(const MeshData& m, std::vector<int>& esup_p, std::vector<int>& esup)
{
	esup_p.assign(m.npoin+1, 0);
	for(int i = 0; i < m.nelem; i++)
		for(int j = 0; j < m.nnode[i]; j++)
			esup_p[m.inpoel[static_cast<size_t>(i)*m.maxnnode+j]+1]++;
	for(int i = 1; i <= m.npoin; i++) esup_p[i] += esup_p[i-1];
	esup.resize(esup_p[m.npoin]);
	std::vector<int> fill(esup_p.begin(), esup_p.end()-1);
	for(int i = 0; i < m.nelem; i++)
		for(int j = 0; j < m.nnode[i]; j++)
			esup[fill[m.inpoel[static_cast<size_t>(i)*m.maxnnode+j]]++] = i;
}

inline int nodeOf(const MeshData& m, int iel, int j) {
	return m.inpoel[static_cast<size_t>(iel)*m.maxnnode + j];
}

/// Local face of element iel whose node set is {a,b}; -1 if none. (getFaceEIndex, mesh.cpp:560)
inline int faceWithNodes(const MeshData& m, int iel, int a, int b)
{
	const int nn = m.nnode[iel];
	for(int f = 0; f < m.nfael[iel]; f++) {
		const int p = nodeOf(m, iel, f % nn), q = nodeOf(m, iel, (f+1) % nn);
		if((p == a && q == b) || (p == b && q == a)) return f;
	}
	return -1;
}

/// Host element and local face of each boundary face (compute_phyBFaceNeighboringElements,
/// mesh.cpp:608-657): the unique element containing both nodes.
void bfaceHosts(const MeshData& m, const std::vector<int>& esup_p, const std::vector<int>& esup,
                std::vector<int>& helem, std::vector<int>& hface)
{
	const int bw = m.nnofa + m.nbtag;
	helem.assign(m.nbface, -1); hface.assign(m.nbface, -1);
	for(int i = 0; i < m.nbface; i++) {
		const int a = m.bface[i*bw], b = m.bface[i*bw+1];
		int found = 0;
		for(int k = esup_p[a]; k < esup_p[a+1]; k++) {
			const int e = esup[k];
			bool hasb = false;
			for(int j = 0; j < m.nnode[e]; j++) if(nodeOf(m,e,j) == b) hasb = true;
			if(hasb) {
				if(found) throw std::logic_error("More than one neighboring element found for bface "
				                                 + std::to_string(i));
				helem[i] = e; found = 1;
			}
		}
		if(!found) throw std::logic_error("No host element for bface " + std::to_string(i));
		hface[i] = faceWithNodes(m, helem[i], a, b);
		if(hface[i] < 0) throw std::logic_error("bface is not an element face");
	}
}

/// Drops points not referenced by any cell, keeping the sorted order, exactly as the 1-rank
/// restriction does (meshpartitioning.cpp:185-222, 36-66).
void compactPoints(MeshData& m)
{
	std::vector<char> used(m.npoin, 0);
	for(int i = 0; i < m.nelem; i++)
		for(int j = 0; j < m.nnode[i]; j++) used[nodeOf(m,i,j)] = 1;
	std::vector<int> g2l(m.npoin, -1);
	int n = 0;
	for(int p = 0; p < m.npoin; p++) if(used[p]) g2l[p] = n++;
	if(n == m.npoin) return;
	std::vector<double> c(static_cast<size_t>(n)*2);
	for(int p = 0; p < m.npoin; p++)
		if(used[p]) { c[2*g2l[p]] = m.coords[2*p]; c[2*g2l[p]+1] = m.coords[2*p+1]; }
	m.coords.swap(c);
	for(auto& v : m.inpoel) if(v >= 0) v = g2l[v];
	const int bw = m.nnofa + m.nbtag;
	for(int i = 0; i < m.nbface; i++)
		for(int j = 0; j < m.nnofa; j++) m.bface[i*bw+j] = g2l[m.bface[i*bw+j]];
	m.npoin = n;
}

}

Mesh buildMesh(MeshData md)
{
	if(md.nnofa != 2) throw std::runtime_error("buildMesh: linear 2D meshes only");
	Mesh M;
	std::vector<int> esup_p, esup, helem, hface;

	// correctBoundaryFaceOrientation (mesh.cpp:55-82)
	buildEsup(md, esup_p, esup);
	bfaceHosts(md, esup_p, esup, helem, hface);
	const int bw = md.nnofa + md.nbtag;
	for(int i = 0; i < md.nbface; i++) {
		const int e = helem[i], f = hface[i], nn = md.nnode[e];
		if(nodeOf(md,e,(f+0)%nn) != md.bface[i*bw] || nodeOf(md,e,(f+1)%nn) != md.bface[i*bw+1])
			std::swap(md.bface[i*bw], md.bface[i*bw+1]);
	}

	// 1-rank restriction (drops unused points) then preprocessMesh's compute_topological
	compactPoints(md);
	buildTopology(std::move(md), M, std::vector<int>());
	return M;
}

namespace {

/// compute_elementsSurroundingElements (mesh.cpp:467-541): neighbour across each local face, -1 if none
std::vector<int> esuelOf(const MeshData& md, const std::vector<int>& esup_p, const std::vector<int>& esup)
{
	const int N = md.nelem, mf = md.maxnfael;
	std::vector<int> esuel(static_cast<size_t>(N)*mf, -1);
	for(int ie = 0; ie < N; ie++) {
		const int nn = md.nnode[ie];
		for(int f = 0; f < md.nfael[ie]; f++) {
			const int a = nodeOf(md,ie,f%nn), b = nodeOf(md,ie,(f+1)%nn);
			for(int k = esup_p[a]; k < esup_p[a+1]; k++) {
				const int je = esup[k];
				if(je == ie) continue;
				const int jf = faceWithNodes(md, je, a, b);
				if(jf >= 0) {
					esuel[static_cast<size_t>(ie)*mf+f] = je;
					esuel[static_cast<size_t>(je)*mf+jf] = ie;
				}
			}
		}
	}
	return esuel;
}

}

/// preprocessMesh's compute_topological + compute_areas + compute_face_data (ameshutils.cpp:40-99,
/// mesh.cpp:290-365, 659-762) and the Spatial ctor's centres (aspatial.cpp:36-119) for one rank's mesh;
/// connface [nconnface][5] as the restriction set it (empty on a single domain)
void buildTopology(MeshData md, Mesh& M, const std::vector<int>& connface)
{
	std::vector<int> esup_p, esup, helem, hface;
	const int bw = md.nnofa + md.nbtag;
	buildEsup(md, esup_p, esup);

	const int N = md.nelem, mf = md.maxnfael;
	M.esuel = esuelOf(md, esup_p, esup);

	// compute_faceConnectivity (mesh.cpp:659-762): physical boundary faces, subdomain interior faces,
	// then the connectivity faces in connface order (none on a single domain)
	M.nconnface = static_cast<int>(connface.size()/5);
	M.connface = connface;
	int ninface = 0;
	for(int ie = 0; ie < N; ie++)
		for(int in = 0; in < md.nfael[ie]; in++) {
			const int je = M.esuel[static_cast<size_t>(ie)*mf+in];
			if(je > ie && je < N) ninface++;
		}
	M.ninface = ninface;
	M.naface = ninface + md.nbface + M.nconnface;
	M.intfac.assign(static_cast<size_t>(M.naface)*4, -1);
	M.elemface.assign(static_cast<size_t>(N)*mf, -1);
	M.btags.assign(static_cast<size_t>(md.nbface)*md.nbtag, 0);

	bfaceHosts(md, esup_p, esup, helem, hface);
	for(int i = 0; i < md.nbface; i++) {
		M.intfac[4*i+0] = helem[i];
		M.intfac[4*i+1] = N + M.nconnface + i;
		M.intfac[4*i+2] = md.bface[i*bw];
		M.intfac[4*i+3] = md.bface[i*bw+1];
		for(int j = 0; j < md.nbtag; j++) M.btags[i*md.nbtag+j] = md.bface[i*bw+md.nnofa+j];
		M.esuel[static_cast<size_t>(helem[i])*mf+hface[i]] = N + M.nconnface + i;
		M.elemface[static_cast<size_t>(helem[i])*mf+hface[i]] = i;
	}
	int fi = md.nbface;
	for(int ie = 0; ie < N; ie++) {
		const int nn = md.nnode[ie];
		for(int in = 0; in < nn; in++) {
			const int je = M.esuel[static_cast<size_t>(ie)*mf+in];
			if(je > ie && je < N) {
				const int in1 = (in+1) % nn;
				M.intfac[4*fi+0] = ie; M.intfac[4*fi+1] = je;
				M.intfac[4*fi+2] = nodeOf(md,ie,in); M.intfac[4*fi+3] = nodeOf(md,ie,in1);
				M.elemface[static_cast<size_t>(ie)*mf+in] = fi;
				for(int jn = 0; jn < md.nnode[je]; jn++)
					if(nodeOf(md,ie,in1) == nodeOf(md,je,jn))
						M.elemface[static_cast<size_t>(je)*mf+jn] = fi;
				fi++;
			}
		}
	}
	if(fi != md.nbface + ninface) throw std::logic_error("buildMesh: face count mismatch");
	// connectivity faces (mesh.cpp:744-757): L = the subdomain cell, R = ghost row nelem+icface, nodes
	// in the cell's own order so the face points out of the subdomain
	for(int ic = 0; ic < M.nconnface; ic++, fi++) {
		const int inelem = connface[5*ic], lf = connface[5*ic+1], nn = md.nnode[inelem];
		M.intfac[4*fi+0] = inelem;
		M.esuel[static_cast<size_t>(inelem)*mf+lf] = N + ic;
		M.elemface[static_cast<size_t>(inelem)*mf+lf] = fi;
		M.intfac[4*fi+1] = N + ic;
		M.intfac[4*fi+2] = nodeOf(md, inelem, (lf+0) % nn);
		M.intfac[4*fi+3] = nodeOf(md, inelem, (lf+1) % nn);
	}

	// compute_areas (mesh.cpp:290-313)
	auto X = [&](int p) { return md.coords[2*p]; };
	auto Y = [&](int p) { return md.coords[2*p+1]; };
	M.area.resize(N);
	for(int i = 0; i < N; i++) {
		const int p0 = nodeOf(md,i,0), p1 = nodeOf(md,i,1), p2 = nodeOf(md,i,2);
		double a = 0.5*(X(p0)*(Y(p1) - Y(p2)) - Y(p0)*(X(p1) - X(p2)) + X(p1)*Y(p2) - X(p2)*Y(p1));
		if(md.nnode[i] == 4) {
			const int p3 = nodeOf(md,i,3);
			a += 0.5*(X(p0)*(Y(p2) - Y(p3)) - Y(p0)*(X(p2) - X(p3)) + X(p2)*Y(p3) - X(p3)*Y(p2));
		}
		M.area[i] = a;
	}

	// compute_face_data (mesh.cpp:346-365): pow(x,2) in glibc is exactly x*x rounded
	M.facemetric.resize(static_cast<size_t>(M.naface)*3);
	for(int i = 0; i < M.naface; i++) {
		const int a = M.intfac[4*i+2], b = M.intfac[4*i+3];
		double nx = Y(b) - Y(a);
		double ny = -1.0*(X(b) - X(a));
		const double len = std::sqrt(nx*nx + ny*ny);
		M.facemetric[3*i+0] = nx/len;
		M.facemetric[3*i+1] = ny/len;
		M.facemetric[3*i+2] = len;
	}

	// compute_cell_centres (mesh.cpp:316-328)
	M.rc.resize(static_cast<size_t>(N + M.nconnface)*2);
	for(int i = 0; i < N; i++)
		for(int d = 0; d < 2; d++) {
			double s = 0;
			for(int j = 0; j < md.nnode[i]; j++) s += md.coords[2*nodeOf(md,i,j)+d];
			M.rc[2*i+d] = s / static_cast<double>(md.nnode[i]);
		}

	// face centres (aspatial.cpp:50-61): gr starts at zero, nodes summed in order, /nnofa
	M.gr.resize(static_cast<size_t>(M.naface)*2);
	for(int i = 0; i < M.naface; i++)
		for(int d = 0; d < 2; d++) {
			double s = 0;
			s += md.coords[2*M.intfac[4*i+2]+d];
			s += md.coords[2*M.intfac[4*i+3]+d];
			M.gr[2*i+d] = s / 2;
		}

	// ghost centres about face midpoints (aspatial.cpp:97-119)
	M.rcbp.resize(static_cast<size_t>(md.nbface)*2);
	for(int i = 0; i < md.nbface; i++) {
		const int ie = M.intfac[4*i];
		for(int d = 0; d < 2; d++) {
			double mid = 0;
			mid += md.coords[2*M.intfac[4*i+2]+d];
			mid += md.coords[2*M.intfac[4*i+3]+d];
			mid /= 2;
			M.rcbp[2*i+d] = 2.0*mid - M.rc[2*ie+d];
		}
	}

	M.md = std::move(md);
}

// ------------------------------------------------------------------------------------------------
// Subdomains (multi-rank meshes)
// ------------------------------------------------------------------------------------------------

std::vector<int> partitionTrivial(int nelem, int nranks)
{
	if(nranks < 1 || nelem < nranks) throw std::runtime_error("Not enough cells in this mesh for "
	                                                            + std::to_string(nranks) + " processes!");
	const int per = nelem / nranks;
	std::vector<int> d(nelem, nranks-1);
	for(int r = 0; r < nranks; r++)
		for(int i = r*per; i < (r+1)*per; i++) d[i] = r;
	return d;
}

Mesh restrictMesh(const Mesh& gm, const int* elemdist, int rank)
{
	const MeshData& g = gm.md;
	if(gm.nconnface != 0) throw std::runtime_error("restrictMesh: expects the global mesh");
	MeshData lm;
	lm.maxnnode = g.maxnnode; lm.maxnfael = g.maxnfael; lm.nnofa = g.nnofa;
	lm.nbtag = g.nbtag; lm.ndtag = g.ndtag;
	// 1. cells of this rank in global order (extractInpoel, :161-182)
	std::vector<int> glob;
	for(int e = 0; e < g.nelem; e++)
		if(elemdist[e] == rank) {
			glob.push_back(e);
			for(int j = 0; j < g.maxnnode; j++) lm.inpoel.push_back(g.inpoel[static_cast<size_t>(e)*g.maxnnode+j]);
			for(int j = 0; j < g.ndtag; j++) lm.vol_regions.push_back(g.vol_regions[static_cast<size_t>(e)*g.ndtag+j]);
			lm.nnode.push_back(g.nnode[e]);
			lm.nfael.push_back(g.nfael[e]);
		}
	lm.nelem = static_cast<int>(glob.size());
	if(lm.nelem == 0) throw std::runtime_error("restrictMesh: rank " + std::to_string(rank) + " owns no cells");
	// 2. the points they use, in ascending global order (extractPointCoords, :184-223)
	std::vector<int> pts;
	for(int e = 0; e < lm.nelem; e++)
		for(int j = 0; j < lm.nnode[e]; j++) pts.push_back(lm.inpoel[static_cast<size_t>(e)*lm.maxnnode+j]);
	std::sort(pts.begin(), pts.end());
	pts.erase(std::unique(pts.begin(), pts.end()), pts.end());
	lm.npoin = static_cast<int>(pts.size());
	std::vector<int> g2l(g.npoin, -1);
	lm.coords.resize(2*static_cast<size_t>(lm.npoin));
	for(int i = 0; i < lm.npoin; i++) {
		g2l[pts[i]] = i;
		lm.coords[2*i] = g.coords[2*static_cast<size_t>(pts[i])];
		lm.coords[2*i+1] = g.coords[2*static_cast<size_t>(pts[i])+1];
	}
	// 3. local point numbers (:66-69)
	for(int e = 0; e < lm.nelem; e++)
		for(int j = 0; j < lm.nnode[e]; j++) {
			int& v = lm.inpoel[static_cast<size_t>(e)*lm.maxnnode+j];
			v = g2l[v];
		}
	// 4. the physical boundary faces whose cell is here, in global order (extractbfaces, :225-276)
	const int gbw = g.nnofa + g.nbtag;
	lm.nbface = 0;
	for(int f = 0; f < g.nbface; f++) {
		if(elemdist[gm.intfac[4*static_cast<size_t>(f)]] != rank) continue;
		for(int j = 0; j < g.nnofa; j++) lm.bface.push_back(g2l[g.bface[static_cast<size_t>(f)*gbw+j]]);
		for(int j = 0; j < g.nbtag; j++) lm.bface.push_back(g.bface[static_cast<size_t>(f)*gbw+g.nnofa+j]);
		lm.nbface++;
	}
	// 5. local esuel; points on a physical boundary face (:76-82, :278-291)
	std::vector<int> esup_p, esup;
	buildEsup(lm, esup_p, esup);
	const std::vector<int> esuel = esuelOf(lm, esup_p, esup);
	std::vector<char> bpoin(lm.npoin, 0);
	const int lbw = lm.nnofa + lm.nbtag;
	for(int f = 0; f < lm.nbface; f++)
		for(int j = 0; j < lm.nnofa; j++) bpoin[lm.bface[static_cast<size_t>(f)*lbw+j]] = 1;
	// 6. connectivity faces: local faces without a local neighbour with a point off the physical
	// boundary (getConnectivityFaceEIndices :293-331), matched to the global cell's face (:98-154)
	std::vector<int> cf;
	for(int e = 0; e < lm.nelem; e++)
		for(int lf = 0; lf < lm.nfael[e]; lf++) {
			if(esuel[static_cast<size_t>(e)*lm.maxnfael+lf] != -1) continue;
			bool conn = false;
			for(int k = 0; k < lm.nnofa; k++)
				if(!bpoin[nodeOf(lm, e, (lf+k) % lm.nnode[e])]) { conn = true; break; }
			if(!conn) continue;
			const int ge = glob[e];
			int nbrank = -1, nbcell = -1;
			for(int jgf = 0; jgf < g.nfael[ge]; jgf++) {
				bool matched = true;
				for(int k = 0; k < g.nnofa; k++) {
					const int gp = nodeOf(g, ge, (jgf+k) % g.nnode[ge]);
					bool pm = false;
					for(int l = 0; l < lm.nnofa; l++)
						if(pts[nodeOf(lm, e, (lf+l) % lm.nnode[e])] == gp) { pm = true; break; }
					if(!pm) { matched = false; break; }
				}
				if(matched) {
					nbcell = gm.esuel[static_cast<size_t>(ge)*g.maxnfael+jgf];
					nbrank = elemdist[nbcell];
					break;
				}
			}
			if(nbrank < 0) throw std::logic_error("Could not find connectivity face!");
			const int c5[5] = {e, lf, nbrank, nbcell, gm.elemface[static_cast<size_t>(ge)*g.maxnfael+lf]};
			cf.insert(cf.end(), c5, c5+5);
		}
	Mesh M;
	buildTopology(std::move(lm), M, cf);
	M.globalElemIndex = glob;
	// ghost rows of the cell centres: the neighbours' centres (the owner computes them from the same
	// points in the same order, so they equal the global mesh's)
	for(int ic = 0; ic < M.nconnface; ic++)
		for(int d = 0; d < 2; d++)
			M.rc[2*(static_cast<size_t>(M.md.nelem)+ic)+d] = gm.rc[2*static_cast<size_t>(cf[5*ic+3])+d];
	return M;
}

// ------------------------------------------------------------------------------------------------
// Synthetic meshes
// ------------------------------------------------------------------------------------------------

namespace {

/// NACA 0012 half-thickness with a closed trailing edge (coefficient -0.1036).
inline double naca0012(double x) {
	return 0.6*(0.2969*std::sqrt(x) - 0.1260*x - 0.3516*x*x + 0.2843*x*x*x - 0.1036*x*x*x*x);
}

/// Adds an O-grid of points (ntheta x (nlayers+1)), layer 0 = body, and returns the point index
void addOgridCells(MeshData& m, int ntheta, int nquad, int ntri, int pt0)
{
	const int nl = nquad + ntri;
	auto P = [&](int i, int j) { return pt0 + j*ntheta + (i % ntheta); };
	for(int j = 0; j < nl; j++)
		for(int i = 0; i < ntheta; i++) {
			// i runs counter-clockwise round the body and j outwards, so (i,j) -> (i,j+1) ->
			// (i+1,j+1) -> (i+1,j) is counter-clockwise
			const int a = P(i,j), b = P(i,j+1), c = P(i+1,j+1), d = P(i+1,j);
			if(j < nquad) {
				m.inpoel.insert(m.inpoel.end(), {a, b, c, d});
				m.nnode.push_back(4); m.nfael.push_back(4);
			} else {
				// alternate the diagonal by cell parity for a less biased triangulation
				if((i + j) % 2 == 0) {
					m.inpoel.insert(m.inpoel.end(), {a, b, c, -1, d, a, c, -1});
				} else {
					m.inpoel.insert(m.inpoel.end(), {a, b, d, -1, b, c, d, -1});
				}
				m.nnode.push_back(3); m.nfael.push_back(3);
				m.nnode.push_back(3); m.nfael.push_back(3);
			}
		}
}

void finishOgrid(MeshData& m, int ntheta, int nl, int wallmarker, int farmarker)
{
	m.nnofa = 2; m.nbtag = 2; m.ndtag = 2;
	m.nelem = static_cast<int>(m.nnode.size());
	m.maxnnode = 0; m.maxnfael = 0;
	for(int i = 0; i < m.nelem; i++) {
		m.maxnnode = std::max(m.maxnnode, m.nnode[i]); m.maxnfael = std::max(m.maxnfael, m.nfael[i]);
	}
	// inpoel was pushed with stride 4; compact to maxnnode if all-triangle
	if(m.maxnnode == 3) {
		std::vector<int> c(static_cast<size_t>(m.nelem)*3);
		for(int i = 0; i < m.nelem; i++) for(int j = 0; j < 3; j++) c[3*i+j] = m.inpoel[4*i+j];
		m.inpoel.swap(c);
	}
	m.vol_regions.assign(static_cast<size_t>(m.nelem)*2, 0);
	for(int i = 0; i < m.nelem; i++) { m.vol_regions[2*i] = 1; m.vol_regions[2*i+1] = 1; }
	// boundary faces: wall (inner loop, traversed so that the outward normal points into the body)
	// then farfield; orientation is fixed later by correctBoundaryFaceOrientation anyway.
	m.nbface = 2*ntheta;
	m.bface.resize(static_cast<size_t>(m.nbface)*4);
	for(int i = 0; i < ntheta; i++) {
		const int a = i, b = (i+1) % ntheta;
		int* f = &m.bface[4*i];
		f[0] = a; f[1] = b; f[2] = wallmarker; f[3] = 1;
	}
	for(int i = 0; i < ntheta; i++) {
		const int a = nl*ntheta + i, b = nl*ntheta + (i+1) % ntheta;
		int* f = &m.bface[4*(ntheta+i)];
		f[0] = b; f[1] = a; f[2] = farmarker; f[3] = 1;
	}
}

}

MeshData generateNacaOgrid(int ntheta, int nquad, int ntri, double rfar, double wallspacing, int farmap)
{
	if(ntheta < 8 || ntheta % 2) throw std::invalid_argument("ntheta must be even and >= 8");
	MeshData m;
	const int nl = nquad + ntri;
	m.npoin = ntheta*(nl+1);
	m.coords.resize(static_cast<size_t>(m.npoin)*2);
	const double PI = 3.14159265358979323846;
	// surface: i = 0 at the trailing edge, going over the lower surface to the LE and back over the
	// upper surface (counter-clockwise), cosine clustering at LE and TE
	std::vector<double> sx(ntheta), sy(ntheta), fx(ntheta), fy(ntheta);
	const int half = ntheta/2;
	for(int i = 0; i < ntheta; i++) {
		double x, y;
		if(i <= half) {
			const double s = static_cast<double>(i)/half;             // 0 at TE, 1 at LE
			x = 0.5*(1.0 + std::cos(PI*s));
			y = -naca0012(x);
		} else {
			const double s = static_cast<double>(i-half)/half;        // 0 at LE, 1 at TE
			x = 0.5*(1.0 - std::cos(PI*s));
			y = naca0012(x);
		}
		sx[i] = x; sy[i] = y;
		// matching far-field point. farmap 0: the direction of the surface point from the mid-chord
		// centre (cosine-clustered surface points crowd the far field fore and aft: the grid lines
		// above and below mid-chord fan out to ~1 degree per cell at ntheta 2048); farmap 1: far-field
		// angles uniform in the surface parameter (lower surface TE -> LE: 0 -> -pi, upper: pi -> 0)
		double ang = std::atan2(y, x - 0.5);
		if(farmap & 1) ang = i <= half ? -PI*static_cast<double>(i)/half : PI - PI*static_cast<double>(i-half)/half;
		if(i == 0) ang = 0.0;
		if(i == half) ang = PI;
		fx[i] = 0.5 + rfar*std::cos(ang); fy[i] = rfar*std::sin(ang);
	}
	// The surface runs clockwise when i increases (TE -> lower -> LE -> upper is clockwise seen
	// from above? lower surface first with y<0 going from x=1 to x=0 is clockwise). Reverse i so
	// that cells come out counter-clockwise.
	std::reverse(sx.begin()+1, sx.end()); std::reverse(sy.begin()+1, sy.end());
	std::reverse(fx.begin()+1, fx.end()); std::reverse(fy.begin()+1, fy.end());
	// radial distribution: geometric growth from wallspacing, capped so the sum reaches 1
	std::vector<double> eta(nl+1, 0.0);
	{
		// find growth ratio q such that wallspacing*(q^nl - 1)/(q - 1) = 1 (in normalised units of
		// the body-to-farfield distance ~ rfar)
		const double target = 1.0/ (wallspacing/rfar);
		double lo = 1.0 + 1e-12, hi = 2.0;
		for(int it = 0; it < 200; it++) {
			const double q = 0.5*(lo+hi);
			const double s = (std::pow(q, nl) - 1.0)/(q - 1.0);
			if(s > target) hi = q; else lo = q;
		}
		const double q = 0.5*(lo+hi);
		double acc = 0, d = 1.0;
		for(int j = 1; j <= nl; j++) { acc += d; eta[j] = acc; d *= q; }
		for(int j = 1; j <= nl; j++) eta[j] /= acc;
	}
	// farmap bit 2: the layers leave the body along its normal. Straight lines from each surface point
	// to its far-field point meet the aft surface at a few degrees (the first layers of the C5 family
	// were 8-9 degree parallelograms over the last percent of chord: a second-order residual on them has no
	// steady state). Point j of line i sits at the distance eta_j*|f - s| from the surface point along
	// the direction (1 - w) n + w t, n the outward normal, t the line's own direction, w = smoothstep(d / 3
	// chords) of that distance d: normal through the boundary layer (w = 0.002 at 0.08 chord), back on the
	// straight line from three chords out (the cells beyond are those of farmap 0/1). The trailing-edge
	// point's normal is the bisector (+x), so the corner is a fan of cells. Blending over 1 / 2 / 3 / 5
	// chords leaves 56 / 8 / 8 / 8 cells skewed by more than 60 degrees (3,390 with straight lines, C5/8).
	const bool wallnormal = (farmap & 2) != 0;
	const double blend = 3.0;
	for(int j = 0; j <= nl; j++)
		for(int i = 0; i < ntheta; i++) {
			const size_t p = static_cast<size_t>(j)*ntheta + i;
			double dx = fx[i] - sx[i], dy = fy[i] - sy[i];
			const double L = std::sqrt(dx*dx + dy*dy);
			if(wallnormal && j > 0 && eta[j]*L < blend) {
				const int ip = (i + 1) % ntheta, im = (i + ntheta - 1) % ntheta;
				double nx = sy[ip] - sy[im], ny = -(sx[ip] - sx[im]);
				if(nx*dx + ny*dy < 0) { nx = -nx; ny = -ny; }
				const double nn = std::sqrt(nx*nx + ny*ny);
				const double x = eta[j]*L/blend;
				const double w = x*x*(3.0 - 2.0*x);
				double ex = (1.0 - w)*nx/nn + w*dx/L, ey = (1.0 - w)*ny/nn + w*dy/L;
				const double en = std::sqrt(ex*ex + ey*ey);
				dx = L*ex/en; dy = L*ey/en;
			}
			m.coords[2*p] = sx[i] + eta[j]*dx;
			m.coords[2*p+1] = sy[i] + eta[j]*dy;
		}
	addOgridCells(m, ntheta, nquad, ntri, 0);
	finishOgrid(m, ntheta, nl, 2, 4);
	return m;
}

/// C-grid round the NACA 0012 (the C5 family, BASELINE config 5's viscous case). A sharp trailing edge
/// in an O-grid either leaves the aft boundary layer as thin parallelograms (straight lines to the far
/// field) or fans one trailing-edge point's cells over the whole wake (wall-normal lines); the C-grid's
/// wake cut carries the boundary-layer spacing downstream instead. Columns i = 0 .. ni-1, ni = 2 nwake +
/// nsurf + 1: the lower wake from the outflow to the trailing edge, the lower surface to the leading edge,
/// the upper surface, the upper wake to the outflow; row 0 is the body and the cut (both wakes' row-0
/// points are the same points), rows 1 .. nquad + ntri go out to a C boundary: a half circle of radius rfar
/// round the trailing edge and the lines y = +-rfar to the outflow at x = 1 + rfar. Surface points are
/// clustered at the leading edge (half-cosine) and, less, at the trailing edge (half of a full cosine); the
/// wake spacing grows geometrically from the trailing-edge spacing. Wake lines run from the cut to the
/// far field, where their spacing starts at the half circle's and grows to the outflow, leaving the cut
/// vertically; a surface point's line leaves along the wall normal (turned vertical over the last tenth of the chord, parallel to
/// the wake lines at the trailing edge) and bends onto the straight line to its far-field point (angles
/// uniform in the surface parameter) by one chord (smoothstep). Rows grow geometrically from
/// `wallspacing`. Quadrangles in the first nquad rows, triangles beyond. Markers: wall 2, far field 4.
namespace {

/// The C-grid's mapping (generateNacaCgrid's columns and rows, shared with generateNacaHybrid): column i's
/// point at the normalised distance eta along its line from the body / wake cut to the far field
struct CgridMap
{
	int nsurf, nwake, ni, half;
	std::vector<double> sx, sy, fx, fy;
	double blend = 1.0;
	CgridMap(int nsurf_, int nwake_, double rfar) : nsurf(nsurf_), nwake(nwake_), ni(2*nwake_ + nsurf_ + 1),
		half(nsurf_/2), sx(ni), sy(ni), fx(ni), fy(ni)
	{
		const double PI = 3.14159265358979323846;
		// surface, upper side parameter t = 0 (LE) .. 1 (TE)
		auto xs = [&](double t) { return 0.5*(1.0 - std::cos(0.5*PI*t)) + 0.25*(1.0 - std::cos(PI*t)); };
		const double dte = 1.0 - xs(1.0 - 1.0/half);               // trailing-edge spacing
		// wake stations x = 1 + w_k, k = 1 .. nwake, geometric from dte to the outflow
		std::vector<double> wx(nwake + 1, 1.0);
		{
			const double L = rfar;
			double lo = 1.0 + 1e-12, hi = 2.0;
			for(int it = 0; it < 200; it++) {
				const double q = 0.5*(lo + hi);
				if(dte*(std::pow(q, nwake) - 1.0)/(q - 1.0) > L) hi = q; else lo = q;
			}
			const double q = 0.5*(lo + hi);
			double acc = 0, d = dte;
			for(int k = 1; k <= nwake; k++) { acc += d; wx[k] = 1.0 + acc; d *= q; }
			for(int k = 1; k <= nwake; k++) wx[k] = 1.0 + (wx[k] - 1.0)*L/acc;
		}
		// the wake lines' far ends along y = +-rfar: spacing from the half circle's (pi rfar / nsurf) growing
		// geometrically to the outflow, so the columns next to the trailing edge's line widen outwards
		// instead of running to the far field as slivers of the trailing-edge spacing
		std::vector<double> ox(nwake + 1, 1.0);
		{
			const double L = rfar, s0 = PI*rfar/nsurf;
			if(s0*nwake >= L) { for(int k = 1; k <= nwake; k++) ox[k] = 1.0 + L*k/nwake; }
			else {
				double lo = 1.0 + 1e-12, hi = 2.0;
				for(int it = 0; it < 200; it++) {
					const double q = 0.5*(lo + hi);
					if(s0*(std::pow(q, nwake) - 1.0)/(q - 1.0) > L) hi = q; else lo = q;
				}
				const double q = 0.5*(lo + hi);
				double acc = 0, d = s0;
				for(int k = 1; k <= nwake; k++) { acc += d; ox[k] = 1.0 + acc; d *= q; }
				for(int k = 1; k <= nwake; k++) ox[k] = 1.0 + (ox[k] - 1.0)*L/acc;
			}
		}
		for(int i = 0; i < ni; i++) {
			if(i < nwake || i > nwake + nsurf) {                     // wake: lines from the cut to y = +-rfar
				const bool lower = i < nwake;
				const int k = lower ? nwake - i : i - (nwake + nsurf);
				sx[i] = wx[k]; sy[i] = 0.0;
				fx[i] = ox[k]; fy[i] = lower ? -rfar : rfar;
			} else {
				const int m = i - nwake;                                // 0 .. nsurf: TE lower -> LE -> TE upper
				const bool lower = m < half;
				const double t = lower ? static_cast<double>(half - m)/half : static_cast<double>(m - half)/half;
				const double x = m == 0 || m == nsurf ? 1.0 : xs(t);
				sx[i] = x; sy[i] = lower ? -naca0012(x) : naca0012(x);
				if(m == 0 || m == nsurf) sy[i] = 0.0;
				const double ang = -0.5*PI - PI*static_cast<double>(m)/nsurf;   // -pi/2 (down) .. -3pi/2 (up)
				fx[i] = 1.0 + rfar*std::cos(ang); fy[i] = rfar*std::sin(ang);
			}
		}
	}
	/// column i's point at eta (0: body / cut, 1: far field); eta > 0 only off the body
	void point(int i, double eta, double& x, double& y) const
	{
		double dx = fx[i] - sx[i], dy = fy[i] - sy[i];
		const double L = std::sqrt(dx*dx + dy*dy);
		const bool body = i > nwake && i < nwake + nsurf;
		const bool te = i == nwake || i == nwake + nsurf;
		if(!te && eta > 0.0 && eta*L < blend) {
			double nx = 0.0, ny = fy[i] > 0 ? 1.0 : -1.0;           // wake: the cut's normal
			if(body) {
				nx = sy[i+1] - sy[i-1]; ny = -(sx[i+1] - sx[i-1]);
				if(nx*dx + ny*dy < 0) { nx = -nx; ny = -ny; }
				if(sx[i] > 0.9) {                               // the normal turns vertical at the trailing
					const double g = (sx[i] - 0.9)/0.1;          // edge, parallel to the wake lines next to it
					nx *= 1.0 - g*g*(3.0 - 2.0*g);
				}
			}
			const double nn = std::sqrt(nx*nx + ny*ny);
			const double xx = eta*L/blend;
			const double w = xx*xx*(3.0 - 2.0*xx);
			const double ex = (1.0 - w)*nx/nn + w*dx/L, ey = (1.0 - w)*ny/nn + w*dy/L;
			const double en = std::sqrt(ex*ex + ey*ey);
			dx = L*ex/en; dy = L*ey/en;
		}
		x = sx[i] + eta*dx;
		y = sy[i] + eta*dy;
	}
};

/// growth ratio q of nl rows whose first is `first` and whose sum is `total`
double rowGrowth(int nl, double total_over_first)
{
	double lo = 1.0 + 1e-12, hi = 2.0;
	for(int it = 0; it < 200; it++) {
		const double q = 0.5*(lo+hi);
		if((std::pow(q, nl) - 1.0)/(q - 1.0) > total_over_first) hi = q; else lo = q;
	}
	return 0.5*(lo+hi);
}

}

/// C-grid round the NACA 0012 (the quadrangle C-grid of round 5). A sharp trailing edge
/// in an O-grid either leaves the aft boundary layer as thin parallelograms (straight lines to the far
/// field) or fans one trailing-edge point's cells over the whole wake (wall-normal lines); the C-grid's
/// wake cut carries the boundary-layer spacing downstream instead. Columns i = 0 .. ni-1, ni = 2 nwake +
/// nsurf + 1: the lower wake from the outflow to the trailing edge, the lower surface to the leading edge,
/// the upper surface, the upper wake to the outflow; row 0 is the body and the cut (both wakes' row-0
/// points are the same points), rows 1 .. nquad + ntri go out to a C boundary: a half circle of radius rfar
/// round the trailing edge and the lines y = +-rfar to the outflow at x = 1 + rfar. Surface points are
/// clustered at the leading edge (half-cosine) and, less, at the trailing edge (half of a full cosine); the
/// wake spacing grows geometrically from the trailing-edge spacing. Wake lines run from the cut to the
/// far field, where their spacing starts at the half circle's and grows to the outflow, leaving the cut
/// vertically; a surface point's line leaves along the wall normal (turned vertical over the last tenth of the chord, parallel to
/// the wake lines at the trailing edge) and bends onto the straight line to its far-field point (angles
/// uniform in the surface parameter) by one chord (smoothstep). Rows grow geometrically from
/// `wallspacing`. Quadrangles in the first nquad rows, triangles beyond. Markers: wall 2, far field 4.
MeshData generateNacaCgrid(int nsurf, int nwake, int nquad, int ntri, double rfar, double wallspacing)
{
	if(nsurf < 8 || nsurf % 2 || nwake < 2) throw std::invalid_argument("nsurf must be even and >= 8, nwake >= 2");
	const CgridMap map(nsurf, nwake, rfar);
	const int nl = nquad + ntri, ni = map.ni;
	// rows: geometric growth from the wall spacing over nl layers (normalised to the line length)
	std::vector<double> eta(nl+1, 0.0);
	{
		const double q = rowGrowth(nl, rfar/wallspacing);
		double acc = 0, d = 1.0;
		for(int j = 1; j <= nl; j++) { acc += d; eta[j] = acc; d *= q; }
		for(int j = 1; j <= nl; j++) eta[j] /= acc;
	}
	// points: row 0 has nwake + nsurf distinct points (the upper wake's are the lower wake's), rows >= 1 ni
	const int n0 = nwake + nsurf;
	auto P = [&](int i, int j) { return j == 0 ? (i < n0 ? i : ni - 1 - i) : n0 + (j-1)*ni + i; };
	MeshData m;
	m.npoin = n0 + nl*ni;
	m.coords.resize(static_cast<size_t>(m.npoin)*2);
	for(int j = 0; j <= nl; j++)
		for(int i = 0; i < ni; i++) {
			if(j == 0 && i >= n0) continue;
			const size_t p = static_cast<size_t>(P(i, j));
			map.point(i, eta[j], m.coords[2*p], m.coords[2*p+1]);
		}
	// cells: (i,j) (i+1,j) (i+1,j+1) (i,j+1) counter-clockwise (i runs clockwise round the body, j outwards)
	for(int j = 0; j < nl; j++)
		for(int i = 0; i < ni - 1; i++) {
			const int a = P(i,j), b = P(i+1,j), c = P(i+1,j+1), d = P(i,j+1);
			if(j < nquad) {
				m.inpoel.insert(m.inpoel.end(), {a, b, c, d});
				m.nnode.push_back(4); m.nfael.push_back(4);
			} else {
				if((i + j) % 2 == 0) m.inpoel.insert(m.inpoel.end(), {a, b, c, -1, a, c, d, -1});
				else m.inpoel.insert(m.inpoel.end(), {a, b, d, -1, b, c, d, -1});
				m.nnode.push_back(3); m.nfael.push_back(3);
				m.nnode.push_back(3); m.nfael.push_back(3);
			}
		}
	m.nnofa = 2; m.nbtag = 2; m.ndtag = 2;
	m.nelem = static_cast<int>(m.nnode.size());
	m.maxnnode = nquad > 0 ? 4 : 3; m.maxnfael = m.maxnnode;
	if(m.maxnnode == 3) {
		std::vector<int> c(static_cast<size_t>(m.nelem)*3);
		for(int e = 0; e < m.nelem; e++) for(int k = 0; k < 3; k++) c[3*e+k] = m.inpoel[4*e+k];
		m.inpoel.swap(c);
	}
	m.vol_regions.assign(static_cast<size_t>(m.nelem)*2, 1);
	// boundary faces: the wall (row 0 along the body), the far field (the outer row and both outflow columns)
	auto bf = [&](int a, int b, int tag) { m.bface.insert(m.bface.end(), {a, b, tag, 1}); };
	for(int i = nwake; i < nwake + nsurf; i++) bf(P(i,0), P(i+1,0), 2);
	for(int i = 0; i < ni - 1; i++) bf(P(i+1,nl), P(i,nl), 4);
	for(int j = 0; j < nl; j++) { bf(P(0,j+1), P(0,j), 4); bf(P(ni-1,j), P(ni-1,j+1), 4); }
	m.nbface = static_cast<int>(m.bface.size()/4);
	return m;
}

MeshData generateNacaHybrid(int nsurf, int nwake, int nquad, int nl, double rfar, double wallspacing)
{
	if(nsurf < 8 || nsurf % 2 || nwake < 2) throw std::invalid_argument("nsurf must be even and >= 8, nwake >= 2");
	if(nquad < 1 || nquad >= nl) throw std::invalid_argument("need 1 <= nquad < nrows");
	const CgridMap map(nsurf, nwake, rfar);
	const int ni = map.ni, ib0 = nwake, ib1 = nwake + nsurf;      // the body's columns [ib0, ib1]
	std::vector<double> eta(nl+1, 0.0);                            // generateNacaCgrid's rows
	{
		const double q = rowGrowth(nl, rfar/wallspacing);
		double acc = 0, d = 1.0;
		for(int j = 1; j <= nl; j++) { acc += d; eta[j] = acc; d *= q; }
		for(int j = 1; j <= nl; j++) eta[j] /= acc;
	}
	MeshData m;
	// C-grid points: every column of rows 0 .. nquad (row 0: the wake points shared), and above row nquad the
	// wake blocks' columns [0, ib0] and [ib1, ni-1] (the trailing edge's columns included)
	const int n0 = nwake + nsurf, nw = nwake + 1;
	auto P = [&](int i, int j) {
		if(j == 0) return i < n0 ? i : ni - 1 - i;
		if(j <= nquad) return n0 + (j-1)*ni + i;
		return n0 + nquad*ni + (j-nquad-1)*2*nw + (i <= ib0 ? i : nw + (i - ib1));
	};
	m.coords.resize(static_cast<size_t>(n0 + nquad*ni + (nl - nquad)*2*nw)*2);
	for(int j = 0; j <= nl; j++)
		for(int i = 0; i < ni; i++) {
			if(j == 0 && i >= n0) continue;
			if(j > nquad && i > ib0 && i < ib1) continue;
			const size_t p = static_cast<size_t>(P(i, j));
			map.point(i, eta[j], m.coords[2*p], m.coords[2*p+1]);
		}
	auto quad = [&](int i, int j) {
		m.inpoel.insert(m.inpoel.end(), {P(i,j), P(i+1,j), P(i+1,j+1), P(i,j+1)});
		m.nnode.push_back(4); m.nfael.push_back(4);
	};
	auto dist = [](double ax, double ay, double bx, double by) { return std::hypot(bx - ax, by - ay); };
	auto ccw = [&](int p0, int p1, int p2) {
		return (m.coords[2*p1] - m.coords[2*p0])*(m.coords[2*p2+1] - m.coords[2*p0+1])
		     - (m.coords[2*p1+1] - m.coords[2*p0+1])*(m.coords[2*p2] - m.coords[2*p0]) > 0.0; };
	auto tri = [&](int a, int b, int c) {
		if(!ccw(a, b, c)) throw std::runtime_error("generateNacaHybrid: an inverted triangle");
		m.inpoel.insert(m.inpoel.end(), {a, b, c, -1});
		m.nnode.push_back(3); m.nfael.push_back(3);
	};
	// zips polylines A (inner) and B (outer) that run the same way, A[0]-B[0] and their last points joined by
	// the trailing edge's columns: the region between them is cut into triangles, advancing along the one
	// whose next diagonal is shorter unless that triangle would be inverted or leave an invalid fan to the
	// other's end
	auto zip = [&](const std::vector<int>& A, const std::vector<int>& B) {
		const size_t M = A.size() - 1, N = B.size() - 1;
		size_t a = 0, b = 0;
		auto d = [&](int p, int q2) { return dist(m.coords[2*p], m.coords[2*p+1], m.coords[2*q2], m.coords[2*q2+1]); };
		while(a < M || b < N) {
			bool advA = a == M ? false : (b == N ? true : d(A[a+1], B[b]) < d(A[a], B[b+1]));
			auto okA = [&]() {
				if(!ccw(A[a], A[a+1], B[b])) return false;
				if(a + 1 == M) for(size_t j = b; j < N; j++) if(!ccw(A[M], B[j+1], B[j])) return false;
				return true; };
			auto okB = [&]() {
				if(!ccw(A[a], B[b+1], B[b])) return false;
				if(b + 1 == N) for(size_t i = a; i < M; i++) if(!ccw(A[i], A[i+1], B[N])) return false;
				return true; };
			if(advA && b < N && !okA()) advA = false;
			else if(!advA && a < M && !okB()) advA = true;
			if(advA) { tri(A[a], A[a+1], B[b]); a++; }
			else { tri(A[a], B[b+1], B[b]); b++; }
		}
	};
	// cells row by row: the wake blocks' quadrangles in every row, the body's in rows below nquad, and above
	// them the lower half of each body row (trailing edge to leading edge, both end points kept) resampled to
	// its distance from the row below over 0.87 (equilateral triangles), within a factor 1.25 of the row
	// below's spacing, and zipped to it; the upper half is its mirror image (y -> -y), so the mesh is
	// symmetric about the chord line as the C-grid is (CL = 0 at alpha 0 up to rounding)
	const double gam = 1.25;
	const int ile = nwake + nsurf/2;                           // the leading edge's column (its own mirror)
	std::vector<int> mir(m.coords.size()/2, -1);               // mirror image of every point
	for(int j = 1; j <= nl; j++)
		for(int i = 0; i < ni; i++) {
			if(j > nquad && i > ib0 && i < ib1) continue;
			mir[P(i, j)] = P(ni - 1 - i, j);
		}
	std::vector<int> below;                                    // the lower half of the body's row below
	std::vector<double> bs;                                    // its nodes' column coordinates
	for(int j = 0; j < nl; j++) {
		for(int i = 0; i < ib0; i++) quad(i, j);
		if(j < nquad) for(int i = ib0; i < ib1; i++) quad(i, j);
		for(int i = ib1; i < ni - 1; i++) quad(i, j);
		if(j + 1 == nquad) {
			for(int i = ib0; i <= ile; i++) { below.push_back(P(i, nquad)); bs.push_back(i); }
		}
		if(j < nquad) continue;
		// row j + 1 at the lower half's columns
		const int nc = ile - ib0 + 1;
		std::vector<double> cx(nc), cy(nc);
		for(int i = 0; i < nc; i++) map.point(ib0 + i, eta[j+1], cx[i], cy[i]);
		std::vector<double> phi(nc, 0.0);
		size_t jb = 0;
		for(int i = 0; i + 1 < nc; i++) {
			const double sm = i + 0.5;
			while(jb + 2 < bs.size() && bs[jb+1] - ib0 < sm) jb++;
			const int pa = below[jb], pb = below[jb+1];
			const double hp = dist(m.coords[2*pa], m.coords[2*pa+1], m.coords[2*pb], m.coords[2*pb+1]);
			double bx0, by0, bx1, by1;
			map.point(ib0 + i, eta[j], bx0, by0); map.point(ib0 + i + 1, eta[j], bx1, by1);
			const double dl = 0.5*(dist(bx0, by0, cx[i], cy[i]) + dist(bx1, by1, cx[i+1], cy[i+1]));
			const double h = std::min(std::max(dl/0.87, hp/gam), gam*hp);
			phi[i+1] = phi[i] + dist(cx[i], cy[i], cx[i+1], cy[i+1])/h;
		}
		const int n = std::max(1, static_cast<int>(std::lround(phi.back())));
		auto addPoint = [&](double x, double y) {
			m.coords.push_back(x); m.coords.push_back(y); mir.push_back(-1);
			return static_cast<int>(m.coords.size()/2) - 1;
		};
		std::vector<int> row(n + 1);
		std::vector<double> rs(n + 1);
		row[0] = P(ib0, j+1); rs[0] = ib0;
		row[n] = addPoint(cx[nc-1], cy[nc-1]); rs[n] = ile;
		mir[row[n]] = row[n];
		for(int a2 = 1, i = 0; a2 < n; a2++) {
			const double target = phi.back()*a2/n;
			while(phi[i+1] < target) i++;
			const double f = (target - phi[i])/(phi[i+1] - phi[i]);
			row[a2] = addPoint(cx[i] + f*(cx[i+1] - cx[i]), cy[i] + f*(cy[i+1] - cy[i])); rs[a2] = ib0 + i + f;
			const int q = addPoint(m.coords[2*row[a2]], -m.coords[2*row[a2]+1]);
			mir[row[a2]] = q; mir[q] = row[a2];
		}
		const size_t t0 = m.nnode.size();
		zip(below, row);
		const size_t t1 = m.nnode.size();
		for(size_t t = t0; t < t1; t++) {                      // the upper half: mirrored, orientation restored
			const int* e = &m.inpoel[4*t];
			tri(mir[e[0]], mir[e[2]], mir[e[1]]);
		}
		below.swap(row); bs.swap(rs);
	}
	m.npoin = static_cast<int>(m.coords.size()/2);
	m.nnofa = 2; m.nbtag = 2; m.ndtag = 2;
	m.nelem = static_cast<int>(m.nnode.size());
	m.maxnnode = 4; m.maxnfael = 4;
	m.vol_regions.assign(static_cast<size_t>(m.nelem)*2, 1);
	auto bf = [&](int a, int b, int tag) { m.bface.insert(m.bface.end(), {a, b, tag, 1}); };
	for(int i = ib0; i < ib1; i++) bf(P(i,0), P(i+1,0), 2);
	for(int i = 0; i < ib0; i++) bf(P(i+1,nl), P(i,nl), 4);
	for(size_t a = 0; a + 1 < below.size(); a++) { bf(below[a+1], below[a], 4); bf(mir[below[a]], mir[below[a+1]], 4); }
	for(int i = ib1; i < ni - 1; i++) bf(P(i+1,nl), P(i,nl), 4);
	for(int j = 0; j < nl; j++) { bf(P(0,j+1), P(0,j), 4); bf(P(ni-1,j), P(ni-1,j+1), 4); }
	m.nbface = static_cast<int>(m.bface.size()/4);
	return m;
}

MeshData generateCylinderOgrid(int ntheta, int nr, double r0, double r1)
{
	MeshData m;
	m.npoin = ntheta*(nr+1);
	m.coords.resize(static_cast<size_t>(m.npoin)*2);
	const double PI = 3.14159265358979323846;
	const double q = std::pow(r1/r0, 1.0/nr);          // geometric radial spacing
	for(int j = 0; j <= nr; j++) {
		const double r = r0*std::pow(q, j);
		for(int i = 0; i < ntheta; i++) {
			const double a = 2.0*PI*i/ntheta;
			const size_t p = static_cast<size_t>(j)*ntheta + i;
			m.coords[2*p] = r*std::cos(a); m.coords[2*p+1] = r*std::sin(a);
		}
	}
	addOgridCells(m, ntheta, 0, nr, 0);
	finishOgrid(m, ntheta, nr, 2, 4);
	return m;
}

MeshData generateFlatPlate(int nx, int ny, double xlead, double h, double wallspacing)
{
	MeshData m;
	m.npoin = (nx+1)*(ny+1);
	m.coords.resize(static_cast<size_t>(m.npoin)*2);
	// x: uniform-ish with clustering at the leading edge x=0
	std::vector<double> xs(nx+1), ys(ny+1);
	const int nlead = std::max(1, nx/8);
	for(int i = 0; i <= nlead; i++) xs[i] = -xlead*(1.0 - static_cast<double>(i)/nlead);
	for(int i = nlead; i <= nx; i++) {
		const double s = static_cast<double>(i - nlead)/(nx - nlead);
		xs[i] = s*s*(3.0 - 2.0*s)*0.0 + s;                 // uniform on the plate
	}
	double lo = 1.0 + 1e-12, hi = 2.0;
	for(int it = 0; it < 200; it++) {
		const double q = 0.5*(lo+hi);
		const double s = wallspacing*(std::pow(q, ny) - 1.0)/(q - 1.0);
		if(s > h) hi = q; else lo = q;
	}
	const double q = 0.5*(lo+hi);
	ys[0] = 0; double d = wallspacing;
	for(int j = 1; j <= ny; j++) { ys[j] = ys[j-1] + d; d *= q; }
	for(int j = 0; j <= ny; j++) ys[j] *= h/ys[ny];
	for(int j = 0; j <= ny; j++)
		for(int i = 0; i <= nx; i++) {
			const size_t p = static_cast<size_t>(j)*(nx+1) + i;
			m.coords[2*p] = xs[i]; m.coords[2*p+1] = ys[j];
		}
	auto P = [&](int i, int j) { return j*(nx+1) + i; };
	for(int j = 0; j < ny; j++)
		for(int i = 0; i < nx; i++) {
			m.inpoel.insert(m.inpoel.end(), {P(i,j), P(i+1,j), P(i+1,j+1), P(i,j+1)});
			m.nnode.push_back(4); m.nfael.push_back(4);
		}
	m.nelem = nx*ny; m.maxnnode = 4; m.maxnfael = 4; m.nnofa = 2; m.nbtag = 2; m.ndtag = 2;
	m.vol_regions.assign(static_cast<size_t>(m.nelem)*2, 1);
	auto addb = [&](int a, int b, int tag) { m.bface.insert(m.bface.end(), {a, b, tag, 1}); };
	for(int i = 0; i < nx; i++) addb(P(i,0), P(i+1,0), xs[i] < 0.0 ? 3 : 2);     // bottom
	for(int j = 0; j < ny; j++) addb(P(nx,j), P(nx,j+1), 5);                   // right (outflow)
	for(int i = nx; i > 0; i--) addb(P(i,ny), P(i-1,ny), 4);                   // top
	for(int j = ny; j > 0; j--) addb(P(0,j), P(0,j-1), 5);                     // left (inflow)
	m.nbface = static_cast<int>(m.bface.size()/4);
	return m;
}

}
