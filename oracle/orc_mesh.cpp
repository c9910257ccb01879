/** \file orc_mesh.cpp
 * \brief ORACLE (test infrastructure only): literal restatement of the FVENS mesh pipeline.
 * See orc_mesh.hpp for the reference lines.
 */
#include "orc_mesh.hpp"
#include <fstream>
#include <cmath>
#include <algorithm>
#include <stdexcept>
#include <iterator>
#include <map>

namespace orc {

OMesh orc_readGmsh2(const std::string& mfile)
{
	OMesh m;
	int dum; double dummy; std::string dums; char ch;
	std::ifstream infile(mfile);
	if(!infile) throw std::runtime_error("cannot open " + mfile);
	for(int i = 0; i < 4; i++)
		do ch = static_cast<char>(infile.get()); while(ch != '\n');
	infile >> m.npoin;
	m.coords.resize(2*static_cast<size_t>(m.npoin));
	for(int i = 0; i < m.npoin; i++) {
		infile >> dum;
		for(int j = 0; j < 2; j++) infile >> m.coords[2*i+j];
		infile >> dummy;
	}
	infile >> dums; infile >> dums;
	const int width_elms = 25;
	int nelm, elmtype, nbtags, ntags;
	m.ndtag = 0; m.nbtag = 0;
	infile >> nelm;
	std::vector<int> elms(static_cast<size_t>(nelm)*width_elms, 0);
	m.nbface = 0; m.nelem = 0;
	std::vector<int> nnodes(nelm,0), nfaels(nelm,0);
	auto E = [&](int i, int j) -> int& { return elms[static_cast<size_t>(i)*width_elms+j]; };
	for(int i = 0; i < nelm; i++) {
		infile >> dum; infile >> elmtype;
		if(elmtype == 1) {
			m.nnofa = 2; infile >> nbtags;
			if(nbtags > m.nbtag) m.nbtag = nbtags;
			for(int j = 0; j < nbtags; j++) infile >> E(i,j+m.nnofa);
			for(int j = 0; j < m.nnofa; j++) infile >> E(i,j);
			m.nbface++;
		} else if(elmtype == 2 || elmtype == 3) {
			nnodes[i] = elmtype == 2 ? 3 : 4; nfaels[i] = nnodes[i]; m.nnofa = 2;
			infile >> ntags;
			if(ntags > m.ndtag) m.ndtag = ntags;
			for(int j = 0; j < ntags; j++) infile >> E(i,j+nnodes[i]);
			for(int j = 0; j < nnodes[i]; j++) infile >> E(i,j);
			m.nelem++;
		} else throw std::runtime_error("oracle reader: only linear edges/tris/quads");
	}
	m.maxnnode = nnodes[m.nbface]; m.maxnfael = nfaels[m.nbface];
	for(int i = 0; i < nelm; i++) {
		if(nnodes[i] > m.maxnnode) m.maxnnode = nnodes[i];
		if(nfaels[i] > m.maxnfael) m.maxnfael = nfaels[i];
	}
	const int bw = m.nnofa+m.nbtag;
	m.bface.resize(static_cast<size_t>(m.nbface)*bw);
	m.inpoel.resize(static_cast<size_t>(m.nelem)*m.maxnnode);
	for(int i = 0; i < m.nbface; i++) {
		for(int j = 0; j < m.nnofa; j++) m.bface[i*bw+j] = E(i,j)-1;
		for(int j = m.nnofa; j < bw; j++) m.bface[i*bw+j] = E(i,j);
	}
	for(int i = 0; i < m.nelem; i++) {
		for(int j = 0; j < nnodes[i+m.nbface]; j++) m.inpoel[static_cast<size_t>(i)*m.maxnnode+j] = E(i+m.nbface,j)-1;
		for(int j = nnodes[i+m.nbface]; j < m.maxnnode; j++) m.inpoel[static_cast<size_t>(i)*m.maxnnode+j] = -1;
		m.nnode.push_back(nnodes[i+m.nbface]);
		m.nfael.push_back(nfaels[i+m.nbface]);
	}
	return m;
}

OMesh orc_fromRaw(int npoin, const double* coords, int nelem, int maxnnode, const int* inpoel,
                  const int* nnode, int nbface, int nbtag, const int* bface)
{
	OMesh m;
	m.npoin = npoin; m.nelem = nelem; m.maxnnode = maxnnode; m.nbface = nbface; m.nbtag = nbtag;
	m.nnofa = 2;
	m.coords.assign(coords, coords + 2*static_cast<size_t>(npoin));
	m.inpoel.assign(inpoel, inpoel + static_cast<size_t>(nelem)*maxnnode);
	m.nnode.assign(nnode, nnode+nelem);
	m.nfael = m.nnode;
	m.maxnfael = maxnnode;
	m.bface.assign(bface, bface + static_cast<size_t>(nbface)*(2+nbtag));
	return m;
}

namespace {

// mesh.cpp:425-465
void esupCompute(OMesh& m)
{
	m.esup_p.assign(m.npoin+1, 0);
	for(int i = 0; i < m.nelem; i++)
		for(int j = 0; j < m.nfael[i]; j++) m.esup_p[m.in(i,j)+1] += 1;
	for(int i = 1; i < m.npoin+1; i++) m.esup_p[i] += m.esup_p[i-1];
	m.esup.assign(m.esup_p[m.npoin], 0);
	for(int i = 0; i < m.nelem; i++)
		for(int j = 0; j < m.nfael[i]; j++) {
			const int ipoin = m.in(i,j);
			m.esup[m.esup_p[ipoin]] = i;
			m.esup_p[ipoin] += 1;
		}
	for(int i = m.npoin; i >= 1; i--) m.esup_p[i] = m.esup_p[i-1];
	m.esup_p[0] = 0;
}

// mesh.cpp:543-606 (getFaceEIndex for a physical boundary face)
int faceEIndex(const OMesh& m, int iface, int lelem)
{
	const int bw = m.nnofa+m.nbtag;
	for(int ifael = 0; ifael < m.nfael[lelem]; ifael++) {
		bool facefound = true;
		for(int inofa = 0; inofa < m.nnofa; inofa++) {
			const int node = m.in(lelem, (ifael + inofa) % m.nnode[lelem]);
			bool nodefound = false;
			for(int jnofa = 0; jnofa < m.nnofa; jnofa++)
				if(m.bface[iface*bw+jnofa] == node) { nodefound = true; break; }
			if(!nodefound) { facefound = false; break; }
		}
		if(facefound) return ifael;
	}
	return -1;
}

// mesh.cpp:608-657
std::vector<std::pair<int,int>> phyBFaceNeighbours(const OMesh& m)
{
	const int bw = m.nnofa+m.nbtag;
	std::vector<std::pair<int,int>> interiorelem(m.nbface);
	for(int iface = 0; iface < m.nbface; iface++) {
		std::vector<std::vector<int>> nbdelems(m.nnofa);
		for(int j = 0; j < m.nnofa; j++) {
			const int point = m.bface[iface*bw+j];
			for(int k = m.esup_p[point]; k < m.esup_p[point+1]; k++) nbdelems[j].push_back(m.esup[k]);
			std::sort(nbdelems[j].begin(), nbdelems[j].end());
		}
		std::vector<int> inter(nbdelems[0]);
		for(int j = 1; j < m.nnofa; j++) {
			std::vector<int> tmp;
			std::set_intersection(nbdelems[j].begin(), nbdelems[j].end(), inter.begin(), inter.end(),
			                      std::back_inserter(tmp));
			inter = tmp;
		}
		if(inter.size() > 1) throw std::logic_error("More than one neighboring element found for bface");
		interiorelem[iface].first = inter.at(0);
		interiorelem[iface].second = faceEIndex(m, iface, inter[0]);
	}
	return interiorelem;
}

// mesh.cpp:467-541
void esuelCompute(OMesh& m)
{
	m.esuel.assign(static_cast<size_t>(m.nelem)*m.maxnfael, -1);
	std::vector<int> lpoin(m.npoin, 0);
	const int nverfa = 2;
	for(int ielem = 0; ielem < m.nelem; ielem++) {
		for(int ifael = 0; ifael < m.nfael[ielem]; ifael++) {
			int lhelp[2];
			for(int i = 0; i < nverfa; i++) {
				lhelp[i] = m.in(ielem, (ifael+i) % m.nnode[ielem]);
				lpoin[lhelp[i]] = 1;
			}
			const int ipoin = lhelp[0];
			for(int istor = m.esup_p[ipoin]; istor < m.esup_p[ipoin+1]; istor++) {
				const int jelem = m.esup[istor];
				if(jelem != ielem) {
					for(int jfael = 0; jfael < m.nfael[jelem]; jfael++) {
						int icoun = 0;
						for(int jnofa = 0; jnofa < nverfa; jnofa++) {
							const int jpoin = m.in(jelem, (jfael+jnofa) % m.nfael[jelem]);
							if(lpoin[jpoin] == 1) icoun++;
						}
						if(icoun == nverfa) {
							m.esuel[static_cast<size_t>(ielem)*m.maxnfael+ifael] = jelem;
							m.esuel[static_cast<size_t>(jelem)*m.maxnfael+jfael] = ielem;
						}
					}
				}
			}
			for(int i = 0; i < nverfa; i++) lpoin[lhelp[i]] = 0;
		}
	}
}

}

void orc_preprocess(OMesh& m)
{
	const int bw = m.nnofa+m.nbtag;
	// correctBoundaryFaceOrientation (mesh.cpp:55-82)
	esupCompute(m);
	{
		const auto host = phyBFaceNeighbours(m);
		for(int iface = 0; iface < m.nbface; iface++) {
			const int he = host[iface].first, ef = host[iface].second;
			if(m.in(he, (ef+0) % m.nnode[he]) != m.bface[iface*bw+0] ||
			   m.in(he, (ef+1) % m.nnode[he]) != m.bface[iface*bw+1])
				std::swap(m.bface[iface*bw+0], m.bface[iface*bw+1]);
		}
	}
	m.nconnface = 0;
	m.connface.clear();
	orc_preprocess_rank(m);
}

void orc_preprocess_rank(OMesh& m)
{
	const int bw = m.nnofa+m.nbtag;
	// compute_topological (mesh.cpp:330-341) with the connectivity faces already in m.connface
	esupCompute(m);
	esuelCompute(m);
	m.ninface = 0;
	for(int ie = 0; ie < m.nelem; ie++)
		for(int in = 0; in < m.nfael[ie]; in++) {
			const int je = m.gesuel(ie,in);
			if(je > ie && je < m.nelem) m.ninface++;
		}
	m.naface = m.ninface + m.nbface + m.nconnface;
	m.intfac.assign(static_cast<size_t>(m.naface)*4, 0);
	m.elemface.assign(static_cast<size_t>(m.nelem)*m.maxnfael, 0);
	m.btags.assign(static_cast<size_t>(m.nbface)*m.nbtag, 0);
	const auto intelems = phyBFaceNeighbours(m);
	for(int iface = 0; iface < m.nbface; iface++) {
		m.intfac[4*iface+0] = intelems[iface].first;
		m.intfac[4*iface+1] = m.nelem + m.nconnface + iface;
		for(int inode = 0; inode < m.nnofa; inode++) m.intfac[4*iface+2+inode] = m.bface[iface*bw+inode];
		for(int j = m.nnofa; j < m.nnofa+m.nbtag; j++) m.btags[iface*m.nbtag+j-m.nnofa] = m.bface[iface*bw+j];
		m.esuel[static_cast<size_t>(intelems[iface].first)*m.maxnfael+intelems[iface].second] = m.nelem+m.nconnface+iface;
		m.elemface[static_cast<size_t>(intelems[iface].first)*m.maxnfael+intelems[iface].second] = iface;
	}
	int faceindex = m.nbface;
	for(int ie = 0; ie < m.nelem; ie++)
		for(int in = 0; in < m.nnode[ie]; in++) {
			const int je = m.gesuel(ie,in);
			if(je > ie && je < m.nelem) {
				const int in1 = (in+1) % m.nnode[ie];
				m.intfac[4*faceindex+0] = ie;
				m.intfac[4*faceindex+1] = je;
				m.intfac[4*faceindex+2] = m.in(ie,in);
				m.intfac[4*faceindex+3] = m.in(ie,in1);
				m.elemface[static_cast<size_t>(ie)*m.maxnfael+in] = faceindex;
				for(int jnode = 0; jnode < m.nnode[je]; jnode++)
					if(m.in(ie,in1) == m.in(je,jnode))
						m.elemface[static_cast<size_t>(je)*m.maxnfael+jnode] = faceindex;
				faceindex++;
			}
		}
	// connectivity faces (mesh.cpp:737-757)
	const int connBFaceStart = m.nbface + m.ninface;
	for(int iface = connBFaceStart; iface < m.naface; iface++) {
		const int icface = iface - connBFaceStart;
		const int inelem = m.gconnface(icface,0);
		m.intfac[4*iface+0] = inelem;
		m.esuel[static_cast<size_t>(inelem)*m.maxnfael+m.gconnface(icface,1)] = m.nelem+icface;
		m.elemface[static_cast<size_t>(inelem)*m.maxnfael+m.gconnface(icface,1)] = iface;
		m.intfac[4*iface+1] = m.nelem+icface;
		for(int inode = 0; inode < m.nnofa; inode++)
			m.intfac[4*iface+2+inode] = m.in(inelem, (m.gconnface(icface,1) + inode) % m.nnode[inelem]);
	}

	// compute_areas (mesh.cpp:290-313)
	auto c = [&](int p, int d) { return m.coords[2*static_cast<size_t>(p)+d]; };
	m.area.assign(m.nelem, 0);
	for(int i = 0; i < m.nelem; i++) {
		if(m.nnode[i] == 3)
			m.area[i] = 0.5*(c(m.in(i,0),0)*(c(m.in(i,1),1) - c(m.in(i,2),1)) - c(m.in(i,0),1)*(c(m.in(i,1),0)
				- c(m.in(i,2),0)) + c(m.in(i,1),0)*c(m.in(i,2),1) - c(m.in(i,2),0)*c(m.in(i,1),1));
		else if(m.nnode[i] == 4) {
			m.area[i] = 0.5*(c(m.in(i,0),0)*(c(m.in(i,1),1) - c(m.in(i,2),1)) - c(m.in(i,0),1)*(c(m.in(i,1),0)
				- c(m.in(i,2),0)) + c(m.in(i,1),0)*c(m.in(i,2),1) - c(m.in(i,2),0)*c(m.in(i,1),1));
			m.area[i] += 0.5*(c(m.in(i,0),0)*(c(m.in(i,2),1) - c(m.in(i,3),1)) - c(m.in(i,0),1)*(c(m.in(i,2),0)
				- c(m.in(i,3),0)) + c(m.in(i,2),0)*c(m.in(i,3),1) - c(m.in(i,3),0)*c(m.in(i,2),1));
		}
	}
	// compute_face_data (mesh.cpp:346-365)
	m.facemetric.assign(static_cast<size_t>(m.naface)*3, 0);
	for(int i = 0; i < m.naface; i++) {
		double* fm = &m.facemetric[3*static_cast<size_t>(i)];
		fm[0] = c(m.intfac[4*i+3],1) - c(m.intfac[4*i+2],1);
		fm[1] = -1.0*(c(m.intfac[4*i+3],0) - c(m.intfac[4*i+2],0));
		fm[2] = std::sqrt(std::pow(fm[0],2) + std::pow(fm[1],2));
		fm[0] /= fm[2];
		fm[1] /= fm[2];
	}
	// compute_cell_centres (mesh.cpp:316-328)
	m.rc.assign(static_cast<size_t>(m.nelem+m.nconnface)*2, 0);
	for(int i = 0; i < m.nelem; i++)
		for(int d = 0; d < 2; d++) {
			m.rc[2*i+d] = 0;
			for(int j = 0; j < m.nnode[i]; j++) m.rc[2*i+d] += c(m.in(i,j),d);
			m.rc[2*i+d] /= static_cast<double>(m.nnode[i]);
		}
	// aspatial.cpp:50-61
	m.gr.assign(static_cast<size_t>(m.naface)*2, 0);
	for(int f = 0; f < m.naface; f++) {
		for(int iv = 0; iv < m.nnofa; iv++)
			for(int d = 0; d < 2; d++) m.gr[2*f+d] += c(m.intfac[4*f+2+iv],d);
		for(int d = 0; d < 2; d++) m.gr[2*f+d] /= m.nnofa;
	}
	// aspatial.cpp:97-119
	m.rcbp.assign(static_cast<size_t>(m.nbface)*2, 0);
	for(int f = 0; f < m.nbface; f++) {
		const int ie = m.intfac[4*f];
		for(int d = 0; d < 2; d++) {
			double mid = 0;
			for(int k = 0; k < m.nnofa; k++) mid += c(m.intfac[4*f+2+k],d);
			mid /= m.nnofa;
			m.rcbp[2*f+d] = 2.0*mid - m.rc[2*ie+d];
		}
	}
}


// meshpartitioning.cpp:354-367
std::vector<int> orc_partition_trivial(int nelem, int nranks)
{
	const int numloceleminit = nelem / nranks;
	std::vector<int> elemdist(nelem);
	for(int irank = 0; irank < nranks; irank++)
		for(int iel = irank*numloceleminit; iel < (irank+1)*numloceleminit; iel++) elemdist[iel] = irank;
	for(int iel = nranks*numloceleminit; iel < nelem; iel++) elemdist[iel] = nranks-1;
	return elemdist;
}

// meshpartitioning.cpp:24-159, then preprocessMesh (ameshutils.cpp:40-99) and the ghost-row centres
// of the Spatial ctor's scatter (aspatial.cpp:41-66): the owner computes them from the same points in
// the same order as gm does
OMesh orc_restrict(const OMesh& gm, const std::vector<int>& elemdist, int rank)
{
	OMesh lm;
	lm.nelem = 0;
	for(int iel = 0; iel < gm.nelem; iel++) if(elemdist[iel] == rank) lm.nelem++;
	lm.maxnnode = gm.maxnnode; lm.maxnfael = gm.maxnfael; lm.nnofa = gm.nnofa;
	// 1. extractInpoel (:161-182)
	lm.inpoel.assign(static_cast<size_t>(lm.nelem)*gm.maxnnode, 0);
	lm.nfael.assign(lm.nelem, 0); lm.nnode.assign(lm.nelem, 0);
	lm.nbtag = gm.nbtag; lm.ndtag = gm.ndtag;
	lm.globalElemIndex.assign(lm.nelem, 0);
	{
		int lociel = 0;
		for(int iel = 0; iel < gm.nelem; iel++)
			if(elemdist[iel] == rank) {
				lm.globalElemIndex[lociel] = iel;
				for(int j = 0; j < gm.maxnnode; j++) lm.inpoel[static_cast<size_t>(lociel)*lm.maxnnode+j] = gm.in(iel,j);
				lm.nnode[lociel] = gm.nnode[iel];
				lm.nfael[lociel] = gm.nfael[iel];
				lociel++;
			}
	}
	// 2. extractPointCoords (:184-223)
	std::vector<int> locpoints;
	for(int iel = 0; iel < lm.nelem; iel++)
		for(int inode = 0; inode < lm.nnode[iel]; inode++) locpoints.push_back(lm.in(iel,inode));
	std::sort(locpoints.begin(), locpoints.end());
	locpoints.erase(std::unique(locpoints.begin(), locpoints.end()), locpoints.end());
	lm.npoin = static_cast<int>(locpoints.size());
	lm.coords.assign(2*static_cast<size_t>(lm.npoin), 0);
	std::map<int,int> g2l;
	for(int i = 0; i < lm.npoin; i++) g2l[locpoints[i]] = i;
	{
		int globpointer = 0, locpointer = 0;
		while(globpointer < gm.npoin && locpointer < lm.npoin) {
			if(globpointer == locpoints[locpointer]) {
				for(int i = 0; i < 2; i++) lm.coords[2*locpointer+i] = gm.coords[2*globpointer+i];
				locpointer++;
			}
			globpointer++;
		}
	}
	// 3. local point numbers (:66-69)
	for(int iel = 0; iel < lm.nelem; iel++)
		for(int j = 0; j < lm.nnode[iel]; j++)
			lm.inpoel[static_cast<size_t>(iel)*lm.maxnnode+j] = g2l.at(lm.in(iel,j));
	// 4. extractbfaces (:225-276)
	const int gbw = gm.nnofa+gm.nbtag;
	lm.nbface = 0;
	for(int iface = 0; iface < gm.nbface; iface++) {
		const int globelem = gm.L(iface);
		if(elemdist[globelem] != rank) continue;
		for(int j = 0; j < gm.nnofa; j++) lm.bface.push_back(g2l.at(gm.bface[iface*gbw+j]));
		for(int j = 0; j < gm.nbtag; j++) lm.bface.push_back(gm.bface[iface*gbw+gm.nnofa+j]);
		lm.nbface++;
	}
	// 5. (:79-82, 278-291)
	esupCompute(lm);
	esuelCompute(lm);
	std::vector<bool> isBounPoin(lm.npoin, false);
	const int lbw = lm.nnofa+lm.nbtag;
	for(int iface = 0; iface < lm.nbface; iface++)
		for(int inode = 0; inode < lm.nnofa; inode++) isBounPoin[lm.bface[iface*lbw+inode]] = true;
	// 6. getConnectivityFaceEIndices (:293-331) and the connface rows (:91-156)
	std::vector<std::vector<int>> connElemLocalFace(lm.nelem);
	for(int iel = 0; iel < lm.nelem; iel++)
		for(int iface = 0; iface < lm.nfael[iel]; iface++)
			if(lm.gesuel(iel,iface) == -1) {
				bool isconnface = false;
				for(int inode = 0; inode < lm.nnofa; inode++)
					if(!isBounPoin[lm.in(iel, (iface+inode) % lm.nnode[iel])]) { isconnface = true; break; }
				if(isconnface) connElemLocalFace[iel].push_back(iface);
			}
	lm.nconnface = 0;
	for(int i = 0; i < lm.nelem; i++) lm.nconnface += static_cast<int>(connElemLocalFace[i].size());
	lm.connface.assign(5*static_cast<size_t>(lm.nconnface), 0);
	int icofa = 0;
	for(int iel = 0; iel < lm.nelem; iel++)
		for(size_t iconface = 0; iconface < connElemLocalFace[iel].size(); iconface++) {
			const int localConnFace = connElemLocalFace[iel][iconface];
			int* c = &lm.connface[5*static_cast<size_t>(icofa)];
			c[0] = iel; c[1] = localConnFace; c[2] = -1; c[3] = -1;
			c[4] = gm.gelemface(lm.globalElemIndex[iel], localConnFace);
			std::vector<int> locfacepoints(lm.nnofa);
			for(int linofa = 0; linofa < lm.nnofa; linofa++)
				locfacepoints[linofa] = lm.in(iel, (localConnFace+linofa) % lm.nnode[iel]);
			const int glind = lm.globalElemIndex[iel];
			for(int jgf = 0; jgf < gm.nfael[glind]; jgf++) {
				bool matched = true;
				for(int jnofa = 0; jnofa < gm.nnofa; jnofa++) {
					const int globpoint = gm.in(glind, (jgf+jnofa) % gm.nnode[glind]);
					bool pointmatched = false;
					for(int linofa = 0; linofa < lm.nnofa; linofa++)
						if(locpoints[locfacepoints[linofa]] == globpoint) { pointmatched = true; break; }
					if(!pointmatched) { matched = false; break; }
				}
				if(matched) {
					c[2] = elemdist[gm.gesuel(glind,jgf)];
					c[3] = gm.gesuel(glind,jgf);
					break;
				}
			}
			if(c[2] < 0) throw std::logic_error("Could not find connectivity face!");
			icofa++;
		}
	orc_preprocess_rank(lm);
	for(int ic = 0; ic < lm.nconnface; ic++)
		for(int d = 0; d < 2; d++)
			lm.rc[2*(static_cast<size_t>(lm.nelem)+ic)+d] = gm.rc[2*static_cast<size_t>(lm.gconnface(ic,3))+d];
	return lm;
}

}
