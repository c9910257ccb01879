/** \file ctx.hpp
 * \brief The library handle (struct fvhip_ctx behind include/fvhip.h's fvhip_handle): device mesh,
 *   state scratch, residual stages with the halo exchange, Jacobian and matrix-free operator, and the
 *   work space of the implicit solver (implicit.cpp). Shared by fvhip_api.cpp and implicit.cpp.
 * No exception crosses the ABI: entry points wrap their bodies in guard().
 */
#ifndef FVHIP_CTX_HPP
#define FVHIP_CTX_HPP

#include "../../include/fvhip.h"
#include "layout.hpp"
#include "kernels.hpp"
#include "jacobian.hpp"
#include "mesh.hpp"
#include "partition.hpp"
#include "halo.hpp"
#include "ode.hpp"
#include "surface.hpp"
#include "amg.hpp"
#include <rccl/rccl.h>
#include <hip/hip_runtime.h>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <string>
#include <vector>
#include <map>
#include <stdexcept>
#include <memory>
#include <functional>
#include <array>
#include <deque>
#include <numeric>

#include "krylov.hpp"

namespace fvhip_detail {

inline thread_local std::string g_err;      ///< fvhip_last_error() text, shared by every TU

struct HipError : std::runtime_error { using std::runtime_error::runtime_error; };

inline void hipCheck(hipError_t e, const char* what) {
	if(e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}
#define HC(x) hipCheck((x), #x)

inline void ncclCheck(ncclResult_t e, const char* what) {
	if(e != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(e));
}
#define NC(x) ncclCheck((x), #x)

template <typename F>
inline int guard(F&& f) {
	try { f(); return 0; }
	catch(const std::exception& e) { g_err = e.what(); return 1; }
	catch(...) { g_err = "unknown error"; return 1; }
}

/// entry-point argument check: a null handle or a null array the call reads or writes is refused
/// with "null <what>" before any host or device access (a null device pointer would fault the GPU)
inline void need(const void* p, const char* what) {
	if(!p) throw std::invalid_argument(std::string("null ") + what);
}

/// the same for a group call's per-rank arrays: the array of pointers and each rank's entry
template <typename T>
inline void needEach(T* const* p, size_t n, const char* what) {
	need(p, what);
	for(size_t i = 0; i < n; i++) need(p[i], what);
}

template <typename T>
inline T* upload(const std::vector<T>& v, std::vector<void*>& owned) {
	if(v.empty()) return nullptr;
	void* p = nullptr;
	HC(hipMalloc(&p, v.size()*sizeof(T)));
	HC(hipMemcpy(p, v.data(), v.size()*sizeof(T), hipMemcpyHostToDevice));
	owned.push_back(p);
	return static_cast<T*>(p);
}

inline double* dalloc(size_t n, std::vector<void*>& owned) {
	if(n == 0) n = 1;
	void* p = nullptr;
	HC(hipMalloc(&p, n*sizeof(double)));
	owned.push_back(p);
	return static_cast<double*>(p);
}

/// interleave int pairs / 4-tuples for vector loads
inline std::vector<int> pack2(const std::vector<int>& a, const std::vector<int>& b) {
	std::vector<int> o(2*a.size());
	for(size_t i = 0; i < a.size(); i++) { o[2*i] = a[i]; o[2*i+1] = b[i]; }
	return o;
}

}

using namespace fvhip;
using namespace fvhip_detail;

struct fvhip_ctx
{
	int device = 0;
	hipStream_t stream = nullptr;
	fvhip_flow_config cfg{};
	std::vector<int> bc_type, bc_tag;
	std::vector<double> bc_vals;
	Layout L;
	DevMesh M{};
	DevPhys P{};
	std::vector<void*> owned;
	int* d_perm = nullptr;
	// state scratch
	double *d_u = nullptr, *d_up = nullptr, *d_grad = nullptr, *d_lgrad = nullptr, *d_phi = nullptr;
	double *d_ubc = nullptr, *d_ug = nullptr, *d_r = nullptr, *d_dtm = nullptr;
	// mat-free state
	double *d_mf_u = nullptr, *d_mf_r = nullptr, *d_mf_mdt = nullptr, *d_mf_aux = nullptr, *d_mf_y = nullptr;
	double mf_eps = 1e-7;
	const double *mf_u = nullptr, *mf_r = nullptr, *mf_mdt = nullptr;   // device state of the operator
	double *d_part = nullptr, *d_pm = nullptr;
	double *d_rn_part = nullptr, *d_rn = nullptr;   // residual-norm reduction of the explicit driver
	double* d_ustage = nullptr;                      // TVD Runge-Kutta stage state (owned rows)
	double* d_ent = nullptr;                        // entropy-error partial sums (fvhip_entropy_error_device)
	/// work space of the implicit solver (implicit.cpp), allocated on first use
	struct ImplicitWork {
		int m = 0;                                  ///< GMRES restart length the basis holds
		double* V = nullptr;                        ///< Krylov basis [m+1][4*ncell]
		double *z = nullptr, *aux = nullptr;        ///< [4*(ncell+nghost)]: operator inputs (ghost rows)
		double *w = nullptr, *t = nullptr, *s = nullptr, *du = nullptr, *yg = nullptr;   ///< [4*ncell]
		double *jd = nullptr, *jlo = nullptr, *jup = nullptr, *dinv = nullptr;            ///< 4x4 blocks
		float *slo = nullptr, *sup = nullptr, *sdinv = nullptr;   ///< fp32 copies for the preconditioner
		float* sdiag = nullptr;                     ///< fp32 diagonal blocks (the multigrid's finest residuals)
		double *part = nullptr, *red = nullptr, *coef = nullptr, *pm = nullptr;           ///< reductions
		double *h_red = nullptr, *h_coef = nullptr, *h_red2 = nullptr;                  ///< pinned host
	} iw;
	std::vector<void*> owned_host;                  ///< pinned host allocations
	// Jacobian
	JacMesh J{};
	bool jac_ready = false;
	double *d_jb = nullptr, *d_jlo = nullptr, *d_jup = nullptr, *d_jdiag = nullptr;
	/// reference-order rows of the host-pointer entries (fvhip_compute_residual & co.): the host array is
	/// copied as it is and reordered on the device (k_gather / k_scatter over d_perm)
	double* d_raw = nullptr;
	size_t raw_cap = 0;
	double* rawScratch(size_t doubles) {
		if(raw_cap < doubles) {
			if(d_raw) { HC(hipStreamSynchronize(stream)); release(d_raw); }   // no transfer still reading it
			d_raw = dalloc(doubles, owned);
			raw_cap = doubles;
		}
		return d_raw;
	}
	// partitioned meshes: halo exchange with the neighbour ranks (RCCL, or in-process for a group)
	int rank = 0, nparts = 1;
	bool rankmesh = false;        ///< one rank's subdomain with connectivity faces (fvhip_create, nconnface > 0)
	bool use_staged = false;      ///< force the staged (gradient + sweep) path even if fused applies
	bool use_pipe = false;        ///< force the pipelined staged path even if fused applies
	// pipelined staged residual (single domain): the sweep groups run on stream2 behind the
	// gradient chunks of `stream`
	int* d_pipe_patch = nullptr;
	hipStream_t stream2 = nullptr;
	std::vector<hipEvent_t> pipe_ev;
	hipEvent_t pipe_start = nullptr, pipe_done = nullptr;
	ncclComm_t comm = nullptr;
	bool in_group = false;
	// halo exchange overlapped with the interior patches of the fused residual (RCCL handles)
	int* d_fz_order = nullptr;
	hipStream_t comm_stream = nullptr;
	hipEvent_t ev_u = nullptr, ev_halo = nullptr;
	hipEvent_t ev_packed = nullptr, ev_copied = nullptr;   ///< in-process overlapped transport (groups)
	bool copied_recorded = false;
	int* d_send = nullptr;
	int* d_border = nullptr;
	int nborder = 0;
	double* d_sendbuf = nullptr;
	int* d_trace_conn = nullptr;     ///< per-rank meshes: Layout::trace_conn on the device
	double* d_tracebuf = nullptr;    ///< [nghost][4] received face traces before the unpack
	int nsend = 0;
	// profiling
	bool prof = false;
	struct Rec { std::string name; hipEvent_t a, b; };
	std::vector<Rec> recs;
	std::map<std::string, std::pair<double,int>> acc;

	~fvhip_ctx() {
		(void)hipSetDevice(device);
		if(comm) (void)ncclCommDestroy(comm);
		for(auto& r : recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
		for(hipEvent_t e : pipe_ev) (void)hipEventDestroy(e);
		if(pipe_start) (void)hipEventDestroy(pipe_start);
		if(pipe_done) (void)hipEventDestroy(pipe_done);
		if(stream2) (void)hipStreamDestroy(stream2);
		if(ev_u) (void)hipEventDestroy(ev_u);
		if(ev_halo) (void)hipEventDestroy(ev_halo);
		if(ev_packed) (void)hipEventDestroy(ev_packed);
		if(ev_copied) (void)hipEventDestroy(ev_copied);
		if(comm_stream) (void)hipStreamDestroy(comm_stream);
		for(void* p : owned) (void)hipFree(p);
		for(void* p : owned_host) (void)hipHostFree(p);
		if(stream) (void)hipStreamDestroy(stream);
	}

	template <typename F>
	void timed(const std::string& name, F&& launch) { timed_on(stream, name, launch); }
	template <typename F>
	void timed_on(hipStream_t st, const std::string& name, F&& launch) {
		if(!prof) { launch(); return; }
		Rec r; r.name = name;
		HC(hipEventCreate(&r.a)); HC(hipEventCreate(&r.b));
		HC(hipEventRecord(r.a, st));
		launch();
		HC(hipEventRecord(r.b, st));
		recs.push_back(r);
	}
	void collect() {
		HC(hipStreamSynchronize(stream));
		for(auto& r : recs) {
			float ms = 0;
			HC(hipEventElapsedTime(&ms, r.a, r.b));
			auto& a = acc[r.name]; a.first += ms; a.second += 1;
			(void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b);
		}
		recs.clear();
	}

	/// kernels of the selected numerics mode (exact: bitwise parity; fast: stated tolerance)
#define KOPS(fn) (cfg.fast_math ? fast::fn : exact::fn)
	int recKind() const {
		if(!cfg.order2) return SR_FIRST;
		return cfg.reconstruction == FVHIP_REC_VANALBADA ? SR_MUSCL : SR_LINEAR;
	}
	int viscKind() const {
		if(!cfg.viscous_sim) return SV_NONE;
		return cfg.const_visc ? SV_CONST : SV_SUTHERLAND;
	}

	bool halo() const { return !L.nbr_rank.empty(); }
	int ntotal() const { return L.ncell + L.nghost; }

	// --- residual stages (FlowFV::compute_residual, flow_spatial.cpp:636-816); between them the
	// ghost rows of u, of the gradients and of limiter data are exchanged on partitioned meshes ---
	void stage_gradients(const double* u) {
		if(L.nghost > 0)
			timed("k_ghost_prim", [&]{ launch_cons2prim_rows(P.gas, u, d_up, L.ncell, L.nghost, stream); });
		if(cfg.gradientscheme == FVHIP_GRAD_LEASTSQUARES) {
			// limited reconstructions: the limiter values come out of the same kernel
			const int lim = fusedLimiter() ? (cfg.reconstruction == FVHIP_REC_VENKATAKRISHNAN ? 2 : 1) : 0;
			timed("k_prep_grad_wls", [&]{ KOPS(launch_prep_grad_wls)(M, P, u, d_up, d_ubc, d_ug, d_grad, stream, 0, -1,
			                                                         lim, d_phi); });
		} else {
			timed("k_prep", [&]{ KOPS(launch_prep)(M, P, u, d_up, d_ubc, d_ug, true, stream); });
			if(cfg.gradientscheme == FVHIP_GRAD_GREENGAUSS)
				timed("k_grad_gg", [&]{ KOPS(launch_grad_gg)(M, d_up, d_ug, d_grad, stream); });
			else KOPS(launch_fill)(d_grad, 0.0, 8LL*ntotal(), stream);
		}
	}
	bool limited() const {
		return cfg.reconstruction == FVHIP_REC_BARTHJESPERSEN || cfg.reconstruction == FVHIP_REC_VENKATAKRISHNAN;
	}
	/// WLS gradients compute the limiter in the same pass (k_prep_grad_wls<LIM>)
	bool fusedLimiter() const { return limited() && cfg.gradientscheme == FVHIP_GRAD_LEASTSQUARES; }
	void stage_limiter() {
		if(fusedLimiter()) return;
		const int venk = cfg.reconstruction == FVHIP_REC_VENKATAKRISHNAN;
		timed("k_limiter", [&]{ KOPS(launch_limiter)(M, P, venk, d_up, d_ug, d_grad, d_phi, stream); });
	}
	void stage_weno() { timed("k_weno", [&]{ KOPS(launch_weno)(M, P, d_grad, d_lgrad, stream); }); }
	void stage_sweep(const double* u, double* r, bool dt, double* dtm, bool overwrite,
	                 const int* plist = nullptr, int pcount = 0, hipStream_t st = nullptr) {
		if(!st) st = stream;
		const int rk = recKind();
		SweepBuffers B{};
		B.u = u; B.r = r; B.dtm = dtm; B.overwrite = overwrite ? 1 : 0;
		B.plist = plist; B.pcount = pcount;
		if(rk != SR_FIRST) {
			B.up = d_up; B.grad = d_grad; B.rgrad = d_grad; B.ubc = d_ubc; B.ug = d_ug;
			if(limited()) B.phi = d_phi;
			if(cfg.reconstruction == FVHIP_REC_WENO) B.rgrad = d_lgrad;
		}
		const char* nm = nullptr;
		// name is only known after launch; record under a generic label then rename
		timed_on(st, "k_sweep", [&]{ nm = KOPS(launch_sweep)(M, P, B, cfg.conv_numflux, rk, viscKind(), dt, st); });
		if(prof && !recs.empty() && recs.back().name == "k_sweep" && nm) recs.back().name = nm;
		HC(hipGetLastError());
	}

	void stage_border_gradients(const double* u, hipStream_t st = nullptr) {
		if(!st) st = stream;
		timed_on(st, "k_grad_wls_list", [&]{ KOPS(launch_grad_wls_list)(M, P, u, d_border, nborder, d_grad, st); });
	}

	/// one-launch residual (WLS + MUSCL / unlimited linear, inviscid)
	bool fused() const { return !L.fz_ext_start.empty() && !use_staged && !use_pipe; }
	/// pipelined staged residual (single domain, WLS + MUSCL / unlimited linear, viscous too), on
	/// request only: on C4 it measured 0.55 ms against 0.46 ms for the serial staged path (the
	/// FP64-bound sweep groups and the HBM-bound gradient chunks slow each other down, and every
	/// group has its own tail)
	bool pipelined() const { return !L.pipe_cell_start.empty() && !halo() && !use_staged && use_pipe; }
	/// gradient chunks on `stream`; each sweep group on stream2 waits for the last chunk it reads.
	/// Same kernels and arithmetic as the staged path, so bitwise its result.
	void residual_pipelined(const double* u, double* r, bool dt, double* dtm, bool overwrite) {
		const int K = static_cast<int>(L.pipe_cell_start.size()) - 1;
		if(!stream2) {
			HC(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
			pipe_ev.resize(K);
			for(hipEvent_t& e : pipe_ev) HC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
			HC(hipEventCreateWithFlags(&pipe_start, hipEventDisableTiming));
			HC(hipEventCreateWithFlags(&pipe_done, hipEventDisableTiming));
		}
		HC(hipEventRecord(pipe_start, stream));          // everything the caller queued before
		HC(hipStreamWaitEvent(stream2, pipe_start, 0));
		for(int k = 0; k < K; k++) {
			timed("k_prep_grad_wls", [&]{
				KOPS(launch_prep_grad_wls)(M, P, u, d_up, d_ubc, d_ug, d_grad, stream, L.pipe_cell_start[k], L.pipe_cell_start[k+1], 0, nullptr);
			});
			HC(hipEventRecord(pipe_ev[k], stream));
		}
		for(int k = 0; k < K; k++) {
			const int n = L.pipe_group_start[k+1] - L.pipe_group_start[k];
			if(n == 0) continue;
			HC(hipStreamWaitEvent(stream2, pipe_ev[k], 0));
			stage_sweep(u, r, dt, dtm, overwrite, d_pipe_patch + L.pipe_group_start[k], n, stream2);
		}
		HC(hipEventRecord(pipe_done, stream2));
		HC(hipStreamWaitEvent(stream, pipe_done, 0));   // the residual completes on `stream`
	}
	void stage_fused(const double* u, double* r, bool dt, double* dtm, bool overwrite,
	                 const int* plist = nullptr, int pcount = 0, hipStream_t st = nullptr) {
		if(!st) st = stream;
		SweepBuffers B{};
		B.u = u; B.r = r; B.dtm = dtm; B.overwrite = overwrite ? 1 : 0;
		B.plist = plist; B.pcount = pcount;
		if(plist && pcount == 0) return;
		B.grad = d_grad;     // received gradients of ghost cells (partitioned meshes)
		if(limited()) B.phi = d_phi;   // layer-1 ghosts' limiter values (two-layer halo)
		B.mfx = mfz.x; B.mfpm = mfz.pm; B.mfres = mfz.res; B.mfmdt = mfz.mdt;
		const char* nm = nullptr;
		timed_on(st, "k_residual_wls", [&]{ nm = KOPS(launch_residual_wls)(M, P, B, cfg.conv_numflux, recKind(), viscKind(),
		                                                                       limKind(), dt, st); });
		if(prof && !recs.empty() && recs.back().name == "k_residual_wls" && nm) recs.back().name = nm;
		HC(hipGetLastError());
	}

	/// the matrix-free operator fused into one launch of the residual kernel (single domain, fused
	/// configurations): y = mdt x + (r(u) - r(u + pm[1] x))/pm[1] with the perturbed state formed where the
	/// kernel reads a state row and the combination where it writes a cell -- k_mf_perturb's and
	/// k_mf_combine's arithmetic, so bitwise the three-launch operator, without its 5 vector passes over HBM
	struct MfFuse { const double *x = nullptr, *pm = nullptr, *res = nullptr, *mdt = nullptr; } mfz;
	/// (x and y must not alias: other blocks read x rows while a block writes its cells' y)
	bool matfreeFusable() const { return fused() && !halo(); }
	/// the fused operator's blocks read rows of x and of the state u that other blocks' cells need while each
	/// block writes its own cells of y: y must share no byte with x or u (else the three-launch operator runs)
	bool matfreeNoAlias(const double* u, const double* x, const double* y) const {
		const size_t n = 4*static_cast<size_t>(L.ncell), nt = 4*static_cast<size_t>(L.ncell + L.nghost);
		auto apart = [](const double* a, size_t na, const double* b, size_t nb) { return a + na <= b || b + nb <= a; };
		return apart(y, n, x, nt) && apart(y, n, u, nt);
	}
	void matfree_fused(const double* u, const double* x, const double* pm, const double* res, const double* mdt, double* y) {
		if(!matfreeFusable()) throw std::logic_error("matfree_fused: not a fused single-domain configuration");
		mfz = MfFuse{x, pm, res, mdt};
		try { stage_fused(u, y, false, nullptr, true); }
		catch(...) { mfz = MfFuse{}; throw; }
		mfz = MfFuse{};
	}

	/// pack the rows of `arr` (width doubles per cell) that the neighbours hold as ghosts
	void pack(const double* arr, int width, hipStream_t st = nullptr) {
		if(!st) st = stream;
		timed_on(st, "k_pack", [&]{ launch_pack_rows(d_send, nsend, arr, width, d_sendbuf, st); });
	}
	/// rows neighbour k sends / receives in an exchange of `layers` halo layers (a one-layer exchange
	/// of a two-layer halo moves the leading layer-1 part of each block)
	int sendCount(size_t k, int layers) const {
		return (layers >= 2 || L.send_l1_end.empty() ? L.send_start[k+1] : L.send_l1_end[k]) - L.send_start[k];
	}
	int ghostCount(size_t k, int layers) const {
		return (layers >= 2 || L.ghost_l1_end.empty() ? L.ghost_start[k+1] : L.ghost_l1_end[k]) - L.ghost_start[k];
	}
	/// L2TraceVector::updateSharedFacesBegin/End (tracevector.cpp:213-340) on a per-rank mesh: left
	/// [nconnface][width] holds this rank's face values of its connectivity faces (icface order); each
	/// neighbour's values of the same faces land in right[icface]. Packed in the exchange order (per
	/// neighbour rank, ascending global face), sent with RCCL, unpacked by face. width <= 4.
	void trace_pack(const double* left, int width, hipStream_t st) {
		if(L.trace_conn.empty()) throw std::logic_error("face-trace exchange: not a per-rank mesh (no connectivity faces)");
		if(width < 1 || width > 4) throw std::invalid_argument("face-trace exchange: width must be 1..4");
		timed_on(st, "k_pack", [&]{ launch_pack_rows(d_trace_conn, nsend, left, width, d_sendbuf, st); });
	}
	void trace_unpack(double* right, int width, hipStream_t st) {
		timed_on(st, "k_unpack", [&]{ launch_unpack_rows(d_trace_conn, L.nghost, d_tracebuf, width, right, st); });
	}
	void trace_exchange_rccl(const double* left, double* right, int width) {
		if(!comm) throw std::runtime_error("face-trace exchange: call fvhip_comm_init (or use a group) first");
		trace_pack(left, width, stream);
		NC(ncclGroupStart());
		for(size_t k = 0; k < L.nbr_rank.size(); k++) {
			const int q = L.nbr_rank[k];
			const size_t ns = static_cast<size_t>(L.send_start[k+1] - L.send_start[k]);
			const size_t ng = static_cast<size_t>(L.ghost_start[k+1] - L.ghost_start[k]);
			if(ns) NC(ncclSend(d_sendbuf + static_cast<size_t>(width)*L.send_start[k], width*ns, ncclDouble, q, comm, stream));
			if(ng) NC(ncclRecv(d_tracebuf + static_cast<size_t>(width)*L.ghost_start[k], width*ng, ncclDouble, q, comm, stream));
		}
		NC(ncclGroupEnd());
		trace_unpack(right, width, stream);
	}
	/// RCCL point-to-point exchange with every neighbour rank, on stream st (default: the handle's);
	/// `layers` 2 fills both layers of a two-layer halo (the residual's state), 1 the first (gradients,
	/// limiter values, Krylov vectors). Both sides derive the counts from the same lists, so a leg
	/// with nothing to move is skipped on both.
	void exchange_rccl(double* arr, int width, hipStream_t st = nullptr, int layers = 1) {
		if(!halo()) return;
		if(!comm) throw std::runtime_error("partitioned handle: call fvhip_comm_init (or use a group) first");
		if(!st) st = stream;
		pack(arr, width, st);
		NC(ncclGroupStart());
		for(size_t k = 0; k < L.nbr_rank.size(); k++) {
			const int q = L.nbr_rank[k];
			const size_t ns = static_cast<size_t>(sendCount(k, layers));
			const size_t ng = static_cast<size_t>(ghostCount(k, layers));
			if(ns) NC(ncclSend(d_sendbuf + static_cast<size_t>(width)*L.send_start[k], width*ns, ncclDouble, q, comm, st));
			if(ng) NC(ncclRecv(arr + static_cast<size_t>(width)*(L.ncell + L.ghost_start[k]), width*ng, ncclDouble, q, comm, st));
		}
		NC(ncclGroupEnd());
	}
	/// the residual's halo protocol: with a two-layer halo and WLS gradients of an unlimited, MUSCL,
	/// Barth-Jespersen or Venkatakrishnan reconstruction, ONE exchange of u (both layers) and the
	/// layer-1 ghosts' gradients (and limiter values) computed locally (k_grad_ghost); otherwise u,
	/// then gradients (and limiter data) in further rounds
	bool singleExchange() const {
		return halo() && L.halo_layers == 2 && cfg.order2 && cfg.gradientscheme == FVHIP_GRAD_LEASTSQUARES &&
		       cfg.reconstruction != FVHIP_REC_WENO && (L.gg_cells.empty() || !L.gg_V.empty());
	}
	int limKind() const { return limited() ? (cfg.reconstruction == FVHIP_REC_VENKATAKRISHNAN ? 2 : 1) : 0; }
	void stage_ghost_gradients(const double* u, hipStream_t st = nullptr) {
		if(!st) st = stream;
		timed_on(st, "k_grad_ghost", [&]{ KOPS(launch_grad_ghost)(M, P, u, d_grad, st, limKind(), d_phi); });
	}

	/// the second stream and events of the overlapped fused residual
	void ensureOverlap() {
		if(comm_stream) return;
		HC(hipStreamCreateWithFlags(&comm_stream, hipStreamNonBlocking));
		for(hipEvent_t* e : {&ev_u, &ev_halo, &ev_packed, &ev_copied}) HC(hipEventCreateWithFlags(e, hipEventDisableTiming));
	}

	/// The overlapped fused residual of a group held by one process (fvhip_group_*): the schedule of
	/// residual_fused_overlapped with the in-process transport placed on each handle's comm stream --
	/// pack, device copies that wait on the sender's pack, ghost gradients, halo event -- while the
	/// interior patches run on the handle's stream and the border patches wait for the halo event.
	/// The stream/event ordering and the send-buffer reuse of the RCCL path therefore run (and are
	/// checked bitwise against one GPU) with several ranks on one device, where RCCL cannot.
	static void residual_group_overlapped(std::vector<fvhip_ctx*>& hs, const std::vector<const double*>& us,
	                                      const std::vector<double*>& rs, bool dt, const std::vector<double*>& dts,
	                                      bool overwrite) {
		const size_t n = hs.size();
		std::vector<fvhip_ctx*> byrank(n, nullptr);
		for(fvhip_ctx* h : hs) {
			if(h->rank < 0 || h->rank >= static_cast<int>(n)) throw std::logic_error("group: ranks are not 0..n-1");
			byrank[h->rank] = h;
		}
		auto on = [&](size_t i) -> fvhip_ctx* { HC(hipSetDevice(hs[i]->device)); return hs[i]; };
		// 1. the comm stream takes u as the caller left it; a send buffer is refilled only after every
		//    receiver has copied the previous exchange out of it
		for(size_t i = 0; i < n; i++) {
			fvhip_ctx* h = on(i);
			h->ensureOverlap();
			HC(hipEventRecord(h->ev_u, h->stream));
			HC(hipStreamWaitEvent(h->comm_stream, h->ev_u, 0));
			for(fvhip_ctx* q : hs) if(q->copied_recorded) HC(hipStreamWaitEvent(h->comm_stream, q->ev_copied, 0));
			h->pack(us[i], 4, h->comm_stream);
			HC(hipEventRecord(h->ev_packed, h->comm_stream));
		}
		// 2. the patches that read no halo data
		for(size_t i = 0; i < n; i++)
			on(i)->stage_fused(us[i], rs[i], dt, dts[i], overwrite, hs[i]->d_fz_order, hs[i]->L.fz_ninner);
		// 3. receive both halo layers (copies wait on the sender's pack), layer-1 ghost gradients
		for(size_t i = 0; i < n; i++) {
			fvhip_ctx* h = on(i);
			const Layout& L = h->L;
			for(size_t k = 0; k < L.nbr_rank.size(); k++) {
				fvhip_ctx* q = byrank[L.nbr_rank[k]];
				const Layout& Q = q->L;
				size_t kk = 0;
				while(kk < Q.nbr_rank.size() && Q.nbr_rank[kk] != h->rank) kk++;
				if(kk == Q.nbr_rank.size()) throw std::logic_error("halo lists are not symmetric");
				const int cnt = h->ghostCount(k, 2);
				if(cnt != q->sendCount(kk, 2)) throw std::logic_error("halo sizes differ");
				if(cnt == 0) continue;
				HC(hipStreamWaitEvent(h->comm_stream, q->ev_packed, 0));
				HC(hipMemcpyAsync(const_cast<double*>(us[i]) + 4*static_cast<size_t>(L.ncell + L.ghost_start[k]),
				                  q->d_sendbuf + 4*static_cast<size_t>(Q.send_start[kk]),
				                  sizeof(double)*4*static_cast<size_t>(cnt), hipMemcpyDeviceToDevice, h->comm_stream));
			}
			h->stage_ghost_gradients(us[i], h->comm_stream);
			HC(hipEventRecord(h->ev_copied, h->comm_stream));
			// 4. the border patches on the comm stream right behind the halo (concurrent with the
			//    interior launch's tail, as in residual_fused_overlapped)
			h->stage_fused(us[i], rs[i], dt, dts[i], overwrite, h->d_fz_order + h->L.fz_ninner,
			               static_cast<int>(h->L.fz_order.size()) - h->L.fz_ninner, h->comm_stream);
			HC(hipEventRecord(h->ev_halo, h->comm_stream));
		}
		for(fvhip_ctx* h : hs) h->copied_recorded = true;
		// 5. the residual completes on each handle's stream; later work there (the next pack of a
		//    synchronous exchange included) also follows every copy out of its send buffer
		for(size_t i = 0; i < n; i++) {
			fvhip_ctx* h = on(i);
			HC(hipStreamWaitEvent(h->stream, h->ev_halo, 0));
			for(fvhip_ctx* q : hs) HC(hipStreamWaitEvent(h->stream, q->ev_copied, 0));
		}
	}

	/// fused residual of one RCCL rank: the halo exchange (ghost u, border gradients, ghost
	/// gradients) runs on comm_stream while the interior patches run on `stream`; the border patches
	/// are launched on comm_stream right behind the halo, so their blocks fill the interior launch's
	/// last partial wave instead of forming a fraction-of-a-wave launch after it. The two launches
	/// write disjoint cells; `stream` joins the comm stream before the residual is complete.
	/// (Round 4 also captured this step in a hipGraph; the capture of the RCCL p2p group overflows the stack
	/// inside the HIP runtime's graph code -- profiles/r05/graph_capture_crash.txt, DESIGN.md section 6 -- and
	/// the host enqueue, ~26 us against ~40 us of kernels per C4/8 rank step, keeps the step GPU-bound
	/// without it, so the path was removed.)
	void residual_fused_overlapped(const double* u, double* r, bool dt, double* dtm, bool overwrite) {
		ensureOverlap();
		double* uu = const_cast<double*>(u);
		HC(hipEventRecord(ev_u, stream));                 // u as the caller left it (and r, dtm free)
		HC(hipStreamWaitEvent(comm_stream, ev_u, 0));
		if(singleExchange()) {
			exchange_rccl(uu, 4, comm_stream, 2);
			stage_ghost_gradients(u, comm_stream);
		} else {
			exchange_rccl(uu, 4, comm_stream);
			stage_border_gradients(u, comm_stream);
			exchange_rccl(d_grad, 8, comm_stream);
		}
		stage_fused(u, r, dt, dtm, overwrite, d_fz_order, L.fz_ninner);
		stage_fused(u, r, dt, dtm, overwrite, d_fz_order + L.fz_ninner, static_cast<int>(L.fz_order.size()) - L.fz_ninner,
		            comm_stream);
		HC(hipEventRecord(ev_halo, comm_stream));
		HC(hipStreamWaitEvent(stream, ev_halo, 0));
	}

	/// the residual with the ghost rows of u already current (FVHIP_RES_HALO_READY): layer-1 ghost
	/// gradients (and limiter values), then every patch on the handle's stream
	void residual_halo_ready(const double* u, double* r, bool dt, double* dtm, bool overwrite) {
		if(!halo()) { residual(u, r, dt, dtm, overwrite); return; }
		if(!fused() || !singleExchange())
			throw std::runtime_error("FVHIP_RES_HALO_READY: only the fused single-exchange configurations (two-layer "
			                         "halo, WLS + MUSCL / linear / Barth-Jespersen / Venkatakrishnan)");
		stage_ghost_gradients(u);
		stage_fused(u, r, dt, dtm, overwrite, d_fz_order, static_cast<int>(L.fz_order.size()));
	}

	/// the device sweep: -r(u) added (or written) into r, time steps into dtm. On a partitioned
	/// mesh u must have room for the ghost rows (ncell+nghost rows), which this fills.
	void residual(const double* u, double* r, bool dt, double* dtm, bool overwrite) {
		std::vector<fvhip_ctx*> one{this};
		residual_seq(one, {u}, {r}, dt, {dtm}, overwrite, GroupExchange());
	}

	typedef std::function<double*(size_t)> ArrayOf;
	/// (array of each rank, row width, halo layers)
	typedef std::function<void(const ArrayOf&, int, int)> GroupExchange;

	static bool h0_single(const std::vector<fvhip_ctx*>& hs) { return hs[0]->singleExchange(); }
	/// The residual as a sequence of stages over one or several handles (several: the ranks of a
	/// partition held by one process, exchanging through device copies, see fvhip_group_*)
	static void residual_seq(std::vector<fvhip_ctx*>& hs, const std::vector<const double*>& us,
	                         const std::vector<double*>& rs, bool dt, const std::vector<double*>& dts,
	                         bool overwrite, const GroupExchange& exg) {
		auto exchange = [&](const ArrayOf& arr_of, int width, int layers = 1) {
			if(exg) { exg(arr_of, width, layers); return; }
			for(size_t i = 0; i < hs.size(); i++) { HC(hipSetDevice(hs[i]->device)); hs[i]->exchange_rccl(arr_of(i), width, nullptr, layers); }
		};
		const bool single = h0_single(hs);
		// every stage launches on the handle's own device (a group may span devices)
		auto on = [&](size_t i) -> fvhip_ctx* { HC(hipSetDevice(hs[i]->device)); return hs[i]; };
		fvhip_ctx* h0 = hs[0];
		if(hs.size() == 1 && !exg && h0->pipelined()) {
			h0->residual_pipelined(us[0], rs[0], dt, dts[0], overwrite);
			return;
		}
		if(h0->fused()) {
			if(h0->halo()) {
				if(hs.size() == 1 && !exg) { h0->residual_fused_overlapped(us[0], rs[0], dt, dts[0], overwrite); return; }
				if(single && exg) { residual_group_overlapped(hs, us, rs, dt, dts, overwrite); return; }
				// interior patches need no halo data: they run first, then the exchange of the ghost
				// rows of u and of the gradients of the cells other ranks hold as ghosts, then the rest
				for(size_t i = 0; i < hs.size(); i++)
					on(i)->stage_fused(us[i], rs[i], dt, dts[i], overwrite, hs[i]->d_fz_order, hs[i]->L.fz_ninner);
				if(single) {
					exchange([&](size_t i) { return const_cast<double*>(us[i]); }, 4, 2);
					for(size_t i = 0; i < hs.size(); i++) on(i)->stage_ghost_gradients(us[i]);
				} else {
					exchange([&](size_t i) { return const_cast<double*>(us[i]); }, 4);
					for(size_t i = 0; i < hs.size(); i++) on(i)->stage_border_gradients(us[i]);
					exchange([&](size_t i) { return hs[i]->d_grad; }, 8);
				}
				for(size_t i = 0; i < hs.size(); i++)
					on(i)->stage_fused(us[i], rs[i], dt, dts[i], overwrite, hs[i]->d_fz_order + hs[i]->L.fz_ninner,
					                   static_cast<int>(hs[i]->L.fz_order.size()) - hs[i]->L.fz_ninner);
				return;
			}
			for(size_t i = 0; i < hs.size(); i++) on(i)->stage_fused(us[i], rs[i], dt, dts[i], overwrite);
			return;
		}
		exchange([&](size_t i) { return const_cast<double*>(us[i]); }, 4, h0->L.halo_layers);
		if(h0->recKind() != SR_FIRST) {
			for(size_t i = 0; i < hs.size(); i++) on(i)->stage_gradients(us[i]);
			if(single) { for(size_t i = 0; i < hs.size(); i++) on(i)->stage_ghost_gradients(us[i]); }
			else exchange([&](size_t i) { return hs[i]->d_grad; }, 8);
			if(h0->limited() && !single) {      // single exchange: the ghosts' limiter values are local
				for(size_t i = 0; i < hs.size(); i++) on(i)->stage_limiter();
				exchange([&](size_t i) { return hs[i]->d_phi; }, 4);
			}
			if(h0->cfg.reconstruction == FVHIP_REC_WENO) {
				for(size_t i = 0; i < hs.size(); i++) on(i)->stage_weno();
				exchange([&](size_t i) { return hs[i]->d_lgrad; }, 8);
			}
		}
		for(size_t i = 0; i < hs.size(); i++) on(i)->stage_sweep(us[i], rs[i], dt, dts[i], overwrite);
	}

	/// face-ordered mesh view and block buffers for the Jacobian, built on first use
	void ensureJacobian() {
		const int jf = cfg.conv_numflux_jac;
		if(jf == FVHIP_FLUX_VANLEER) throw std::runtime_error(" ! VanLeerFlux: Not implemented!");   // anumericalflux.cpp:253-257
		if(jf == FVHIP_FLUX_AUSMPLUS) throw std::runtime_error(" ! AUSMPlusFlux: Not implemented!"); // :556-560
		if(jf < 0 || jf > 6) throw std::invalid_argument("unknown Jacobian flux");
		for(int i = 0; i < cfg.nbc; i++)
			if(bc_type[i] == FVHIP_BC_SUBSONIC_INFLOW)   // InFlow::computeGhostStateAndJacobian, abc.cpp:178-185
				throw std::runtime_error("subsonic inflow BC has no Jacobian (Not implemented!)");
		if(jac_ready) return;
		auto& o = owned;
		J.ncell = L.ncell; J.nbface = L.nbface; J.ninface = L.ninface;
		J.if_LR = reinterpret_cast<const int2*>(upload(pack2(L.if_L, L.if_R), o));
		J.if_n = reinterpret_cast<const double2*>(upload(L.if_n, o));
		J.if_len = upload(L.if_len, o);
		J.bf_L = M.bf_L; J.bf_bc = M.bf_bc; J.bf_n = M.bf_n; J.bf_rcbp = M.bf_rcbp; J.rc = M.rc;
		J.bf_len = upload(L.bf_len, o);
		J.cell_rfaces = reinterpret_cast<const int4*>(upload(L.cell_rfaces, o));
		J.cell_nbr_fo = M.cell_nbr_fo;
		d_jb = dalloc(16*static_cast<size_t>(std::max(L.nbface,1)), o);
		jac_ready = true;
	}

	/// Spatial::assemble_jacobian into (diag internal order, lower/upper reference face order); with
	/// cfl > 0 also the pseudo-time term (SteadyBackwardEulerSolver, aodesolver.cpp:300-329, 467) in the
	/// diagonal pass: dtm <- area/(cfl dtm), diag += dtm I
	void assemble(const double* u, double* diag, double* lower, double* upper, double cfl = 0.0, double* dtm = nullptr) {
		ensureJacobian();
		timed("k_jac_faces", [&]{ launch_jac_faces(J, P, cfg.conv_numflux_jac, viscKind(), u, d_jb, lower, upper, stream); });
		timed("k_jac_diag", [&]{ launch_jac_diag(J, d_jb, lower, upper, diag, stream, cfl > 0 ? M.area : nullptr, cfl, dtm); });
		HC(hipGetLastError());
	}

	/// reduction scratch of the device drivers (global sums, GMRES coefficients)
	void ensureReductions() {
		if(iw.red) return;
		auto& o = owned;
		iw.red = dalloc(KRY_MAXK + 2, o); iw.coef = dalloc(KRY_MAXK + 2, o); iw.pm = dalloc(2, o);
		iw.part = dalloc(kry_scratch(2), o);
		for(double** hp : {&iw.h_red, &iw.h_coef, &iw.h_red2}) {
			void* p = nullptr;
			HC(hipHostMalloc(&p, (KRY_MAXK + 2)*sizeof(double), hipHostMallocDefault));
			owned_host.push_back(p);
			*hp = static_cast<double*>(p);
		}
	}
	/// operand buffers of the matrix-free operator and GMRES (ghost rows where an operator reads them)
	void ensureVectors() {
		ensureReductions();
		if(iw.z) return;
		const size_t N = static_cast<size_t>(L.ncell), NT = N + static_cast<size_t>(L.nghost);
		auto& o = owned;
		iw.z = dalloc(4*NT, o); iw.aux = dalloc(4*NT, o);
		iw.w = dalloc(4*N, o); iw.t = dalloc(4*N, o); iw.s = dalloc(4*N, o); iw.du = dalloc(4*N, o);
		iw.yg = dalloc(4*N, o);
	}
	/// implicit-solver work space for GMRES(m): the above, the Jacobian blocks and the Krylov basis
	void ensureImplicit(int m) {
		ensureJacobian();
		if(m < 1) throw std::invalid_argument("GMRES restart length must be positive");
		ensureVectors();
		const size_t N = static_cast<size_t>(L.ncell);
		const size_t Fi = static_cast<size_t>(std::max(L.ninface, 1));
		auto& o = owned;
		if(m > KRY_MAXK) throw std::invalid_argument("GMRES restart length exceeds " + std::to_string(KRY_MAXK));
		if(!iw.jd) {
			iw.jd = dalloc(16*N, o); iw.jlo = dalloc(16*Fi, o); iw.jup = dalloc(16*Fi, o); iw.dinv = dalloc(16*N, o);
		}
		if(iw.m < m) {                  // a larger basis: the old one stays owned until destroy
			iw.V = dalloc(4*N*static_cast<size_t>(m + 1), o);
			iw.part = dalloc(kry_scratch(m + 2), o);
			iw.m = m;
		}
	}

	/// the boundary faces of one marker for the surface functionals, uploaded on first use
	struct SurfCache { SurfaceFaces S{}; double *faceout = nullptr, *contrib = nullptr, *sums = nullptr; };
	std::map<int, SurfCache> surf;
	SurfCache& surfaceFaces(int marker) {
		auto it = surf.find(marker);
		if(it != surf.end()) return it->second;
		std::vector<int> Lc;
		std::vector<double> geo;
		for(int f = 0; f < L.nbface; f++) {
			if(L.bf_tag[f] != marker) continue;
			Lc.push_back(L.bf_L[f]);
			const double g5[5] = {L.bf_n[2*f], L.bf_n[2*f+1], L.bf_len[f], L.bf_gr[2*f], L.bf_gr[2*f+1]};
			geo.insert(geo.end(), g5, g5 + 5);
		}
		SurfCache c;
		c.S.n = static_cast<int>(Lc.size());
		if(c.S.n > 0) {
			c.S.L = upload(Lc, owned);
			c.S.geo = upload(geo, owned);
			c.faceout = dalloc(4*Lc.size(), owned);
			c.contrib = dalloc(4*Lc.size(), owned);
		}
		c.sums = dalloc(4, owned);
		return surf.emplace(marker, c).first->second;
	}

	/// multicolour block Gauss-Seidel (fvhip_implicit_config::prec_gs): greedy colouring of the owned
	/// cells in internal (Hilbert) order over interior faces; ghost cells are not coloured (within a
	/// sweep they hold the values of the last exchange)
	std::vector<int> gs_colour_start;
	std::vector<int> gs_colour;          ///< colour of every owned cell (also the ILU(0) order)
	long long gs_triples = 0;            ///< owned cells sharing faces pairwise three at a time (ILU(0) fill off the diagonal)
	int* d_gs_cells = nullptr;
	int* d_gs_colour = nullptr;
	void ensureColouring() {
		if(d_gs_cells) return;
		const int N = L.ncell;
		auto nbr = [&](int c, int j) {        // owned neighbour across interior face j of c, else -1
			const int code = L.cell_rfaces[4*static_cast<size_t>(c)+j];
			if(code < 0 || (code >> 1) < L.nbface) return -1;
			const int nb = L.cell_nbr_fo[4*static_cast<size_t>(c)+j];
			return (nb >= 0 && nb < N) ? nb : -1;
		};
		gs_triples = 0;
		for(int c = 0; c < N; c++)
			for(int j = 0; j < 4; j++) {
				const int a = nbr(c, j);
				if(a <= c) continue;
				for(int k = j + 1; k < 4; k++) {
					const int b = nbr(c, k);
					if(b <= c) continue;
					for(int m = 0; m < 4; m++) if(nbr(a, m) == b) gs_triples++;
				}
			}
		std::vector<int> col(static_cast<size_t>(N), -1);
		int ncol = 0;
		for(int c = 0; c < N; c++) {
			unsigned long long used = 0;
			for(int j = 0; j < 4; j++) {
				const int code = L.cell_rfaces[4*static_cast<size_t>(c)+j];
				if(code < 0 || (code >> 1) < L.nbface) continue;
				const int nb = L.cell_nbr_fo[4*static_cast<size_t>(c)+j];
				if(nb >= 0 && nb < N && col[nb] >= 0) used |= 1ull << col[nb];
			}
			int k = 0;
			while(used & (1ull << k)) k++;
			col[c] = k;
			ncol = std::max(ncol, k + 1);
		}
		gs_colour_start.assign(static_cast<size_t>(ncol) + 1, 0);
		for(int c = 0; c < N; c++) gs_colour_start[col[c] + 1]++;
		for(int k = 0; k < ncol; k++) gs_colour_start[k+1] += gs_colour_start[k];
		std::vector<int> cells(static_cast<size_t>(std::max(N, 1)));
		std::vector<int> pos(gs_colour_start.begin(), gs_colour_start.end() - 1);
		for(int c = 0; c < N; c++) cells[pos[col[c]]++] = c;   // ascending within a colour
		d_gs_cells = upload(cells, owned);
		d_gs_colour = upload(col, owned);
		gs_colour = std::move(col);
	}
	/// block ILU(0) factorisation in colour order (fvhip_implicit_config::prec_ilu): dinv = the inverted
	/// pivot blocks Dt^-1, colour after colour (each colour reads the earlier colours' pivots)
	void iluFactor(const double* diag, const double* lower, const double* upper, double* dinv, hipStream_t st = nullptr) {
		if(!st) st = stream;
		ensureColouring();
		const int nc = static_cast<int>(gs_colour_start.size()) - 1;
		timed_on(st, "k_ilu_factor", [&]{
			for(int q = 0; q < nc; q++) {
				const int b = gs_colour_start[q], n = gs_colour_start[q+1] - b;
				launch_ilu_factor_colour(L.ncell, L.nbface, J.cell_rfaces, J.cell_nbr_fo, d_gs_colour, q, diag, lower, upper,
				                         dinv, d_gs_cells + b, n, st);
			}
		});
	}

	/// lines of the line-implicit preconditioner (fvhip_implicit_config::prec_lines), built on first use
	/// from the mesh: coupling of a cell to a neighbour across an interior face = face length / centre
	/// distance (what dominates the Jacobian blocks of thin cells). A cell is anisotropic if its
	/// strongest coupling is at least `thr` times its weakest; lines start at the most anisotropic
	/// unassigned cell and grow at both ends through the end cell's strongest unassigned owned
	/// neighbour while that neighbour is anisotropic and the link is one of its own two strongest
	/// (Mavriplis' line construction); every other cell is a line of one. Lines are sorted by length
	/// so that a wave's threads walk lines of similar length.
	LineSet lines{};
	double lines_thr = -1.0;
	std::vector<int> h_line_start, h_line_cells, h_line_faces;   ///< the lines in line order (fvhip_lines)
	void ensureLines(double thr) {
		if(!(thr >= 0.0) || !std::isfinite(thr)) throw std::invalid_argument("line_threshold must be finite and >= 0 (0: 4)");
		if(thr == 0.0) thr = 4.0;
		if(lines.gstart && lines_thr == thr) return;
		// a rebuild (another threshold) releases the previous line set's device arrays
		for(const void* p : {static_cast<const void*>(lines.gstart), static_cast<const void*>(lines.cell),
		                     static_cast<const void*>(lines.face), static_cast<const void*>(lines.D),
		                     static_cast<const void*>(lines.Lb), static_cast<const void*>(lines.W),
		                     static_cast<const void*>(lines.len),
		                     static_cast<const void*>(lines.G), static_cast<const void*>(lines.zpart)}) release(p);
		lines = LineSet{};
		const int N = L.ncell, nb = L.nbface;
		struct Nb { int c, fi; double w; };
		std::vector<std::array<Nb,4>> nbr(static_cast<size_t>(N));
		std::vector<int> nn(static_cast<size_t>(N), 0);
		std::vector<double> ratio(static_cast<size_t>(N), 1.0);
		for(int c = 0; c < N; c++) {
			double wmax = 0, wmin = INFINITY;
			for(int j = 0; j < 4; j++) {
				const int code = L.cell_rfaces[4*static_cast<size_t>(c)+j];
				if(code < 0 || (code >> 1) < nb) continue;           // boundary face
				const int fi = (code >> 1) - nb;
				const int o = L.cell_nbr_fo[4*static_cast<size_t>(c)+j];
				const double dx = L.rc[2*static_cast<size_t>(c)] - L.rc[2*static_cast<size_t>(o)];
				const double dy = L.rc[2*static_cast<size_t>(c)+1] - L.rc[2*static_cast<size_t>(o)+1];
				const double w = L.if_len[fi]/std::sqrt(dx*dx + dy*dy);
				wmax = std::max(wmax, w); wmin = std::min(wmin, w);
				if(o < N) nbr[c][nn[c]++] = Nb{o, fi, w};
			}
			std::sort(nbr[c].begin(), nbr[c].begin() + nn[c], [](const Nb& a, const Nb& b) {
				return a.w > b.w || (a.w == b.w && a.c < b.c); });
			if(wmin < INFINITY && wmin > 0) ratio[c] = wmax/wmin;
		}
		auto strong2 = [&](int c, int o) {               // o among c's two strongest owned neighbours
			for(int j = 0; j < std::min(nn[c], 2); j++) if(nbr[c][j].c == o) return true;
			return false;
		};
		std::vector<int> order(static_cast<size_t>(N));
		std::iota(order.begin(), order.end(), 0);
		std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return ratio[a] > ratio[b]; });
		std::vector<char> used(static_cast<size_t>(N), 0);
		std::vector<std::vector<std::pair<int,int>>> all;   // (cell, face to previous) per line
		for(const int c0 : order) {
			if(used[c0]) continue;
			used[c0] = 1;
			std::deque<std::pair<int,int>> line{{c0, -1}};
			if(ratio[c0] >= thr) {
				for(int dir = 0; dir < 2; dir++) {
					int e = dir == 0 ? line.back().first : line.front().first;
					for(;;) {
						int nxt = -1, fi = -1;
						for(int j = 0; j < std::min(nn[e], 2); j++) {
							const Nb& b = nbr[e][j];
							if(!used[b.c]) { nxt = b.c; fi = b.fi; break; }
						}
						if(nxt < 0 || ratio[nxt] < thr || !strong2(nxt, e)) break;
						used[nxt] = 1;
						if(dir == 0) line.push_back({nxt, fi});
						else {                              // prepend: the face now links nxt to e
							line.front().second = fi;
							line.push_front({nxt, -1});
						}
						e = nxt;
					}
				}
			}
			// lines longer than LINE_MAX_CELLS are cut into pieces: the recurrence along a line is
			// sequential, so one line of thousands of cells (circumferential lines of the outer O-grid
			// layers) would set the whole sweep's time
			for(size_t b = 0; b < line.size(); b += LINE_MAX_CELLS) {
				const size_t e = std::min(line.size(), b + static_cast<size_t>(LINE_MAX_CELLS));
				std::vector<std::pair<int,int>> piece(line.begin() + b, line.begin() + e);
				piece[0].second = -1;
				all.push_back(std::move(piece));
			}
		}
		// longest first; lines of equal length in ascending internal (Hilbert) order of their first cell, so
		// that the 64 lanes of a group walk neighbouring lines side by side: their k-th cells' rows of v and
		// z share 128-byte lines (the cells are gathered by index), instead of 64 unrelated places of the mesh.
		// Each line's recurrence is independent of the lane it runs on: the same z bit for bit.
		std::stable_sort(all.begin(), all.end(), [](const std::vector<std::pair<int,int>>& a,
		                                            const std::vector<std::pair<int,int>>& b) {
			return a.size() > b.size() || (a.size() == b.size() && a[0].first < b[0].first); });
		// lanes: a line of at least LINE_TWIST_MIN cells is solved from both ends (twisted factorisation):
		// its top half t = (n-1)/2 cells in order, then the twist cell t, on lane j of a twisted group; its
		// bottom half n-1 .. t+1 in reverse order, then t, on lane j+32. Every other line is one lane of a
		// group of 64. Entries (cell, interior face to the previous entry); rows line-interleaved
		// (krylov.hpp LineSet)
		const int nl = static_cast<int>(all.size());
		int ntw = 0;
		while(ntw < nl && static_cast<int>(all[static_cast<size_t>(ntw)].size()) >= LINE_TWIST_MIN) ntw++;
		typedef std::vector<std::pair<int,int>> Lane;
		std::vector<std::array<Lane,64>> grp;
		for(int l0 = 0; l0 < ntw; l0 += 32) {
			grp.emplace_back();
			for(int q = 0; q < 32 && l0 + q < ntw; q++) {
				const auto& ln = all[static_cast<size_t>(l0 + q)];
				const int n = static_cast<int>(ln.size()), tc = (n - 1)/2;
				Lane top(ln.begin(), ln.begin() + tc + 1), bot;
				for(int k = n - 1; k >= tc; k--)
					bot.push_back({ln[static_cast<size_t>(k)].first, k == n - 1 ? -1 : ln[static_cast<size_t>(k) + 1].second});
				grp.back()[static_cast<size_t>(q)] = std::move(top);
				grp.back()[static_cast<size_t>(q) + 32] = std::move(bot);
			}
		}
		const int ntg = static_cast<int>(grp.size());
		for(int l0 = ntw; l0 < nl; l0 += 64) {
			grp.emplace_back();
			for(int q = 0; q < 64 && l0 + q < nl; q++) grp.back()[static_cast<size_t>(q)] = all[static_cast<size_t>(l0 + q)];
		}
		const int ng = static_cast<int>(grp.size());
		std::vector<int> gst(static_cast<size_t>(ng) + 1, 0);
		for(int g = 0; g < ng; g++) {
			size_t mx = 0;
			for(const Lane& ln : grp[static_cast<size_t>(g)]) mx = std::max(mx, ln.size());
			gst[g+1] = gst[g] + static_cast<int>(mx);
		}
		const size_t nslot = 64*static_cast<size_t>(gst[ng]);
		std::vector<int> cells(std::max<size_t>(nslot, 1), -1), faces(std::max<size_t>(nslot, 1), -1);
		std::vector<int> lens(std::max<size_t>(64*static_cast<size_t>(ng), 1), 0);
		for(int g = 0; g < ng; g++)
			for(size_t lane = 0; lane < 64; lane++) {
				const Lane& ln = grp[static_cast<size_t>(g)][lane];
				lens[64*static_cast<size_t>(g) + lane] = static_cast<int>(ln.size());
				for(size_t k = 0; k < ln.size(); k++) {
					const size_t slot = (static_cast<size_t>(gst[g]) + k)*64 + lane;
					cells[slot] = ln[k].first;
					if(k > 0) {
						const int fi = ln[k].second, p = ln[k-1].first;
						faces[slot] = (fi << 1) | (L.if_L[fi] == p ? 0 : 1);
					}
				}
			}
		// the lines as built (fvhip_lines), longest first
		h_line_start.assign(1, 0);
		h_line_cells.clear(); h_line_faces.clear();
		for(const auto& ln : all) {
			for(size_t k = 0; k < ln.size(); k++) {
				h_line_cells.push_back(ln[k].first);
				h_line_faces.push_back(k > 0 ? (ln[k].second << 1) | (L.if_L[ln[k].second] == ln[k-1].first ? 0 : 1) : -1);
			}
			h_line_start.push_back(static_cast<int>(h_line_cells.size()));
		}
		lines.twisted_groups = ntg;
		lines.nlines = nl;
		lines.ngroups = ng;
		lines.nrows = gst[ng];
		lines.gstart = upload(gst, owned);
		lines.cell = upload(cells, owned);
		lines.face = upload(faces, owned);
		lines.len = upload(lens, owned);
		const size_t rows = std::max<size_t>(static_cast<size_t>(gst[ng]), 1);
		lines.D = dalloc(1024*rows, owned);
		// zeroed once: in a twisted group the factorisation writes the twist row of D for lane j only
		// (the pivot); k_line_solve's forward prefetch also requests that row for lane j+32 and discards
		// it, so it must hold defined values, never garbage a later change could start using
		HC(hipMemsetAsync(lines.D, 0, sizeof(double)*1024*rows, stream));
		lines.Lb = dalloc(1024*rows, owned);
		lines.W = dalloc(1024*rows, owned);
		lines.G = dalloc(256*rows, owned);
		lines.zpart = dalloc(static_cast<size_t>(std::max(ng, 1)), owned);
		lines_thr = thr;
	}

	/// aggregation multigrid hierarchy (fvhip_implicit_config::prec_amg), built on first use from the mesh:
	/// the finest level's graph is the owned cells over interior faces with couplings face length / centre
	/// distance (ghost couplings dropped: block-Jacobi across ranks), its block indices those of the
	/// face-ordered Jacobian (diag c, lower N + fi, upper N + Fi + fi); coarsening stops at `levels` levels
	/// or when a level has fewer than 64 rows or shrinks by less than 1.25
	std::vector<AmgLevel> amg;
	int amg_levels = 0;
	double amg_thr = -1.0;
	void ensureAmg(int levels, double thr) {
		if(levels < 2) throw std::invalid_argument("prec_amg: at least 2 levels");
		if(!(thr >= 0.0 && thr < 1.0)) throw std::invalid_argument("amg_threshold must be in [0, 1)");
		if(amg_levels == levels && amg_thr == thr) return;
		if(!amg.empty()) throw std::runtime_error("prec_amg: the hierarchy is built once per handle (same levels and threshold)");
		const int N = L.ncell, nb = L.nbface, Fi = L.ninface;
		AmgGraph g;
		g.n = N;
		g.rowptr.assign(static_cast<size_t>(N) + 1, 0);
		g.dblk.resize(static_cast<size_t>(N));
		std::vector<std::array<double,3>> row;          // (column, coupling, block)
		for(int c = 0; c < N; c++) {
			g.dblk[c] = c;
			row.clear();
			for(int j = 0; j < 4; j++) {
				const int code = L.cell_rfaces[4*static_cast<size_t>(c)+j];
				if(code < 0 || (code >> 1) < nb) continue;
				const int o = L.cell_nbr_fo[4*static_cast<size_t>(c)+j];
				if(o < 0 || o >= N) continue;
				const int fi = (code >> 1) - nb;
				const double dx = L.rc[2*static_cast<size_t>(c)] - L.rc[2*static_cast<size_t>(o)];
				const double dy = L.rc[2*static_cast<size_t>(c)+1] - L.rc[2*static_cast<size_t>(o)+1];
				const int blk = (code & 1) ? N + fi : N + Fi + fi;     // A[c][o]: c = R reads lower, c = L upper
				row.push_back({static_cast<double>(o), L.if_len[fi]/std::sqrt(dx*dx + dy*dy), static_cast<double>(blk)});
			}
			std::sort(row.begin(), row.end());
			for(const auto& r : row) {
				g.col.push_back(static_cast<int>(r[0])); g.w.push_back(r[1]); g.blk.push_back(static_cast<int>(r[2]));
			}
			g.rowptr[c+1] = static_cast<int>(g.col.size());
		}
		for(int l = 1; l < levels; l++) {
			if(g.n < 64) break;
			AmgLevelHost H = amgCoarsen(g, thr);
			if(H.n*5 > g.n*4) break;                         // shrinks by less than 1.25: stop
			AmgLevel D;
			D.n = H.n; D.nnz = H.rowptr[H.n]; D.nfine = g.n;
			D.rowptr = upload(H.rowptr, owned); D.col = upload(H.col, owned); D.dpos = upload(H.dpos, owned);
			D.cstart = upload(H.cstart, owned); D.csrc = upload(H.csrc, owned);
			D.mstart = upload(H.mstart, owned); D.members = upload(H.members, owned); D.agg = upload(H.agg, owned);
			D.cells = upload(H.cells, owned); D.cstart_colour = H.cstart_colour;
			D.d_cstart_colour = upload(H.cstart_colour, owned);
			D.val = dalloc(16*static_cast<size_t>(D.nnz), owned); D.dinv = dalloc(16*static_cast<size_t>(D.n), owned);
			D.x = dalloc(4*static_cast<size_t>(D.n), owned); D.b = dalloc(4*static_cast<size_t>(D.n), owned);
			D.r = dalloc(4*static_cast<size_t>(D.n), owned);
			amg.push_back(D);
			g = amgGraphOf(H);
		}
		if(amg.empty()) throw std::runtime_error("prec_amg: the mesh does not coarsen");
		amg_levels = levels;
		amg_thr = thr;
	}
	/// Galerkin operators of every coarse level from the finest blocks, and their diagonal inverses
	void amgSetup(const double* diag, const double* lower, const double* upper) {
		timed("k_amg_galerkin", [&]{
			for(size_t l = 0; l < amg.size(); l++) {
				if(l == 0) launch_amg_galerkin_fine(amg[0], L.ncell, L.ninface, diag, lower, upper, stream);
				else launch_amg_galerkin(amg[l], amg[l-1].val, stream);
				launch_amg_invert(amg[l], stream);
			}
		});
	}

	/// frees one device array of `owned` before the handle's destruction
	void release(const void* p) {
		if(!p) return;
		auto it = std::find(owned.begin(), owned.end(), p);
		if(it == owned.end()) throw std::logic_error("release: not a buffer of this handle");
		(void)hipFree(*it);
		owned.erase(it);
	}

	/// fp32 copies of the preconditioner blocks (fvhip_implicit_config::prec_single)
	void ensureSinglePrecond() {
		if(iw.sdinv) return;
		const size_t N = static_cast<size_t>(L.ncell);
		const size_t Fi = static_cast<size_t>(std::max(L.ninface, 1));
		iw.sdinv = reinterpret_cast<float*>(dalloc(8*N, owned));
		iw.slo = reinterpret_cast<float*>(dalloc(8*Fi, owned));
		iw.sup = reinterpret_cast<float*>(dalloc(8*Fi, owned));
		iw.sdiag = reinterpret_cast<float*>(dalloc(8*N, owned));
	}

	/// MatrixFreeSpatialJacobian::apply on device vectors (internal order), single domain (the
	/// partitioned operator is sys_matfree, implicit.cpp)
	void matfree(const double* x, double* y) {
		if(!mf_u || !mf_r || !mf_mdt) throw std::runtime_error("matrix-free operator: state not set");
		if(halo()) throw std::logic_error("fvhip_ctx::matfree is the single-domain operator (partitioned: sysMatfree)");
		const size_t N = static_cast<size_t>(L.ncell);
		if(!d_part) { d_part = dalloc(mf_partials(), owned); d_pm = dalloc(2, owned); }
		if(!d_mf_aux) { d_mf_aux = dalloc(4*N, owned); d_mf_y = dalloc(4*N, owned); }
		timed("k_mf_norm", [&]{ launch_mf_norm(4LL*L.ncell, x, mf_eps, d_part, d_pm, stream); });
		if(matfreeFusable() && matfreeNoAlias(mf_u, x, y)) { matfree_fused(mf_u, x, d_pm, mf_r, mf_mdt, y); HC(hipGetLastError()); return; }
		timed("k_mf_perturb", [&]{ launch_mf_perturb(4LL*L.ncell, mf_u, x, d_pm, d_mf_aux, stream); });
		residual(d_mf_aux, d_mf_y, false, nullptr, true);
		timed("k_mf_combine", [&]{ launch_mf_combine(L.ncell, mf_mdt, x, d_mf_y, mf_r, d_pm, y, stream); });
		HC(hipGetLastError());
	}
};

/// all ranks of one partition driven from one process (fvhip_group_*)
struct fvhip_group_s { std::vector<fvhip_ctx*> hs; };

namespace fvhip_detail {
/// in-process halo transport of a group: pack on every rank, then device copies into the ghost blocks
fvhip_ctx::GroupExchange groupExchange(const fvhip_group_s* g);
/// MatrixFreeSpatialJacobian::apply over all ranks of a partition (global |x|), implicit.cpp
void sysMatfree(const std::vector<fvhip_ctx*>& hs, const fvhip_ctx::GroupExchange& exg,
                const std::vector<const double*>& x, const std::vector<double*>& y);
}

#endif
