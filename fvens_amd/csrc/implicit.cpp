/** \file implicit.cpp
 * \brief Device-resident pseudo-time solvers over one global system:
 *   SteadyForwardEulerSolver::solve (aodesolver.cpp:135-282) and SteadyBackwardEulerSolver::solve
 *   (aodesolver.cpp:363-638), plus the partitioned matrix-free operator.
 *
 * The reference hands each linear system to PETSc (KSPSolve, aodesolver.cpp:483; GMRES with a
 * block-Jacobi/ILU or SOR preconditioner from the .solverc files). Here it is solved on the device
 * by restarted GMRES: right-preconditioned (the residual it monitors is the true one), classical
 * Gram-Schmidt with selective (DGKS) re-orthogonalisation (one fused multi-dot reduction, i.e. one
 * small host round trip, per Arnoldi step in the common case, a second only when the projection
 * cancelled more than half of |w|^2; modified Gram-Schmidt would take j+1), preconditioned by
 * block-Jacobi sweeps on the assembled first-order Jacobian. PETSc's ILU/SOR are sequential
 * recurrences; a block-Jacobi sweep is one launch over all cells, and several sweeps approach the
 * block Gauss-Seidel effect. The matrix-free operator (alinalg.cpp:142-233) uses the assembled
 * blocks as preconditioner, as the reference's KSPSetOperators(A_mf, M) does (casesolvers.cpp:170).
 *
 * A system is either one handle (one GPU, or one rank of a partition with its RCCL communicator:
 * partial sums combined by ncclAllReduce) or all ranks of a partition driven from one process (a
 * group: halo rows by device copies, partial sums added on the host in handle order).
 */
#include "ctx.hpp"

#include <cmath>
#include <vector>

namespace fvhip_detail {

struct System
{
	std::vector<fvhip_ctx*> hs;
	fvhip_ctx::GroupExchange exg;        ///< in-process halo transport of a group, else empty

	size_t size() const { return hs.size(); }
	bool halo() const { return hs[0]->halo(); }
	template <typename F> void each(F&& f) {
		for(size_t i = 0; i < hs.size(); i++) { HC(hipSetDevice(hs[i]->device)); f(i, hs[i]); }
	}
	void exchange(const fvhip_ctx::ArrayOf& arr, int width) {
		if(!halo()) return;
		if(exg) { exg(arr, width, 1); return; }
		each([&](size_t i, fvhip_ctx* h) { h->exchange_rccl(arr(i), width); });
	}
	/// global sums of k values every handle left in its iw.red, needed on the device only: one handle
	/// reduces over its ranks in place (ncclAllReduce, or nothing on one GPU) without a host round trip;
	/// a group sums on the host (allsum)
	void allsumDevice(int k) {
		if(hs.size() == 1) {
			fvhip_ctx* h = hs[0];
			if(h->comm) { HC(hipSetDevice(h->device)); NC(ncclAllReduce(h->iw.red, h->iw.red, k, ncclDouble, ncclSum, h->comm, h->stream)); }
			return;
		}
		allsum(k, true);
	}
	/// global sums of the k values every handle left in its iw.red: returned on the host and, if
	/// to_device, present in every handle's iw.red afterwards
	std::vector<double> allsum(int k, bool to_device) {
		each([&](size_t, fvhip_ctx* h) {
			if(h->comm) NC(ncclAllReduce(h->iw.red, h->iw.red, k, ncclDouble, ncclSum, h->comm, h->stream));
			HC(hipMemcpyAsync(h->iw.h_red, h->iw.red, k*sizeof(double), hipMemcpyDeviceToHost, h->stream));
		});
		std::vector<double> tot(k, 0.0);
		each([&](size_t, fvhip_ctx* h) {
			HC(hipStreamSynchronize(h->stream));
			for(int j = 0; j < k; j++) tot[j] += h->iw.h_red[j];
		});
		if(hs.size() > 1 && to_device)
			each([&](size_t, fvhip_ctx* h) {
				std::copy(tot.begin(), tot.end(), h->iw.h_red);
				HC(hipMemcpyAsync(h->iw.red, h->iw.h_red, k*sizeof(double), hipMemcpyHostToDevice, h->stream));
			});
		return tot;
	}
	void sync() { each([&](size_t, fvhip_ctx* h) { HC(hipStreamSynchronize(h->stream)); }); }
	/// one handle: the global sums of the k values in iw.red, copied to iw.h_red2 behind the reduction
	/// without waiting (read them after a later wait on the stream)
	void allsumQueue(int k) {
		fvhip_ctx* h = hs[0];
		HC(hipSetDevice(h->device));
		if(h->comm) NC(ncclAllReduce(h->iw.red, h->iw.red, k, ncclDouble, ncclSum, h->comm, h->stream));
		HC(hipMemcpyAsync(h->iw.h_red2, h->iw.red, k*sizeof(double), hipMemcpyDeviceToHost, h->stream));
	}
};

typedef fvhip_ctx::ArrayOf ArrayOf;

/// MatrixFreeSpatialJacobian::apply (alinalg.cpp:142-233) over a system: |x| is the global norm,
/// the perturbed state gets its ghost rows from the residual's own exchange
/// have_norm: |x|^2 is already in iw.red (the line solve that produced x summed it, LinOp::precondition)
static void matfreeApply(System& S, const ArrayOf& x, const ArrayOf& y, bool have_norm = false)
{
	S.each([&](size_t i, fvhip_ctx* h) {
		if(!h->mf_u || !h->mf_r || !h->mf_mdt) throw std::runtime_error("matrix-free operator: state not set");
		if(!have_norm) launch_mdot(4LL*h->L.ncell, 0, nullptr, 0, x(i), true, h->iw.part, h->iw.red, h->stream);
	});
	if(!have_norm) S.allsumDevice(1);          // |x|^2 stays on the device (launch_pertmag reads it there)
	if(S.size() == 1 && !S.exg && S.hs[0]->matfreeFusable() && S.hs[0]->matfreeNoAlias(S.hs[0]->mf_u, x(0), y(0))) {
		// one launch: the perturbed state and the combination inside the residual kernel (bitwise the same)
		fvhip_ctx* h = S.hs[0];
		launch_pertmag(h->iw.red, h->mf_eps, h->iw.pm, h->stream);
		h->matfree_fused(h->mf_u, x(0), h->iw.pm, h->mf_r, h->mf_mdt, y(0));
		HC(hipGetLastError());
		return;
	}
	std::vector<const double*> aux;
	std::vector<double*> yg, none(S.size(), nullptr);
	S.each([&](size_t i, fvhip_ctx* h) {
		launch_pertmag(h->iw.red, h->mf_eps, h->iw.pm, h->stream);
		launch_mf_perturb(4LL*h->L.ncell, h->mf_u, x(i), h->iw.pm, h->iw.aux, h->stream);
		aux.push_back(h->iw.aux);
		yg.push_back(h->iw.yg);
	});
	fvhip_ctx::residual_seq(S.hs, aux, yg, false, none, true, S.exg);
	S.each([&](size_t i, fvhip_ctx* h) {
		launch_mf_combine(h->L.ncell, h->mf_mdt, x(i), h->iw.yg, h->mf_r, h->iw.pm, y(i), h->stream);
		HC(hipGetLastError());
	});
}

/// The linear operator and preconditioner of one implicit step
struct LinOp
{
	System& S;
	bool matfree = false;
	bool single = false;                      ///< preconditioner blocks in fp32 (iw.sdinv/slo/sup; line factors: LineSet::single)
	bool gs = false;                          ///< multicolour block Gauss-Seidel instead of Jacobi
	bool lines = false;                       ///< line-implicit (block-tridiagonal along lines)
	bool ilu = false;                         ///< block ILU(0) in multicolour order
	double line_thr = 0.0;
	int sweeps = 1;
	int amg = 0;                              ///< aggregation multigrid levels (0: one-level preconditioner)
	int amg_sweeps = 2, amg_coarse = 6, amg_fine = 2;
	double amg_thr = 0.2;
	std::vector<const double*> D, Lo, Up;     ///< per handle: diagonal / lower / upper blocks

	/// y = A x with the assembled blocks; x has ghost rows, which are filled here
	void blocks(const ArrayOf& x, const ArrayOf& y) {
		S.exchange(x, 4);
		S.each([&](size_t i, fvhip_ctx* h) {
			h->timed("k_block_apply", [&]{ launch_block_apply(h->J, D[i], Lo[i], Up[i], x(i), y(i), h->stream); });
		});
	}
	/// set by a precondition call asked for the norm of its output (the Arnoldi step's z), consumed by the
	/// next apply: the matrix-free operator needs |z| and the line solve summed it while writing z
	bool znorm = false;
	void apply(const ArrayOf& x, const ArrayOf& y) {
		const bool have = znorm;
		znorm = false;
		if(matfree) matfreeApply(S, x, y, have);
		else blocks(x, y);
	}
	/// z = M^-1 v: `sweeps` block-Jacobi sweeps on A z = v from z = 0 (z has ghost rows). The iterates
	/// alternate between z and aux (both with ghost rows) so that the last one lands in z.
	void precondition(const ArrayOf& v, const ArrayOf& z, bool want_norm = false) {
		znorm = false;
		if(amg) { amgApply(v, z); return; }
		if(gs) { gaussSeidel(v, z); return; }
		if(lines) { lineSweeps(v, z, want_norm); return; }
		if(ilu) { iluSweeps(v, z); return; }
		const ArrayOf aux = [&](size_t i) { return S.hs[i]->iw.aux; };
		auto buf = [&](int k) -> const ArrayOf& { return ((sweeps - 1 - k) % 2 == 0) ? z : aux; };
		S.each([&](size_t i, fvhip_ctx* h) {
			h->timed("k_bjac_apply", [&]{
				if(single) launch_bjac_apply(h->L.ncell, h->iw.sdinv, v(i), buf(0)(i), h->stream);
				else launch_bjac_apply(h->L.ncell, h->iw.dinv, v(i), buf(0)(i), h->stream);
			});
		});
		for(int k = 1; k < sweeps; k++) {
			const ArrayOf& zin = buf(k-1);
			const ArrayOf& zout = buf(k);
			S.exchange(zin, 4);
			S.each([&](size_t i, fvhip_ctx* h) {
				h->timed("k_bjac_sweep", [&]{
					if(single) launch_bjac_sweep(h->J, h->iw.sdinv, h->iw.slo, h->iw.sup, v(i), zin(i), zout(i), h->stream);
					else launch_bjac_sweep(h->J, h->iw.dinv, Lo[i], Up[i], v(i), zin(i), zout(i), h->stream);
				});
			});
		}
	}
	/// z = M^-1 v by `sweeps` multicolour block Gauss-Seidel sweeps from z = 0, colours in forward
	/// then backward order on alternate sweeps (symmetric Gauss-Seidel pairs). Across ranks the
	/// sweep is block-Jacobi: ghost rows are exchanged once per sweep -- the reference's PETSc
	/// setting -pc_type bjacobi -sub_pc_type sor, with a colour order instead of a row order.
	void gaussSeidel(const ArrayOf& v, const ArrayOf& z) {
		S.each([&](size_t i, fvhip_ctx* h) {
			exact::launch_fill(z(i), 0.0, 4LL*(h->L.ncell + h->L.nghost), h->stream);
		});
		for(int k = 0; k < sweeps; k++) {
			if(k > 0) S.exchange(z, 4);
			const bool fwd = (k % 2) == 0;
			S.each([&](size_t i, fvhip_ctx* h) {
				const int nc = static_cast<int>(h->gs_colour_start.size()) - 1;
				h->timed("k_bgs_colour", [&]{
					for(int q = 0; q < nc; q++) {
						const int col = fwd ? q : nc - 1 - q;
						const int b = h->gs_colour_start[col], n = h->gs_colour_start[col+1] - b;
						if(single) launch_bgs_colour(h->J, h->iw.sdinv, h->iw.slo, h->iw.sup, v(i), z(i), h->d_gs_cells + b, n, h->stream);
						else launch_bgs_colour(h->J, h->iw.dinv, Lo[i], Up[i], v(i), z(i), h->d_gs_cells + b, n, h->stream);
					}
				});
			});
		}
	}
	/// z = M^-1 v for the block ILU(0) M = (Dt + L) Dt^-1 (Dt + U) in colour order: a forward pass over
	/// the colours from z = 0 gives y = (Dt + L)^-1 v, the backward pass z_i = Dt_i^-1 (v_i - sum_{earlier}
	/// A_ik y_k - sum_{later} A_ij z_j) = y_i - Dt_i^-1 sum_{later} A_ij z_j -- both are the Gauss-Seidel
	/// colour kernel with the ILU pivots. Ghost rows stay zero (no exchange: block-Jacobi across ranks)
	void iluApply(const ArrayOf& v, const ArrayOf& z) {
		S.each([&](size_t i, fvhip_ctx* h) {
			exact::launch_fill(z(i), 0.0, 4LL*(h->L.ncell + h->L.nghost), h->stream);
			const int nc = static_cast<int>(h->gs_colour_start.size()) - 1;
			h->timed("k_ilu_solve", [&]{
				// forward over colours 0..nc-1, backward over nc-2..0: the last colour's backward value
				// would be its forward one again (all its neighbours are of earlier colours)
				for(int q = 0; q < 2*nc - 1; q++) {
					const int col = q < nc ? q : 2*nc - 2 - q;
					const int b = h->gs_colour_start[col], n = h->gs_colour_start[col+1] - b;
					if(single) launch_bgs_colour(h->J, h->iw.sdinv, h->iw.slo, h->iw.sup, v(i), z(i), h->d_gs_cells + b, n, h->stream);
					else launch_bgs_colour(h->J, h->iw.dinv, Lo[i], Up[i], v(i), z(i), h->d_gs_cells + b, n, h->stream);
				}
			});
		});
	}
	/// ILU(0), then `sweeps` - 1 corrections z += M^-1 (v - A z) (A with the ghost coupling)
	void iluSweeps(const ArrayOf& v, const ArrayOf& z) {
		const ArrayOf aux = [&](size_t i) { return S.hs[i]->iw.aux; };
		const ArrayOf t = [&](size_t i) { return S.hs[i]->iw.t; };
		iluApply(v, z);
		for(int k = 1; k < sweeps; k++) {
			blocks(z, t);
			S.each([&](size_t i, fvhip_ctx* h) { launch_axpby(4LL*h->L.ncell, 1.0, v(i), -1.0, t(i), h->stream); });
			iluApply(t, aux);
			S.each([&](size_t i, fvhip_ctx* h) { launch_add_rows(h->L.ncell, aux(i), z(i), h->stream); });
		}
	}
	/// z = M^-1 v with M the block-tridiagonal line part of A (factorised in setup), then `sweeps` - 1
	/// corrections z += M^-1 (v - A z) (A with the ghost coupling: block-Jacobi across ranks)
	void lineSweeps(const ArrayOf& v, const ArrayOf& z, bool want_norm = false) {
		const ArrayOf aux = [&](size_t i) { return S.hs[i]->iw.aux; };
		const ArrayOf t = [&](size_t i) { return S.hs[i]->iw.t; };
		// one sweep on one domain for the matrix-free operator: the line solve also returns |z|^2
		const bool norm = want_norm && matfree && sweeps == 1 && S.size() == 1 && !S.exg && !S.halo();
		S.each([&](size_t i, fvhip_ctx* h) {
			h->timed("k_line_solve", [&]{ launch_line_solve(h->lines, v(i), z(i), h->stream, norm ? h->iw.red : nullptr); });
		});
		znorm = norm;
		for(int k = 1; k < sweeps; k++) {
			blocks(z, t);
			S.each([&](size_t i, fvhip_ctx* h) {
				launch_axpby(4LL*h->L.ncell, 1.0, v(i), -1.0, t(i), h->stream);
				h->timed("k_line_solve", [&]{ launch_line_solve(h->lines, t(i), aux(i), h->stream); });
				launch_add_rows(h->L.ncell, aux(i), z(i), h->stream);
			});
		}
	}
	/// z = the finest smoother applied to v (line solve, else D^-1 v)
	void smooth0(fvhip_ctx* h, size_t i, const double* v, double* z) {
		if(lines) h->timed("k_line_solve", [&]{ launch_line_solve(h->lines, v, z, h->stream); });
		else if(single) launch_bjac_apply(h->L.ncell, h->iw.sdinv, v, z, h->stream);
		else launch_bjac_apply(h->L.ncell, h->iw.dinv, v, z, h->stream);
	}
	/// t = v - A z (A with the ghost coupling)
	void residual0(const ArrayOf& v, const ArrayOf& z, const ArrayOf& t) {
		S.exchange(z, 4);
		S.each([&](size_t i, fvhip_ctx* h) {
			h->timed("k_block_residual", [&]{
				if(single) launch_block_residual(h->J, h->iw.sdiag, h->iw.slo, h->iw.sup, z(i), v(i), t(i), h->stream);
				else launch_block_residual(h->J, D[i], Lo[i], Up[i], z(i), v(i), t(i), h->stream);
			});
		});
	}
	/// coarse level l of handle h's hierarchy: V-cycle on A_l x_l = b_l from x_l = 0 (colour Gauss-Seidel
	/// forward before the coarse correction, backward after it; the coarsest level amg_coarse sweeps)
	void cycle(fvhip_ctx* h, size_t l) {
		AmgLevel& C = h->amg[l];
		const bool small = C.n <= AMG_BLOCK_ROWS;        // one workgroup sweeps the level (no launch per colour)
		if(!small) exact::launch_fill(C.x, 0.0, 4LL*C.n, h->stream);
		const int nc = static_cast<int>(C.cstart_colour.size()) - 1;
		auto sweep = [&](bool fwd) {
			for(int q = 0; q < nc; q++) launch_amg_gs_colour(C, fwd ? q : nc - 1 - q, C.b, C.x, h->stream);
		};
		if(l + 1 == h->amg.size()) {
			if(small) launch_amg_gs_block(C, C.b, C.x, amg_coarse, true, true, true, h->stream);
			else for(int k = 0; k < amg_coarse; k++) sweep(k % 2 == 0);
			return;
		}
		if(small) launch_amg_gs_block(C, C.b, C.x, amg_sweeps, true, false, true, h->stream);
		else for(int k = 0; k < amg_sweeps; k++) sweep(true);
		launch_amg_residual(C, C.x, C.b, C.r, h->stream);
		AmgLevel& F = h->amg[l+1];
		launch_amg_restrict(F, C.r, F.b, h->stream);
		cycle(h, l + 1);
		launch_amg_prolong(F, F.x, C.x, h->stream);
		if(small) launch_amg_gs_block(C, C.b, C.x, amg_sweeps, false, false, false, h->stream);
		else for(int k = 0; k < amg_sweeps; k++) sweep(false);
	}
	/// z = M^-1 v, M one V-cycle of the aggregation multigrid (block-Jacobi across ranks: each handle's hierarchy
	/// covers its owned cells; the finest residuals include the ghost coupling)
	void amgApply(const ArrayOf& v, const ArrayOf& z) {
		const ArrayOf aux = [&](size_t i) { return S.hs[i]->iw.aux; };
		const ArrayOf t = [&](size_t i) { return S.hs[i]->iw.t; };
		S.each([&](size_t i, fvhip_ctx* h) { smooth0(h, i, v(i), z(i)); });
		auto correct = [&]() {             // z += M0^-1 (v - A z)
			residual0(v, z, t);
			S.each([&](size_t i, fvhip_ctx* h) { smooth0(h, i, t(i), aux(i)); launch_add_rows(h->L.ncell, aux(i), z(i), h->stream); });
		};
		for(int k = 1; k < amg_fine; k++) correct();
		residual0(v, z, t);
		S.each([&](size_t i, fvhip_ctx* h) {
			h->timed("k_amg_cycle", [&]{
				launch_amg_restrict(h->amg[0], t(i), h->amg[0].b, h->stream);
				cycle(h, 0);
				launch_amg_prolong(h->amg[0], h->amg[0].x, z(i), h->stream);
			});
		});
		for(int k = 0; k < amg_fine; k++) correct();
	}
	/// block inverses of the current diagonal blocks (or the line factorisation)
	void setup() {
		if(amg) {
			S.each([&](size_t i, fvhip_ctx* h) {
				if(lines) {
					h->ensureLines(line_thr);
					h->lines.single = single;
					h->timed("k_line_factor", [&]{ launch_line_factor(h->lines, D[i], Lo[i], Up[i], h->stream); });
				} else h->timed("k_bjac_invert", [&]{ launch_bjac_invert(h->L.ncell, D[i], h->iw.dinv, h->stream); });
				if(single) {                  // fp32 copies of the finest operator for the smoother's residuals
					h->ensureSinglePrecond();
					const long long nf = 16LL*std::max(h->L.ninface, 0);
					h->timed("k_to_single", [&]{
						launch_to_single(16LL*h->L.ncell, D[i], h->iw.sdiag, h->stream);
						launch_to_single(nf, Lo[i], h->iw.slo, h->stream);
						launch_to_single(nf, Up[i], h->iw.sup, h->stream);
						if(!lines) launch_to_single(16LL*h->L.ncell, h->iw.dinv, h->iw.sdinv, h->stream);
					});
				}
				h->ensureAmg(amg, amg_thr);
				h->amgSetup(D[i], Lo[i], Up[i]);
			});
			return;
		}
		S.each([&](size_t i, fvhip_ctx* h) {
			if(lines) {
				h->ensureLines(line_thr);
				h->lines.single = single;
				h->timed("k_line_factor", [&]{ launch_line_factor(h->lines, D[i], Lo[i], Up[i], h->stream); });
				return;
			}
			if(ilu) h->iluFactor(D[i], Lo[i], Up[i], h->iw.dinv);
			else h->timed("k_bjac_invert", [&]{ launch_bjac_invert(h->L.ncell, D[i], h->iw.dinv, h->stream); });
			if(gs) h->ensureColouring();
			if(single) {
				h->ensureSinglePrecond();
				const long long nf = 16LL*std::max(h->L.ninface, 0);
				h->timed("k_to_single", [&]{
					launch_to_single(16LL*h->L.ncell, h->iw.dinv, h->iw.sdinv, h->stream);
					if(sweeps > 1 || gs || ilu) {
						launch_to_single(nf, Lo[i], h->iw.slo, h->stream);
						launch_to_single(nf, Up[i], h->iw.sup, h->stream);
					}
				});
			}
		});
	}
};

struct GmresOut { int iters; double rnorm0, rnorm; };

/// Restarted GMRES(m) for A x = b, x0 = 0; stops when |b - A x| <= rtol |b| or after maxit
/// Arnoldi steps in total (KSPSolve with -ksp_rtol, -ksp_max_it, -ksp_gmres_restart)
static GmresOut gmres(System& S, LinOp& A, const ArrayOf& b, const ArrayOf& x, double rtol, int maxit, int m,
                      int refine = 0)
{
	if(refine < 0 || refine > 2) throw std::invalid_argument("cgs_refine must be 0 (never), 1 (ifneeded) or 2 (always)");
	auto n4 = [&](size_t i) { return 4LL*S.hs[i]->L.ncell; };
	auto V = [&](size_t i, int j) { return S.hs[i]->iw.V + static_cast<size_t>(j)*static_cast<size_t>(n4(i)); };
	const ArrayOf z = [&](size_t i) { return S.hs[i]->iw.z; };
	const ArrayOf w = [&](size_t i) { return S.hs[i]->iw.w; };
	const ArrayOf sv = [&](size_t i) { return S.hs[i]->iw.s; };
	auto norm = [&](const ArrayOf& v) {
		S.each([&](size_t i, fvhip_ctx* h) { launch_mdot(n4(i), 0, nullptr, 0, v(i), true, h->iw.part, h->iw.red, h->stream); });
		return std::sqrt(S.allsum(1, false)[0]);
	};
	S.each([&](size_t i, fvhip_ctx* h) { exact::launch_fill(x(i), 0.0, n4(i), h->stream); });
	const double beta0 = norm(b);
	GmresOut out{0, beta0, beta0};
	if(!(beta0 > 0.0) || maxit <= 0) return out;

	std::vector<double> H(static_cast<size_t>(m+1)*m, 0.0), cs(m), sn(m), g(m+1), y(m);
	auto Hij = [&](int i, int j) -> double& { return H[static_cast<size_t>(j)*(m+1) + i]; };
	double beta = beta0;
	bool first = true;
	while(true) {
		if(first) S.each([&](size_t i, fvhip_ctx* h) { launch_axpby(n4(i), 1.0/beta, b(i), 0.0, V(i,0), h->stream); });
		else {
			// restart: r = b - A x (x into the ghosted operand buffer first)
			S.each([&](size_t i, fvhip_ctx* h) {
				HC(hipMemcpyAsync(z(i), x(i), n4(i)*sizeof(double), hipMemcpyDeviceToDevice, h->stream));
			});
			A.apply(z, w);
			S.each([&](size_t i, fvhip_ctx* h) { launch_axpby(n4(i), 1.0, b(i), -1.0, w(i), h->stream); });
			beta = norm(w);
			out.rnorm = beta;
			if(beta <= rtol*beta0) break;
			S.each([&](size_t i, fvhip_ctx* h) { launch_axpby(n4(i), 1.0/beta, w(i), 0.0, V(i,0), h->stream); });
		}
		std::fill(g.begin(), g.end(), 0.0);
		g[0] = beta;
		int j = 0;
		bool done = false;
		while(j < m && out.iters < maxit) {
			A.precondition([&](size_t i) { return V(i,j); }, z, true);
			A.apply(z, w);
			// classical Gram-Schmidt (PETSc's KSPGMRESClassicalGramSchmidtOrthogonalization). refine 0
			// (PETSc's default, KSP_GMRES_CGS_REFINE_NEVER): one projection h = V^T w, w -= V h, and the new
			// norm computed from the projected w in the same pass (k_maxpy_norm) -- two passes over the
			// basis per step. refine 1 (ifneeded): the projection pass also returns |w|^2, so |w - V h|^2
			// follows by Pythagoras and a second projection runs only when the first removed more than half
			// of |w|^2 (DGKS); refine 2 (always): two projections every step.
			double hn2 = 0.0;
			if(refine == 0 && S.size() == 1) {
				// one handle: the projection's coefficients stay on the device for k_maxpy_norm and reach
				// the host with its norm -- one wait per Arnoldi step
				fvhip_ctx* h = S.hs[0];
				launch_mdot(n4(0), j+1, V(0,0), n4(0), w(0), false, h->iw.part, h->iw.red, h->stream);
				S.allsumQueue(j+1);
				launch_maxpy_norm(n4(0), j+1, V(0,0), n4(0), h->iw.red, w(0), h->iw.part, h->iw.red, h->stream);
				hn2 = S.allsum(1, false)[0];
				for(int k = 0; k <= j; k++) Hij(k,j) = h->iw.h_red2[k];
			} else if(refine != 1) {
				S.each([&](size_t i, fvhip_ctx* h) {
					launch_mdot(n4(i), j+1, V(i,0), n4(i), w(i), false, h->iw.part, h->iw.red, h->stream);
				});
				const std::vector<double> h1 = S.allsum(j+1, true);
				for(int k = 0; k <= j; k++) Hij(k,j) = h1[k];
				if(refine == 2) {
					S.each([&](size_t i, fvhip_ctx* h) { launch_maxpy(n4(i), j+1, V(i,0), n4(i), h->iw.red, w(i), h->stream); });
					S.each([&](size_t i, fvhip_ctx* h) {
						launch_mdot(n4(i), j+1, V(i,0), n4(i), w(i), false, h->iw.part, h->iw.red, h->stream);
					});
					const std::vector<double> h2 = S.allsum(j+1, true);
					for(int k = 0; k <= j; k++) Hij(k,j) += h2[k];
				}
				S.each([&](size_t i, fvhip_ctx* h) {
					launch_maxpy_norm(n4(i), j+1, V(i,0), n4(i), h->iw.red, w(i), h->iw.part, h->iw.red, h->stream);
				});
				hn2 = S.allsum(1, false)[0];
			} else {
				S.each([&](size_t i, fvhip_ctx* h) {
					launch_mdot(n4(i), j+1, V(i,0), n4(i), w(i), true, h->iw.part, h->iw.red, h->stream);
				});
				const std::vector<double> h1 = S.allsum(j+2, true);
				S.each([&](size_t i, fvhip_ctx* h) { launch_maxpy(n4(i), j+1, V(i,0), n4(i), h->iw.red, w(i), h->stream); });
				double corr = 0.0;
				for(int k = 0; k <= j; k++) { Hij(k,j) = h1[k]; corr += h1[k]*h1[k]; }
				hn2 = h1[j+1] - corr;
				if(!(hn2 > 0.5*h1[j+1])) {
					S.each([&](size_t i, fvhip_ctx* h) {
						launch_mdot(n4(i), j+1, V(i,0), n4(i), w(i), true, h->iw.part, h->iw.red, h->stream);
					});
					const std::vector<double> h2 = S.allsum(j+2, true);
					S.each([&](size_t i, fvhip_ctx* h) { launch_maxpy(n4(i), j+1, V(i,0), n4(i), h->iw.red, w(i), h->stream); });
					corr = 0.0;
					for(int k = 0; k <= j; k++) { Hij(k,j) += h2[k]; corr += h2[k]*h2[k]; }
					hn2 = h2[j+1] - corr;
					if(!(hn2 > 1e-4*h2[j+1])) { const double t = norm(w); hn2 = t*t; }   // cancellation: measure
				}
			}
			const double hn = std::sqrt(hn2);
			Hij(j+1,j) = hn;
			if(hn > 0.0) S.each([&](size_t i, fvhip_ctx* h) { launch_axpby(n4(i), 1.0/hn, w(i), 0.0, V(i,j+1), h->stream); });
			// Givens rotations of the Hessenberg column
			for(int k = 0; k < j; k++) {
				const double t = cs[k]*Hij(k,j) + sn[k]*Hij(k+1,j);
				Hij(k+1,j) = -sn[k]*Hij(k,j) + cs[k]*Hij(k+1,j);
				Hij(k,j) = t;
			}
			const double d = std::hypot(Hij(j,j), Hij(j+1,j));
			cs[j] = d > 0.0 ? Hij(j,j)/d : 1.0;
			sn[j] = d > 0.0 ? Hij(j+1,j)/d : 0.0;
			Hij(j,j) = d; Hij(j+1,j) = 0.0;
			g[j+1] = -sn[j]*g[j];
			g[j] = cs[j]*g[j];
			j++;
			out.iters++;
			out.rnorm = std::fabs(g[j]);
			if(!std::isfinite(out.rnorm)) throw std::runtime_error("GMRES: non-finite residual");
			if(out.rnorm <= rtol*beta0 || hn == 0.0) { done = true; break; }
		}
		// x += M^-1 V y with H y = g (upper triangular after the rotations)
		for(int k = j-1; k >= 0; k--) {
			double s = g[k];
			for(int l = k+1; l < j; l++) s -= Hij(k,l)*y[l];
			y[k] = s/Hij(k,k);
		}
		S.each([&](size_t i, fvhip_ctx* h) {
			std::copy(y.begin(), y.begin() + j, h->iw.h_coef);
			HC(hipMemcpyAsync(h->iw.coef, h->iw.h_coef, j*sizeof(double), hipMemcpyHostToDevice, h->stream));
			launch_lincomb(n4(i), j, V(i,0), n4(i), h->iw.coef, sv(i), h->stream);
		});
		A.precondition(sv, z);
		S.each([&](size_t i, fvhip_ctx* h) { launch_axpby(n4(i), 1.0, z(i), 1.0, x(i), h->stream); });
		S.sync();            // h_coef is rewritten by the next cycle
		if(done || out.iters >= maxit) break;
		first = false;
	}
	return out;
}

/// SteadySolver::expResidualRamp (aodesolver.cpp:110-120)
static double expResidualRamp(double cflmin, double cflmax, double prevcfl, double resratio,
                              double paramup, double paramdown)
{
	const double newcfl = resratio > 1.0 ? prevcfl * std::pow(resratio, paramup)
		: prevcfl * std::pow(resratio, paramdown);
	if(newcfl < cflmin) return cflmin;
	else if(newcfl > cflmax) return cflmax;
	else return newcfl;
}

static void checkImplicit(const fvhip_implicit_config& c)
{
	if(c.restart < 1 || c.restart > KRY_MAXK) throw std::invalid_argument("restart must be in [1, 128]");
	if(c.cgs_refine < 0 || c.cgs_refine > 2) throw std::invalid_argument("cgs_refine must be 0 (never), 1 (ifneeded) or 2 (always)");
	if(c.prec_sweeps < 1) throw std::invalid_argument("prec_sweeps must be >= 1");
	if(c.prec_amg != 0 && c.prec_amg < 2) throw std::invalid_argument("prec_amg must be 0 (off) or >= 2 levels");
	if(c.amg_sweeps < 0 || c.amg_coarse_sweeps < 0 || c.amg_fine_sweeps < 0 || !(c.amg_threshold >= 0.0 && c.amg_threshold < 1.0))
		throw std::invalid_argument("amg_sweeps / amg_coarse_sweeps must be >= 0 and amg_threshold in [0, 1)");
	if(!(c.min_relax > 0.0)) throw std::domain_error("Minimum relaxation factor is invalid!");  // nonlinearrelaxation.cpp:20-21
	if(c.matrix_free && !(c.mf_eps > 0.0)) throw std::invalid_argument("matrix-free difference step must be positive");
	if(!(c.line_threshold >= 0.0) || !std::isfinite(c.line_threshold))
		throw std::invalid_argument("line_threshold must be finite and >= 0 (0: the default 4)");
}

/// SteadyBackwardEulerSolver::solve (aodesolver.cpp:363-638) on device states us (internal order,
/// ghost rows included on partitioned handles)
static void backwardEuler(System& S, const std::vector<double*>& us, const fvhip_implicit_config& c,
                          fvhip_solve_stats* st, double* hist)
{
	checkImplicit(c);
	S.each([&](size_t, fvhip_ctx* h) { h->ensureImplicit(c.restart); h->mf_eps = c.mf_eps; });
	LinOp A{S};
	A.matfree = c.matrix_free != 0;
	A.sweeps = c.prec_sweeps;
	A.single = c.prec_single != 0;
	A.gs = c.prec_gs != 0;
	A.lines = c.prec_lines != 0;
	A.line_thr = c.line_threshold;
	A.ilu = c.prec_ilu != 0;
	if(A.lines && A.gs) throw std::invalid_argument("prec_lines does not combine with prec_gs");
	if(A.ilu && (A.gs || A.lines)) throw std::invalid_argument("prec_ilu does not combine with prec_gs / prec_lines");
	A.amg = c.prec_amg;
	A.amg_sweeps = c.amg_sweeps > 0 ? c.amg_sweeps : 2;
	A.amg_coarse = c.amg_coarse_sweeps > 0 ? c.amg_coarse_sweeps : 6;
	A.amg_fine = c.amg_fine_sweeps > 0 ? c.amg_fine_sweeps : A.amg_sweeps;
	A.amg_thr = c.amg_threshold > 0.0 ? c.amg_threshold : 0.2;
	if(A.amg && (A.gs || A.ilu || A.sweeps != 1))
		throw std::invalid_argument("prec_amg combines with prec_lines and prec_single only (prec_gs / prec_ilu / prec_sweeps > 1 are one-level options)");
	for(fvhip_ctx* h : S.hs) { A.D.push_back(h->iw.jd); A.Lo.push_back(h->iw.jlo); A.Up.push_back(h->iw.jup); }
	std::vector<const double*> cu(us.begin(), us.end());
	std::vector<double*> rs, dts;
	for(fvhip_ctx* h : S.hs) { rs.push_back(h->d_r); dts.push_back(h->d_dtm); }
	const ArrayOf bs = [&](size_t i) { return S.hs[i]->d_r; };
	const ArrayOf xs = [&](size_t i) { return S.hs[i]->iw.du; };

	double curCFL = 0, resi = 1.0, resiold = 1.0, initres = 1.0, linworst = 0.0;
	int step = 0, lin = 0, linbad = 0;
	const bool resume = c.resume_res0 > 0.0;
	if(resume) {                     // a checkpointed solve: its residuals and CFL, the ramp continues from them
		if(!(c.resume_res > 0.0 && c.resume_res_prev > 0.0 && c.resume_cfl > 0.0))
			throw std::invalid_argument("resume: the last residual, the one before and the last CFL must be positive");
		initres = c.resume_res0; resi = c.resume_res; resiold = c.resume_res_prev; curCFL = c.resume_cfl;
	}
	while(resi/initres > c.tol && step < c.maxiter) {
		// r = 0 + (-r(u)) with local time steps (:421-452); fills the ghost rows of u
		fvhip_ctx::residual_seq(S.hs, cu, rs, true, dts, true, S.exg);
		curCFL = expResidualRamp(c.cflinit, c.cflfin, curCFL, resiold/resi, 0.25, 0.3);           // :462
		// Jacobian (:456-457) with the pseudo-time term (:467) added in its diagonal pass
		S.each([&](size_t i, fvhip_ctx* h) { h->assemble(us[i], h->iw.jd, h->iw.jlo, h->iw.jup, curCFL, h->d_dtm); });
		A.setup();
		if(A.matfree)                                                                               // :386-394
			S.each([&](size_t i, fvhip_ctx* h) { h->mf_u = us[i]; h->mf_r = h->d_r; h->mf_mdt = h->d_dtm; });
		const GmresOut g = gmres(S, A, bs, xs, c.lin_rtol, c.lin_maxit, c.restart, c.cgs_refine);    // :483
		lin += g.iters;
		if(g.rnorm0 > 0.0) {
			linworst = std::max(linworst, g.rnorm/g.rnorm0);
			if(g.rnorm > c.lin_rtol*g.rnorm0) linbad++;
		}
		S.each([&](size_t i, fvhip_ctx* h) {                                                        // :494-512
			launch_relaxed_update(h->L.ncell, h->P.gas, c.min_relax, h->iw.du, us[i], h->stream);
			launch_energy_sumsq(h->L.ncell, h->d_r, h->M.area, h->iw.part, h->iw.red, h->stream);   // :516-526
			HC(hipGetLastError());
		});
		resiold = resi;
		resi = std::sqrt(S.allsum(1, false)[0]);                                                    // :528-530
		if(!std::isfinite(resi))
			throw std::runtime_error("Steady backward Euler diverged - residual is Nan or inf!");  // :533-534
		if(step == 0 && !resume) initres = resi;
		step++;
		if(hist) hist[step-1] = resi;
	}
	if(A.matfree) S.each([&](size_t, fvhip_ctx* h) { h->mf_u = h->mf_r = h->mf_mdt = nullptr; });
	st->steps = step;
	st->lin_iters = lin;
	st->resratio = resi/initres;
	st->converged = (step < c.maxiter && resi/initres <= c.tol) ? 1 : 0;                            // :618-632
	st->cfl = curCFL;
	st->lin_unconverged = linbad;
	st->lin_worst = linworst;
}

/// SteadyForwardEulerSolver::solve (aodesolver.cpp:135-282): u += cflinit dtm/area r (the ramped
/// CFL is only reported by the reference, :194, :208)
static void forwardEuler(System& S, const std::vector<double*>& us, double cfl, double tol, int maxiter,
                         int* steps, double* resratio, double* hist)
{
	S.each([&](size_t, fvhip_ctx* h) { h->ensureReductions(); });
	std::vector<const double*> cu(us.begin(), us.end());
	std::vector<double*> rs, dts;
	for(fvhip_ctx* h : S.hs) { rs.push_back(h->d_r); dts.push_back(h->d_dtm); }
	double resi = 1.0, initres = 1.0;
	int step = 0;
	while(resi/initres > tol && step < maxiter) {
		fvhip_ctx::residual_seq(S.hs, cu, rs, true, dts, true, S.exg);                          // :180-189
		S.each([&](size_t i, fvhip_ctx* h) {
			launch_fe_update(h->L.ncell, h->d_r, h->d_dtm, h->M.area, cfl, us[i], h->stream);   // :204-209
			launch_energy_sumsq(h->L.ncell, h->d_r, h->M.area, h->iw.part, h->iw.red, h->stream);
			HC(hipGetLastError());
		});
		resi = std::sqrt(S.allsum(1, false)[0]);                                                  // :214-230
		if(step == 0) initres = resi;
		if(hist) hist[step] = resi;
		step++;
		if(!std::isfinite(resi))
			throw std::runtime_error("Steady forward Euler diverged - residual is Nan or inf!");  // :250-251
	}
	if(steps) *steps = step;
	if(resratio) *resratio = resi/initres;
}

/// TVDRKSolver::solve (aodesolver.cpp:669-758) on the device, restated as written: ustage = u once
/// before the time loop (:701-704); per step, every stage's residual is computed at u -- the step's
/// start state, since the reference passes uvec, not the stage state, to compute_residual (:719) --
/// dtmin = min over cells of the first stage's local time steps (:722-728; across ranks the global
/// minimum, so a partitioned run takes the 1-GPU steps, where the reference's ranks would each take
/// their own), ustage = c0 u + c1 ustage - c2 dtmin cfl / area r (:735-744), then u = ustage and
/// time += dtmin cfl (:747-757), while time <= finaltime - 1e-12 (A_SMALL_NUMBER). The stages' residuals
/// are the same bits (same input, deterministic kernels), so one residual per step is computed and
/// reused. maxsteps caps the loop (the reference has no cap).
static void tvdrk(System& S, const std::vector<double*>& us, int order, double cfl, double finaltime, int maxsteps,
                  int* steps, double* time_out)
{
	static const double coef[3][3][3] = {                                       // initialize_TVDRK_Coeffs :45-67
		{{1.0, 0.0, 1.0}, {0, 0, 0}, {0, 0, 0}},
		{{1.0, 0.0, 1.0}, {0.5, 0.5, 0.5}, {0, 0, 0}},
		{{1.0, 0.0, 1.0}, {0.75, 0.25, 0.25}, {0.3333333333333333, 0.6666666666666667, 0.6666666666666667}}};
	if(order < 1 || order > 3) throw std::invalid_argument("TVD RK: temporal order must be 1, 2 or 3");
	if(maxsteps < 1) throw std::invalid_argument("TVD RK: maxsteps must be >= 1");
	const double (*tc)[3] = coef[order-1];
	S.each([&](size_t i, fvhip_ctx* h) {
		h->ensureReductions();
		if(!h->d_ustage) h->d_ustage = dalloc(4*static_cast<size_t>(std::max(h->L.ncell, 1)), h->owned);
		HC(hipMemcpyAsync(h->d_ustage, us[i], sizeof(double)*4*static_cast<size_t>(h->L.ncell), hipMemcpyDeviceToDevice,
		                  h->stream));
	});
	std::vector<const double*> cu(us.begin(), us.end());
	std::vector<double*> rs, dts;
	for(fvhip_ctx* h : S.hs) { rs.push_back(h->d_r); dts.push_back(h->d_dtm); }
	int step = 0;
	double time = 0;
	while(time <= finaltime - 1e-12 && step < maxsteps) {
		fvhip_ctx::residual_seq(S.hs, cu, rs, true, dts, true, S.exg);              // :712-719 (zeroed, -r(u))
		S.each([&](size_t, fvhip_ctx* h) {
			launch_min(h->L.ncell, h->d_dtm, h->iw.part, h->iw.red, h->stream);
			if(h->comm) NC(ncclAllReduce(h->iw.red, h->iw.red, 1, ncclDouble, ncclMin, h->comm, h->stream));
			HC(hipMemcpyAsync(h->iw.h_red, h->iw.red, sizeof(double), hipMemcpyDeviceToHost, h->stream));
		});
		double dtmin = INFINITY;
		S.each([&](size_t, fvhip_ctx* h) { HC(hipStreamSynchronize(h->stream)); dtmin = std::min(dtmin, h->iw.h_red[0]); });
		if(!std::isfinite(dtmin)) throw std::runtime_error("TVDRK solver diverged - dtmin is Nan or inf!");   // :730-731
		for(int s = 0; s < order; s++) {
			const double sc = tc[s][2]*dtmin*cfl;
			S.each([&](size_t i, fvhip_ctx* h) {
				launch_tvdrk_stage(h->L.ncell, tc[s][0], tc[s][1], sc, h->M.area, h->d_r, us[i], h->d_ustage, h->stream);
			});
		}
		S.each([&](size_t i, fvhip_ctx* h) {
			HC(hipMemcpyAsync(us[i], h->d_ustage, sizeof(double)*4*static_cast<size_t>(h->L.ncell), hipMemcpyDeviceToDevice,
			                  h->stream));
			HC(hipGetLastError());
		});
		step++;
		time += dtmin*cfl;
	}
	if(steps) *steps = step;
	if(time_out) *time_out = time;
}

static System single(fvhip_ctx* h)
{
	if(h->in_group) throw std::runtime_error("handle belongs to a group: use the fvhip_group_* entry point");
	if(h->halo() && !h->comm) throw std::runtime_error("partitioned handle: call fvhip_comm_init (or use a group) first");
	return System{{h}, {}};
}

static System ofGroup(fvhip_group_s* g) { return System{g->hs, groupExchange(g)}; }

void sysMatfree(const std::vector<fvhip_ctx*>& hs, const fvhip_ctx::GroupExchange& exg,
                const std::vector<const double*>& x, const std::vector<double*>& y)
{
	System S{hs, exg};
	S.each([&](size_t, fvhip_ctx* h) { h->ensureVectors(); });
	const ArrayOf xo = [&](size_t i) { return const_cast<double*>(x[i]); };
	const ArrayOf yo = [&](size_t i) { return y[i]; };
	matfreeApply(S, xo, yo);
}

}

extern "C" {

int fvhip_steady_backward_euler_device(fvhip_handle h, double* d_u, const fvhip_implicit_config* cfg,
                                       fvhip_solve_stats* stats, double* reshistory)
{
	return guard([&] {
		need(h, "handle");
		need(d_u, "u");
		if(!cfg || !stats) throw std::invalid_argument("null argument");
		System S = single(h);
		backwardEuler(S, {d_u}, *cfg, stats, reshistory);
		S.sync();
	});
}

int fvhip_group_steady_backward_euler_device(fvhip_group g, double* const* d_u, const fvhip_implicit_config* cfg,
                                             fvhip_solve_stats* stats, double* reshistory)
{
	return guard([&] {
		need(g, "group");
		needEach(d_u, g->hs.size(), "u");
		if(!cfg || !stats) throw std::invalid_argument("null argument");
		System S = ofGroup(g);
		backwardEuler(S, std::vector<double*>(d_u, d_u + S.size()), *cfg, stats, reshistory);
		S.sync();
	});
}

int fvhip_steady_forward_euler_device(fvhip_handle h, double* d_u, double cfl, double tol, int maxiter,
                                      int* steps, double* resratio, double* reshistory)
{
	return guard([&] {
		need(h, "handle");
		need(d_u, "u");
		System S = single(h);
		forwardEuler(S, {d_u}, cfl, tol, maxiter, steps, resratio, reshistory);
		S.sync();
	});
}

int fvhip_group_steady_forward_euler_device(fvhip_group g, double* const* d_u, double cfl, double tol, int maxiter,
                                            int* steps, double* resratio, double* reshistory)
{
	return guard([&] {
		need(g, "group");
		needEach(d_u, g->hs.size(), "u");
		System S = ofGroup(g);
		forwardEuler(S, std::vector<double*>(d_u, d_u + S.size()), cfl, tol, maxiter, steps, resratio, reshistory);
		S.sync();
	});
}

int fvhip_tvdrk_device(fvhip_handle h, double* d_u, int order, double cfl, double finaltime, int maxsteps,
                       int* steps, double* time)
{
	return guard([&] {
		need(h, "handle");
		need(d_u, "u");
		System S = single(h);
		tvdrk(S, {d_u}, order, cfl, finaltime, maxsteps, steps, time);
		S.sync();
	});
}

int fvhip_group_tvdrk_device(fvhip_group g, double* const* d_u, int order, double cfl, double finaltime, int maxsteps,
                             int* steps, double* time)
{
	return guard([&] {
		need(g, "group");
		needEach(d_u, g->hs.size(), "u");
		System S = ofGroup(g);
		tvdrk(S, std::vector<double*>(d_u, d_u + S.size()), order, cfl, finaltime, maxsteps, steps, time);
		S.sync();
	});
}

int fvhip_gmres_blocks_device(fvhip_handle h, const double* d_diag, const double* d_lower, const double* d_upper,
                              const double* d_b, double* d_x, double rtol, int maxit, int restart, int sweeps,
                              int* iters, double* resnorm)
{
	return guard([&] {
		need(h, "handle");
		need(d_diag, "diag"); if(h->L.ninface > 0) { need(d_lower, "lower"); need(d_upper, "upper"); } need(d_b, "b"); need(d_x, "x");
		if(restart < 1 || restart > KRY_MAXK) throw std::invalid_argument("restart must be in [1, 128]");
		if(sweeps < 1) throw std::invalid_argument("sweeps must be >= 1");
		System S = single(h);
		h->ensureImplicit(restart);
		LinOp A{S};
		A.sweeps = sweeps;
		A.D = {d_diag}; A.Lo = {d_lower}; A.Up = {d_upper};
		A.setup();
		// the standalone solver keeps the selective reorthogonalisation it was pinned with (cgs_refine 1)
		const GmresOut g = gmres(S, A, [&](size_t) { return const_cast<double*>(d_b); },
		                         [&](size_t) { return d_x; }, rtol, maxit, restart, 1);
		S.sync();
		if(iters) *iters = g.iters;
		if(resnorm) *resnorm = g.rnorm;
	});
}

int fvhip_line_precondition_device(fvhip_handle h, const double* d_diag, const double* d_lower, const double* d_upper,
                                   double line_threshold, int single, const double* d_v, double* d_z)
{
	return guard([&] {
		need(h, "handle");
		need(d_diag, "diag"); if(h->L.ninface > 0) { need(d_lower, "lower"); need(d_upper, "upper"); } need(d_v, "v"); need(d_z, "z");
		if(!d_diag || !d_v || !d_z || (h->L.ninface > 0 && (!d_lower || !d_upper))) throw std::invalid_argument("null argument");
		HC(hipSetDevice(h->device));
		h->ensureLines(line_threshold);
		h->lines.single = single != 0;
		launch_line_factor(h->lines, d_diag, d_lower, d_upper, h->stream);
		launch_line_solve(h->lines, d_v, d_z, h->stream);
		HC(hipGetLastError());
		HC(hipStreamSynchronize(h->stream));
	});
}

int fvhip_ilu_precondition_device(fvhip_handle h, const double* d_diag, const double* d_lower, const double* d_upper,
                                  const double* d_v, double* d_z)
{
	return guard([&] {
		need(h, "handle");
		need(d_diag, "diag"); if(h->L.ninface > 0) { need(d_lower, "lower"); need(d_upper, "upper"); } need(d_v, "v"); need(d_z, "z");
		if(!d_diag || !d_v || !d_z || (h->L.ninface > 0 && (!d_lower || !d_upper))) throw std::invalid_argument("null argument");
		System S = single(h);
		h->ensureImplicit(1);
		LinOp A{S};
		A.ilu = true;
		A.D = {d_diag}; A.Lo = {d_lower}; A.Up = {d_upper};
		A.setup();
		A.precondition([&](size_t) { return const_cast<double*>(d_v); }, [&](size_t) { return d_z; });
		HC(hipGetLastError());
		S.sync();
	});
}

int fvhip_amg_precondition_device(fvhip_handle h, const double* d_diag, const double* d_lower, const double* d_upper,
                                  int levels, double threshold, int sweeps, int coarse_sweeps, double line_threshold,
                                  const double* d_v, double* d_z, int* nlevels)
{
	return guard([&] {
		need(h, "handle");
		need(d_diag, "diag"); if(h->L.ninface > 0) { need(d_lower, "lower"); need(d_upper, "upper"); }
		if(levels < 2 || sweeps < 1 || coarse_sweeps < 1) throw std::invalid_argument("levels >= 2, sweeps >= 1, coarse_sweeps >= 1");
		if((d_v == nullptr) != (d_z == nullptr)) throw std::invalid_argument("v and z go together");
		System S = single(h);
		h->ensureImplicit(1);
		LinOp A{S};
		A.amg = levels; A.amg_sweeps = A.amg_fine = sweeps; A.amg_coarse = coarse_sweeps; A.amg_thr = threshold;
		A.lines = line_threshold > 0.0; A.line_thr = line_threshold;
		A.D = {d_diag}; A.Lo = {d_lower}; A.Up = {d_upper};
		A.setup();
		if(d_v) {
			// z needs ghost rows for the finest residuals: the handle's own operand buffer
			A.precondition([&](size_t) { return const_cast<double*>(d_v); }, [&](size_t) { return h->iw.z; });
			HC(hipMemcpyAsync(d_z, h->iw.z, 4*sizeof(double)*static_cast<size_t>(h->L.ncell), hipMemcpyDeviceToDevice, h->stream));
		}
		HC(hipGetLastError());
		S.sync();
		if(nlevels) *nlevels = static_cast<int>(h->amg.size());
	});
}

int fvhip_amg_level(fvhip_handle h, int level, int* n, int* nnz, int* agg, int* rowptr, int* col, double* val)
{
	return guard([&] {
		need(h, "handle");
		if(level < 1 || level > static_cast<int>(h->amg.size())) throw std::invalid_argument("no such multigrid level");
		const AmgLevel& L = h->amg[static_cast<size_t>(level) - 1];
		HC(hipSetDevice(h->device));
		HC(hipStreamSynchronize(h->stream));
		if(n) *n = L.n;
		if(nnz) *nnz = L.nnz;
		if(agg) HC(hipMemcpy(agg, L.agg, sizeof(int)*static_cast<size_t>(L.nfine), hipMemcpyDeviceToHost));
		if(rowptr) HC(hipMemcpy(rowptr, L.rowptr, sizeof(int)*(static_cast<size_t>(L.n) + 1), hipMemcpyDeviceToHost));
		if(col) HC(hipMemcpy(col, L.col, sizeof(int)*static_cast<size_t>(L.nnz), hipMemcpyDeviceToHost));
		if(val) HC(hipMemcpy(val, L.val, 16*sizeof(double)*static_cast<size_t>(L.nnz), hipMemcpyDeviceToHost));
	});
}

int fvhip_colouring(fvhip_handle h, int* ncolours, int* colour, long long* triples)
{
	return guard([&] {
		need(h, "handle");
		h->ensureColouring();
		if(ncolours) *ncolours = static_cast<int>(h->gs_colour_start.size()) - 1;
		if(colour) std::copy(h->gs_colour.begin(), h->gs_colour.end(), colour);
		if(triples) *triples = h->gs_triples;
	});
}

int fvhip_lines(fvhip_handle h, double line_threshold, int* nlines, int* start, int* cells, int* faces)
{
	return guard([&] {
		need(h, "handle");
		HC(hipSetDevice(h->device));
		h->ensureLines(line_threshold);
		if(nlines) *nlines = h->lines.nlines;
		if(start) std::copy(h->h_line_start.begin(), h->h_line_start.end(), start);
		if(cells) std::copy(h->h_line_cells.begin(), h->h_line_cells.end(), cells);
		if(faces) std::copy(h->h_line_faces.begin(), h->h_line_faces.end(), faces);
	});
}

}
