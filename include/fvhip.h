/** \file fvhip.h
 * \brief C-ABI of the MI355X face-sweep library (libfvhip.so).
 *
 * This is the drop-in boundary for FVENS's spatial-discretisation hot path. Each entry point
 * replaces one method of the reference's operator classes (paths under /root/reference/src):
 *
 *   fvhip_create             FlowFV<scalar,order2,constVisc>::FlowFV      spatial/flow_spatial.cpp:312-337
 *                            (+ FlowFV_base ctor :34-59, Spatial ctor spatial/aspatial.cpp:36-76,
 *                             factory create_const_flowSpatialDiscretization utilities/afactory.cpp:251-267)
 *   fvhip_destroy            FlowFV::~FlowFV                               spatial/flow_spatial.cpp:339-346
 *   fvhip_compute_residual   FlowFV::compute_residual                      spatial/flow_spatial.cpp:636-816
 *                            (virtual Spatial::compute_residual            spatial/aspatial.hpp:62-63)
 *   fvhip_get_gradients      FlowFV_base::getGradients                     spatial/flow_spatial.cpp:95-112
 *   fvhip_surface_data_device FlowFV_base::computeSurfaceData              spatial/flow_spatial.cpp:130-310
 *   fvhip_assemble_jacobian  Spatial::assemble_jacobian                    spatial/aspatial.cpp:242-340
 *   fvhip_matfree_set_state  MatrixFreeSpatialJacobian::set_state          linalg/alinalg.cpp:131-140
 *   fvhip_matfree_apply      MatrixFreeSpatialJacobian::apply              linalg/alinalg.cpp:142-233
 *   fvhip_local_flux         InviscidFlux::get_flux                        spatial/anumericalflux.hpp:32-34
 *   fvhip_local_flux_jacobian InviscidFlux::get_jacobian                   spatial/anumericalflux.hpp:43-45
 *
 * Conventions (identical to the reference, spatial/flow_spatial.hpp:73-85, aspatial.hpp:49-66):
 *  - u is the ghosted conserved state (rho, rho*vx, rho*vy, rho*E), row-major [nelem+nconnface][4]
 *    in the reference's cell numbering; r is [nelem][4]; dtm is [nelem].
 *  - compute_residual ADDS -r(u) into r; dtm[i] = area_i / sum_faces(spectral radius * length).
 *  - Jacobian blocks are row-major 4x4 and are ADDED (ADD_VALUES) into the caller's arrays.
 *  - Every function returns 0 on success, nonzero on failure; fvhip_last_error() describes it.
 *    No C++ exception crosses this boundary. A null handle, or a null array the call reads or
 *    writes, is refused ("null <what>") before any host or device access; fvhip_create refuses a
 *    configuration the reference's factories cannot build (unknown flux, Jacobian flux or
 *    reconstruction, periodic or unknown BC type, Venkatakrishnan K <= 0). fvhip_destroy(NULL) and
 *    fvhip_group_destroy(NULL) do nothing. Calls on one handle are not thread-safe
 *    (like the reference, flow_spatial.hpp:196-197); each handle owns one HIP stream.
 *  - *_device variants take device pointers in the library's internal cell order (see
 *    fvhip_to_internal / fvhip_from_internal) and are asynchronous on the handle's stream, a
 *    non-blocking stream: input arrays a caller writes on another stream (e.g. PyTorch's) must be
 *    complete before the call (synchronize that stream), and outputs are complete after
 *    fvhip_synchronize (or any later call that returns host results). */
#ifndef FVHIP_H
#define FVHIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define FVHIP_NVARS 4
#define FVHIP_NDIM 2

/* Numerical inviscid fluxes, afactory.cpp:38-81 ("VANLEER","ROE","HLL","HLLC","LLF","AUSM","AUSMPLUS") */
enum fvhip_flux_type {
	FVHIP_FLUX_LLF = 0, FVHIP_FLUX_VANLEER = 1, FVHIP_FLUX_AUSM = 2, FVHIP_FLUX_AUSMPLUS = 3,
	FVHIP_FLUX_ROE = 4, FVHIP_FLUX_HLL = 5, FVHIP_FLUX_HLLC = 6
};
/* Gradient schemes, afactory.cpp:111-127 ("LEASTSQUARES","GREENGAUSS", anything else -> zero) */
enum fvhip_gradient_type { FVHIP_GRAD_ZERO = 0, FVHIP_GRAD_GREENGAUSS = 1, FVHIP_GRAD_LEASTSQUARES = 2 };
/* Reconstructions, afactory.cpp:178-211 ("NONE","WENO","VANALBADA","BARTHJESPERSEN","VENKATAKRISHNAN") */
enum fvhip_recon_type {
	FVHIP_REC_NONE = 0, FVHIP_REC_WENO = 1, FVHIP_REC_VANALBADA = 2, FVHIP_REC_BARTHJESPERSEN = 3,
	FVHIP_REC_VENKATAKRISHNAN = 4
};
/* Boundary condition types in the reference's enum order, spatial/abctypes.hpp:12-21 */
enum fvhip_bc_type {
	FVHIP_BC_SLIPWALL = 0, FVHIP_BC_FARFIELD = 1, FVHIP_BC_INFLOW_OUTFLOW = 2,
	FVHIP_BC_SUBSONIC_INFLOW = 3, FVHIP_BC_EXTRAPOLATION = 4, FVHIP_BC_PERIODIC = 5,
	FVHIP_BC_ISOTHERMAL_WALL = 6, FVHIP_BC_ADIABATIC_WALL = 7
};

/** FlowPhysicsConfig (flow_spatial.hpp:33-44) + FlowNumericsConfig (:47-55) + FlowBCConfig list */
typedef struct fvhip_flow_config {
	double gamma, Minf, Tinf, Reinf, Pr, aoa;   /* aoa in radians */
	int viscous_sim, const_visc;
	int conv_numflux;         /* enum fvhip_flux_type */
	int conv_numflux_jac;     /* enum fvhip_flux_type, used by the Jacobian */
	int gradientscheme;       /* enum fvhip_gradient_type */
	int reconstruction;       /* enum fvhip_recon_type */
	double limiter_param;     /* Venkatakrishnan K / WENO lambda (must be given explicitly) */
	int order2;               /* second-order (gradients + reconstruction) if nonzero */
	int nbc;                  /* number of boundary conditions */
	const int* bc_type;       /* [nbc] enum fvhip_bc_type */
	const int* bc_tag;        /* [nbc] boundary marker (gbtags(face,0)) */
	const double* bc_vals;    /* [nbc][2] boundary_values (wall velocity, temperature, ...) */
	int fast_math;            /* 0: parity mode, residuals bitwise equal to the reference's
	                             single-thread arithmetic; 1: contracted FMAs and approximate
	                             division/sqrt in the residual sweep (relative differences ~1e-15,
	                             tested at 1e-11 of max|r|). Not a reference option. */
} fvhip_flow_config;

/** The UMesh data the sweep needs, exactly as the reference's accessors return it
 *  (mesh/mesh.hpp: gcoords, ginpoel, gnnode, gintfac, gbtags, gfacemetric, garea, gesuel,
 *  gelemface; cell centres rc from Spatial::rcvec, ghost centres rcbp, face centres gr). */
typedef struct fvhip_mesh {
	int nelem, npoin, nbface, naface, nconnface, maxnnode, maxnfael, nbtag;
	const double* coords;     /* [npoin][2] */
	const int* inpoel;        /* [nelem][maxnnode] */
	const int* nnode;         /* [nelem] (== nfael for linear 2D cells) */
	const int* esuel;         /* [nelem][maxnfael] */
	const int* elemface;      /* [nelem][maxnfael] */
	const int* intfac;        /* [naface][4] = {L, R, node0, node1} */
	const int* btags;         /* [nbface][nbtag] */
	const double* facemetric; /* [naface][3] = {nx, ny, length} */
	const double* area;       /* [nelem] */
	const double* rc;         /* [nelem+nconnface][2] */
	const double* rcbp;       /* [nbface][2] */
	const double* gr;         /* [naface][2] */
	const int* connface;      /* [nconnface][5] gconnface (mesh.hpp:60-70): cell, local face, neighbour's
	                             rank, global neighbour cell, global face; NULL when nconnface == 0 */
} fvhip_mesh;

typedef struct fvhip_ctx* fvhip_handle;

/** Text of the last error on this thread */
const char* fvhip_last_error(void);
/** Library version string */
const char* fvhip_version(void);
/** build provenance: "src_sha256_16=<first 16 hex digits of sha256 over the sorted fvens_amd/csrc
 *  .hip, .cpp and .hpp files and include/fvhip.h> arch=gfx950 extra=<experiment defines>" */
const char* fvhip_build_info(void);
/** Number of visible HIP devices (0 if none; never fails) */
int fvhip_device_count(void);

/** Builds the device-resident discretisation for a mesh on a device. A mesh with connectivity faces
 *  (nconnface > 0) is one rank's subdomain as the reference's multi-rank driver holds it
 *  (restrictMeshToPartitions, mesh/meshpartitioning.cpp:24-159): the residual is that rank's residual
 *  of the reference (flow_spatial.cpp:636-816 with its connectivity faces; the face traces and ghost
 *  gradients L2TraceVector / VecGhostUpdate exchange, tracevector.cpp:213-340, alinalg.cpp:17-29, come
 *  from the library's RCCL exchange), once fvhip_comm_init (or fvhip_set_rank + a group) gave the rank.
 *  Ghost rows of u are refreshed by the library's exchange (the rows the caller's VecGhostUpdate holds). */
int fvhip_create(const fvhip_mesh* mesh, const fvhip_flow_config* cfg, int device, fvhip_handle* out);
/** Rank of a per-rank-mesh handle within nranks (PETSC_COMM_WORLD's rank in the reference); needed
 *  before fvhip_group_create, implied by fvhip_comm_init */
int fvhip_set_rank(fvhip_handle h, int rank, int nranks);
int fvhip_destroy(fvhip_handle h);

/* ---------------------------------------------------------------------------------------------
 * Multi-GPU (one rank per GPU). Replaces the reference's partitioned mesh (meshpartitioning.cpp:
 * 24-159, Scotch :376-458) and ghost scatters (alinalg.cpp:17-29, tracevector.cpp:213-340).
 * Every rank passes the single-domain mesh and the same partition vector; the handle holds the
 * rank's owned cells plus a two-layer halo, faces in global order with global orientation, so the
 * residual of every owned cell is bitwise the single-GPU one. For WLS gradients with an unlimited or
 * MUSCL reconstruction one RCCL ncclSend/ncclRecv round of u per residual fills both halo layers
 * and the layer-1 ghosts' gradients are computed locally; other schemes exchange u, gradients and
 * limiter data in turn (one-layer exchanges).
 * -------------------------------------------------------------------------------------------- */
typedef struct fvhip_group_s* fvhip_group;
/** Recursive coordinate bisection of the cell centres into nparts (part [nelem]) */
int fvhip_partition_rcb(const fvhip_mesh* mesh, int nparts, int* part);
/** Graph partition of the cell dual graph into nparts (stand-in for the reference's Scotch
 *  SCOTCH_graphPart, mesh/meshpartitioning.cpp:376-458): recursive bisection grown breadth-first from
 *  a pseudo-peripheral cell and refined by balanced Kernighan-Lin boundary swaps */
int fvhip_partition_graph(const fvhip_mesh* mesh, int nparts, int* part);
/** The same with cell weights weight[nelem] in 1..4096 (NULL: 1): every bisection splits the total
 *  weight to within the largest weight. Not a reference option (its Scotch graph carries no vertex
 *  weights, meshpartitioning.cpp:443-444): weight = the cell's face count balances the fused residual's
 *  time per rank on a mixed triangle/quadrangle mesh (a quadrangle costs ~1.3 triangles) */
int fvhip_partition_graph_weighted(const fvhip_mesh* mesh, int nparts, const int* weight, int* part);
/** Number of interior faces cut by a partition */
long long fvhip_partition_edge_cut(const fvhip_mesh* mesh, const int* part);
/** The reference's line finder for its line orderings (host only): findLines + computeWeights,
 *  mesh/meshordering.cpp:143-264 -- from each physical boundary face's cell, walk to the neighbour of
 *  largest inverse centre distance (relative to the cell's smallest) while that ratio exceeds
 *  `threshold`. *nlines, *ncells (cells on lines); start [nlines+1] into cells [ncells] (reference cell
 *  numbers, discovery order); NULL arrays are skipped (call once for the sizes) */
int fvhip_find_lines(const fvhip_mesh* mesh, double threshold, int* nlines, int* ncells, int* start, int* cells);
/** Halo description of one rank (host only). counts[6] = {owned, ghosts, boundary faces, faces,
 *  neighbour ranks, send rows}; arrays may be NULL: cell_global [owned+ghosts] (owned ascending,
 *  then ghosts by owner rank), nbr_rank [nnbr], ghost_start/send_start [nnbr+1], send_global [nsend] */
int fvhip_partition_info(const fvhip_mesh* mesh, const int* part, int rank, int* counts, int* cell_global,
                         int* nbr_rank, int* ghost_start, int* send_start, int* send_global);
/** The two halo layers inside those lists (host only): each neighbour's ghost block and send block
 *  hold its layer-1 cells (across a face of an owned cell) first, then its layer-2 cells (across a
 *  face of a layer-1 ghost); ghost_l1_end / send_l1_end [nnbr] are where layer 1 ends (same base as
 *  ghost_start / send_start). One exchange of u fills both layers and the layer-1 ghosts' WLS
 *  gradients are then computed locally: the reference's two exchanges (state, then ghost gradients,
 *  flow_spatial.cpp:636-816) become one. */
int fvhip_partition_halo_layers(const fvhip_mesh* mesh, const int* part, int rank, int* ghost_l1_end,
                                int* send_l1_end);
/** The rank's handle; host u/r/dtm then hold the owned cells in ascending global order, device
 *  u has owned+ghost rows (fvhip_layout_stats[6] = ghosts) and the ghost rows are filled by it */
int fvhip_create_partitioned(const fvhip_mesh* mesh, const fvhip_flow_config* cfg, const int* part, int nparts,
                             int rank, int device, fvhip_handle* out);
/** RCCL communicator of the partition: rank 0 creates the 128-byte id, all ranks pass it */
int fvhip_comm_unique_id(void* id128);
int fvhip_comm_init(fvhip_handle h, int nranks, int rank, const void* id128);
/** All ranks of a partition in ONE process (e.g. on one device): exchange by device copies */
int fvhip_group_create(fvhip_handle* handles, int n, fvhip_group* out);
/** L2TraceVector::updateSharedFacesBegin + End (linalg/tracevector.cpp:213-340) on a per-rank mesh
 *  (nconnface > 0): d_left [nconnface][width] (device, the mesh's connectivity-face order) holds this
 *  rank's face values; on return d_right[icface] holds the neighbour rank's value of the same face
 *  (its left). width 1..4. RCCL ranks (fvhip_comm_init) / all ranks of a group in one process. */
int fvhip_trace_exchange_device(fvhip_handle h, const double* d_left, double* d_right, int width);
int fvhip_group_trace_exchange_device(fvhip_group g, const double* const* d_left, double* const* d_right, int width);
int fvhip_group_destroy(fvhip_group g);
int fvhip_group_compute_residual_device(fvhip_group g, const double* const* d_u, double* const* d_r,
                                        int gettimesteps, double* const* d_dtm, int flags);

/** FlowFV::compute_residual on host arrays (copies through PCIe) */
int fvhip_compute_residual(fvhip_handle h, const double* u, double* r, int gettimesteps, double* dtm);
/** Device-resident sweep; u/r/dtm in internal order. flags: FVHIP_RES_OVERWRITE = r is known
 *  to be zero on entry (as every reference caller guarantees), so it is written, not read. */
#define FVHIP_RES_OVERWRITE 1
/** flags: FVHIP_RES_STAGED = use the gradient kernel + sweep kernel even where the one-launch
 *  fused residual applies (WLS + MUSCL/unlimited linear, inviscid, single domain); same results */
#define FVHIP_RES_STAGED 2
/** flags: FVHIP_RES_PIPELINED = gradient kernel in chunks on the handle's stream, overlapped with
 *  the sweep of the patches whose inputs are ready on a second stream (single domain, WLS +
 *  MUSCL/unlimited linear, viscous too); same results. Opt-in: slower than the serial path on C4 */
#define FVHIP_RES_PIPELINED 4
/** flags: FVHIP_RES_HALO_READY = partitioned handle (two-layer halo, fused single-exchange
 *  configurations): the caller has already filled the ghost rows of d_u (both layers), as the
 *  reference's drivers do with VecGhostUpdate before compute_residual (aodesolver.cpp:514/558); no
 *  exchange runs, the layer-1 ghosts' gradients are computed and every patch is swept on the handle's
 *  stream. For a rank's compute time alone (tools/scale_proxy.py) and callers that own the exchange. */
#define FVHIP_RES_HALO_READY 8
int fvhip_compute_residual_device(fvhip_handle h, const double* d_u, double* d_r, int gettimesteps,
                                  double* d_dtm, int flags);
/** FlowFV_base::getGradients: conserved-variable gradients, GradBlock layout [nelem][4 vars][2 dims] */
int fvhip_get_gradients(fvhip_handle h, const double* u, double* grads);
/** FlowFV_base::computeSurfaceData (spatial/flow_spatial.cpp:130-310) for the device state d_u (internal
 *  order; on a partitioned handle with room for its ghost rows, which are exchanged): funcs[3] =
 *  {CL, CDp, CDsf} over the faces of boundary marker `marker` (summed over ranks); if faces is not
 *  NULL it receives (x, y, Cp, Cf) per face [nfaces][4] (host, this rank's faces in reference order). */
int fvhip_surface_data_device(fvhip_handle h, const double* d_u, int marker, double* funcs, double* faces,
                              int* nfaces);

/** FlowOutput::compute_entropy_cell (spatial/aoutput.cpp:28-62) for the device state d_u (internal order):
 *  err = sqrt(sum over cells of ((s - s_inf)/s_inf)^2 area), s = p/rho^gamma, summed over all ranks of a
 *  partitioned handle (RCCL); the reference's mesh-size parameter is 1/sqrt(global cell count) */
int fvhip_entropy_error_device(fvhip_handle h, const double* d_u, double* err);
int fvhip_group_entropy_error_device(fvhip_group g, const double* const* d_u, double* err);

/** Spatial::assemble_jacobian into block-sparse storage: diag [nelem][16] (diagonal blocks),
 *  lower/upper [ninface][16] for interior faces in face order (A[R][L] += L, A[L][R] += U). */
int fvhip_assemble_jacobian(fvhip_handle h, const double* u, double* diag, double* lower, double* upper);
/** Same on device arrays: d_u, d_diag in internal cell order; d_lower/d_upper [ninface][16] in
 *  reference interior-face order. The Jacobian flux is cfg.conv_numflux_jac (LLF/AUSM/Roe/HLL/HLLC). */
int fvhip_assemble_jacobian_device(fvhip_handle h, const double* d_u, double* d_diag, double* d_lower,
                                   double* d_upper);
/** SteadyBackwardEulerSolver::addPseudoTimeTerm (aodesolver.cpp:300-329) on device arrays:
 *  d_dtm <- area/(cfl*d_dtm); d_diag += d_dtm * I */
int fvhip_add_pseudo_time_term_device(fvhip_handle h, double cfl, double* d_dtm, double* d_diag);
/** y = A x with the face-based blocks (the product PETSc's MatMult forms, alinalg.cpp:90-119) */
int fvhip_block_apply_device(fvhip_handle h, const double* d_diag, const double* d_lower,
                             const double* d_upper, const double* d_x, double* d_y);
/** setJacobianPreallocation (alinalg.cpp:42-85) as block CSR in reference cell numbering:
 *  rowptr [nelem+1], colind [nelem + 2*ninface] sorted per row */
int fvhip_jacobian_pattern(fvhip_handle h, int* rowptr, int* colind);
/** assemble_jacobian into row-major 4x4 blocks vals [nnzb][16] of that pattern (BAIJ, bs = 4) */
int fvhip_assemble_jacobian_bsr(fvhip_handle h, const double* u, const int* rowptr, const int* colind,
                                double* vals);

/* ---------------------------------------------------------------------------------------------
 * Pseudo-time solvers on the device. States are device arrays in the
 * internal cell order; on partitioned handles they have owned + ghost rows. Partitioned handles
 * need their RCCL communicator (fvhip_comm_init); the fvhip_group_* variants drive all ranks of a
 * partition from one process.
 * -------------------------------------------------------------------------------------------- */
/** SteadyForwardEulerSolver::solve (aodesolver.cpp:135-282): explicit local-time-step iterations
 *  u += cfl dtm/area r until ||r||/||r0|| <= tol or maxiter steps; reshistory [maxiter] (may be
 *  NULL) receives the residual norms sqrt(sum r_energy^2 area) */
int fvhip_steady_forward_euler_device(fvhip_handle h, double* d_u, double cfl, double tol, int maxiter,
                                      int* steps, double* resratio, double* reshistory);
int fvhip_group_steady_forward_euler_device(fvhip_group g, double* const* d_u, double cfl, double tol, int maxiter,
                                            int* steps, double* resratio, double* reshistory);
/** TVDRKSolver::solve (aodesolver.cpp:669-758), the unsteady explicit driver, restated as written:
 *  temporal order 1-3 (initialize_TVDRK_Coeffs :45-67), dtmin = min over cells of the local time steps
 *  (over all ranks), every stage's residual at the step's start state (the reference passes uvec to
 *  compute_residual, :719), until time > finaltime - 1e-12 or maxsteps steps; returns the steps taken
 *  and the physical time reached */
int fvhip_tvdrk_device(fvhip_handle h, double* d_u, int order, double cfl, double finaltime, int maxsteps,
                       int* steps, double* time);
int fvhip_group_tvdrk_device(fvhip_group g, double* const* d_u, int order, double cfl, double finaltime, int maxsteps,
                             int* steps, double* time);

/** SteadySolverConfig of the main (or starter) solve (aodesolver.hpp, controlparser.cpp:150-206) and
 *  the linear-solver options of the reference's .solverc files */
typedef struct fvhip_implicit_config {
	double cflinit, cflfin;   /* pseudotime cfl_min / cfl_max (exponential ramp, aodesolver.cpp:110-120) */
	double tol;               /* stop when ||r||/||r0|| <= tol */
	int maxiter;              /* max_timesteps */
	int matrix_free;          /* -matrix_free_jacobian: Krylov products by finite differences
	                             (alinalg.cpp:142-233), the assembled blocks precondition */
	double mf_eps;            /* -matrix_free_difference_step (reference default 1e-7) */
	double lin_rtol;          /* -ksp_rtol: |b - A du| <= lin_rtol |b| */
	int lin_maxit;            /* -ksp_max_it: Arnoldi steps per pseudo-time step */
	int restart;              /* -ksp_gmres_restart (PETSc default 30; at most 128) */
	int prec_sweeps;          /* block-Jacobi sweeps per preconditioner application (1: point-block Jacobi) */
	double min_relax;         /* nonlinear_update_scheme: >= 1 "full"; else "robust_flow" with
	                             min_nonlinear_relaxation_factor = min_relax (nonlinearrelaxation.cpp) */
	int prec_single;          /* 1: the preconditioner's blocks (inverted diagonal, lower, upper; with
	                             prec_lines the line factors) are kept in fp32 (sweeps read half the bytes;
	                             vectors and arithmetic stay fp64). The operator itself is unchanged, so the
	                             solution tolerance is too. */
	int prec_gs;              /* 1: multicolour block Gauss-Seidel sweeps (forward/backward colour order on
	                             alternate sweeps; block-Jacobi across ranks, i.e. PETSc's bjacobi + sor)
	                             instead of block-Jacobi sweeps */
	int prec_lines;           /* 1: line-implicit preconditioner: exact block-tridiagonal solves along lines of
	                             strongly coupled cells (wall-normal in boundary layers; the coupling the
	                             reference's line ordering, mesh/ameshutils.cpp hybridLineReorder, exploits),
	                             block-Jacobi between lines and across ranks; prec_sweeps - 1 further
	                             residual-correction sweeps. Not combined with prec_gs. */
	double line_threshold;    /* a cell joins a line if its strongest coupling (face length / centre distance)
	                             is at least this many times its weakest (0: 4.0) */
	int prec_ilu;             /* 1: block ILU(0) of the assembled operator in multicolour order (the reference's
	                             -pc_type bjacobi -sub_pc_type ilu, opts.solverc / flatplate.solverc, with a colour
	                             order instead of PETSc's row order): one forward and one backward colour pass per
	                             application, block-Jacobi across ranks; prec_sweeps - 1 further residual-correction
	                             sweeps. Not combined with prec_gs / prec_lines. */
	int cgs_refine;           /* -ksp_gmres_cgs_refinement_type of the classical Gram-Schmidt step: 0 = never
	                             (PETSc's default, KSP_GMRES_CGS_REFINE_NEVER: one projection per Arnoldi step,
	                             the new vector's norm computed from the projected vector), 1 = ifneeded (a second
	                             projection when the first removed more than half of |w|^2, DGKS), 2 = always */
	int prec_amg;             /* >= 2: aggregation multigrid with this many levels (mgopts.solverc: -pc_type gamg
	                             -pc_gamg_type agg -pc_gamg_agg_nsmooths 0 -pc_mg_levels 3 -pc_mg_cycle_type v),
	                             one V-cycle per application: the one-level preconditioner (prec_lines, else
	                             point-block Jacobi) as the finest smoother, multicolour block Gauss-Seidel on the
	                             coarse levels; the coarse operators are the Galerkin sums over cell aggregates,
	                             rebuilt from every assembled Jacobian. 0: off */
	int amg_sweeps;           /* smoothing sweeps before and after the coarse correction on each level
	                             (-mg_levels_ksp_max_it; 0: the deck's 2) */
	int amg_coarse_sweeps;    /* Gauss-Seidel sweeps on the coarsest level (-mg_coarse_ksp_max_it; 0: the deck's 6) */
	double amg_threshold;     /* two cells aggregate when their coupling (face length / centre distance) is at least
	                             this fraction of both cells' strongest (-pc_gamg_threshold; 0: the deck's 0.2) */
	int amg_fine_sweeps;      /* smoothing sweeps of the finest level before and after the coarse correction
	                             (0: amg_sweeps); each costs a residual with the finest blocks and a line solve */
	double resume_res0;       /* > 0: continue a solve stopped earlier (a checkpoint): its first residual norm, so
	                             that the tolerance stays relative to it (the reference's initres, aodesolver.cpp:537) */
	double resume_res;        /*   ... its last residual norm and the one before (the CFL ramp's ratio, :462) */
	double resume_res_prev;
	double resume_cfl;        /*   ... and the CFL of its last step (the ramp continues from it) */
} fvhip_implicit_config;

typedef struct fvhip_solve_stats {
	int steps;                /* pseudo-time steps taken */
	int converged;            /* the reference's test: steps < maxiter and ratio <= tol (aodesolver.cpp:618-632) */
	int lin_iters;            /* total Krylov iterations */
	double resratio;          /* final ||r||/||r0|| */
	double cfl;               /* CFL of the last step */
	int lin_unconverged;      /* linear solves that stopped at lin_maxit above lin_rtol (PETSc's
	                             KSP_DIVERGED_ITS: not fatal, the step goes on with that update) */
	double lin_worst;         /* largest final |b - A du| / |b| over the steps' linear solves */
} fvhip_solve_stats;

/** SteadyBackwardEulerSolver::solve (aodesolver.cpp:363-638) with the linear systems solved on the
 *  device by restarted GMRES (instead of PETSc's KSPSolve, :483); reshistory [maxiter] may be NULL */
int fvhip_steady_backward_euler_device(fvhip_handle h, double* d_u, const fvhip_implicit_config* cfg,
                                       fvhip_solve_stats* stats, double* reshistory);
int fvhip_group_steady_backward_euler_device(fvhip_group g, double* const* d_u, const fvhip_implicit_config* cfg,
                                             fvhip_solve_stats* stats, double* reshistory);
/** The linear solver alone: GMRES(restart) with `sweeps` block-Jacobi sweeps as right preconditioner
 *  on the block operator (d_diag internal order [ncell][16], d_lower/d_upper [ninface][16]); solves
 *  A x = b from x = 0 until |b - A x| <= rtol |b| or maxit iterations */
int fvhip_gmres_blocks_device(fvhip_handle h, const double* d_diag, const double* d_lower, const double* d_upper,
                              const double* d_b, double* d_x, double rtol, int maxit, int restart, int sweeps,
                              int* iters, double* resnorm);

/** The line-implicit preconditioner alone (fvhip_implicit_config::prec_lines): block-Thomas factorisation
 *  of M, the block-tridiagonal part of the block operator along the lines built with `line_threshold`
 *  (0: 4), then z = M^-1 v (internal order, [ncell][4]). Blocks as in fvhip_gmres_blocks_device.
 *  single: the factors are stored in fp32 (prec_single), the recurrence runs in fp64. */
int fvhip_line_precondition_device(fvhip_handle h, const double* d_diag, const double* d_lower, const double* d_upper,
                                   double line_threshold, int single, const double* d_v, double* d_z);
/** The block ILU(0) preconditioner alone (fvhip_implicit_config::prec_ilu): factorisation of the block
 *  operator in the colour order of fvhip_colouring, then z = M^-1 v (internal order, [ncell][4]) */
int fvhip_ilu_precondition_device(fvhip_handle h, const double* d_diag, const double* d_lower, const double* d_upper,
                                  const double* d_v, double* d_z);
/** The aggregation multigrid (fvhip_implicit_config::prec_amg) alone: builds the hierarchy of `levels` levels
 *  with strength threshold `threshold` (once per handle), forms the coarse Galerkin operators of the block
 *  operator (d_diag / d_lower / d_upper as in fvhip_gmres_blocks_device), then, if d_v and d_z are given,
 *  z = M^-1 v by one V-cycle (the line-implicit finest smoother if line_threshold > 0, else point-block
 *  Jacobi; `sweeps` per level, `coarse_sweeps` on the coarsest). *nlevels = coarse levels built. */
int fvhip_amg_precondition_device(fvhip_handle h, const double* d_diag, const double* d_lower, const double* d_upper,
                                  int levels, double threshold, int sweeps, int coarse_sweeps, double line_threshold,
                                  const double* d_v, double* d_z, int* nlevels);
/** Coarse level `level` (1 = the first coarse level) of the hierarchy built by the call above: *n rows, *nnz blocks;
 *  then, where the arrays are not NULL, agg [rows of the finer level] (its aggregate), rowptr [n+1], col [nnz] and
 *  val [nnz][16] (the Galerkin blocks, row-major). Rows of level 1 aggregate the internal (Hilbert) cell order. */
int fvhip_amg_level(fvhip_handle h, int level, int* n, int* nnz, int* agg, int* rowptr, int* col, double* val);
/** The colouring of the owned cells that prec_gs and prec_ilu use (greedy over interior faces in internal
 *  order): *ncolours, colour [ncell] (internal order; may be NULL), and *triples = the number of owned
 *  cells sharing faces pairwise three at a time (0: the colour-order D-ILU is exactly ILU(0)) */
int fvhip_colouring(fvhip_handle h, int* ncolours, int* colour, long long* triples);
/** The lines of that preconditioner (pieces of at most 256 cells), longest first: *nlines; start
 *  [nlines+1] into cells [ncell] (internal ids, line order) and faces [ncell] (link of a cell to the previous
 *  one: interior face fi << 1 | (previous cell is the face's R), -1 for a line's first cell); NULL
 *  arrays are skipped */
int fvhip_lines(fvhip_handle h, double line_threshold, int* nlines, int* start, int* cells, int* faces);

/** MatrixFreeSpatialJacobian: set_state(u, r = -r(u), mdt = area/(CFL*dt)) then y = J x */
int fvhip_matfree_set_state(fvhip_handle h, const double* u, const double* r, const double* mdt);
int fvhip_matfree_apply(fvhip_handle h, const double* x, double* y);
/** Device variants (internal order). set_state keeps the pointers, as the reference keeps the Vecs.
 *  On a partitioned handle |x| is the global norm and d_u needs room for the ghost rows. d_y may alias any
 *  input: the one-launch operator (the residual kernel with the perturbation and the combination fused in)
 *  runs only when d_y shares no byte with d_x or the state d_u, else the three-launch operator does. */
int fvhip_matfree_set_state_device(fvhip_handle h, const double* d_u, const double* d_r, const double* d_mdt);
int fvhip_matfree_apply_device(fvhip_handle h, const double* d_x, double* d_y);
int fvhip_group_matfree_set_state_device(fvhip_group g, const double* const* d_u, const double* const* d_r,
                                         const double* const* d_mdt);
int fvhip_group_matfree_apply_device(fvhip_group g, const double* const* d_x, double* const* d_y);
/** -matrix_free_difference_step (default 1e-7, alinalg.cpp:124-129) */
int fvhip_matfree_set_eps(fvhip_handle h, double eps);

/** Permute a cell array [nelem][width] between reference order (host) and internal order (device) */
int fvhip_to_internal(fvhip_handle h, const double* host_ref, double* d_internal, int width);
int fvhip_from_internal(fvhip_handle h, const double* d_internal, double* host_ref, int width);
/** Internal order of cells: perm[internal] = reference cell index */
int fvhip_get_permutation(fvhip_handle h, int* perm);

/** Device scratch allocation helpers (hipMalloc on the handle's device) */
int fvhip_device_alloc(fvhip_handle h, unsigned long long bytes, void** ptr);
int fvhip_device_free(fvhip_handle h, void* ptr);
int fvhip_synchronize(fvhip_handle h);
/** The handle's HIP stream (hipStream_t as void*) */
void* fvhip_stream(fvhip_handle h);

/** Kernel timing with HIP events on the handle's stream. enable=1 starts recording every
 *  kernel launch; fvhip_kernel_times returns, per kernel id, (total ms, launches). */
int fvhip_profile(fvhip_handle h, int enable);
int fvhip_kernel_times(fvhip_handle h, int maxk, char* names, int namelen, double* ms, int* counts);

/** Layout statistics (stats[12]): [0]=cells [1]=faces [2]=face slots incl. duplicated cut faces
 *  [3]=patches [4]=max slots per patch [5]=boundary faces [6]=ghost cells [7]=neighbour ranks
 *  [8]=rows sent per exchange [9]=fused-residual patches that need no halo data (partitioned)
 *  [10]=ring-1 cells staged by the fused residual over all patches [11]=patches staging more cells
 *  than a block has threads */
int fvhip_layout_stats(fvhip_handle h, long long* stats);
/** The same statistics for a mesh and configuration without a device (host only: builds the layout
 *  fvhip_create would upload). stats[16]: [0..11] as fvhip_layout_stats, [12]=ring-2 cells staged by
 *  the fused residual over all patches, [13]=most cells one patch stages, [14]=faces per patch
 *  (threads per face-sweep block), [15]=0 */
int fvhip_layout_probe(const fvhip_mesh* mesh, const fvhip_flow_config* cfg, long long* stats);

/** Point-wise numerical flux on the device (get_flux) for nf faces: ul, ur [nf][4], n [nf][2] */
int fvhip_local_flux(int flux_type, const double* gas5, int nf, const double* ul, const double* ur,
                     const double* n, double* flux);
/** Diagnostics of the parity-mode arithmetic (not a reference interface): on the device, out[i] =
 *  {div_rn(a,b), a/b, sqrt_rn(a), sqrt(a)} -- the shortened correctly rounded division and square
 *  root of the residual kernels next to the device's full IEEE operations (gasdyn.hpp) */
int fvhip_divsqrt_probe(int n, const double* a, const double* b, double* out);
/** Point-wise flux Jacobians (get_jacobian) on the device: dfdl, dfdr [nf][16] */
int fvhip_local_flux_jacobian(int flux_type, const double* gas5, int nf, const double* ul,
                              const double* ur, const double* n, double* dfdl, double* dfdr);

/* ---------------------------------------------------------------------------------------------
 * Mesh builder (host). Produces the reference's UMesh arrays from a Gmsh-2 file or a synthetic
 * generator, index-for-index as readGmsh2 + constructMesh + preprocessMesh would on one rank.
 * ------------------------------------------------------------------------------------------- */
typedef struct fvmesh_s* fvmesh_handle;
int fvmesh_read_gmsh(const char* path, fvmesh_handle* out);
/** kind: 0 = NACA0012 hybrid O-grid (a=ntheta, b=nquad, c=ntri, x=rfar, y=wall spacing, z=far-field map:
 *            0 = direction of the surface point from mid-chord, 1 = angles uniform in the surface parameter)
 *        1 = cylinder triangle O-grid (a=ntheta, b=nr, x=r0, y=r1)
 *        2 = flat plate quads (a=nx, b=ny, x=lead length, y=height, z=wall spacing)
 *        3 = NACA 0012 C-grid (a=nsurf, b=nquad, c=ntri, x=rfar, y=wall spacing, z=nwake: columns along
 *            each wake; 2 nwake + nsurf columns of cells) */
int fvmesh_generate(int kind, int a, int b, int c, double x, double y, double z, fvmesh_handle* out);
/** NACA 0012 hybrid mesh of the visc-naca0012 grids' topology (testcases/visc-naca0012/grids/
 *  naca0012nasa-blcirc.geo, NACA0012_lam_hybrid_1.msh: a quadrangle block round the body, triangles
 *  outside it): the C-grid of kind 3 with nrows rows; quadrangles in the body's first nquad rows (the
 *  boundary layer) and in the two wake blocks (nwake columns each), near-isotropic triangles above the
 *  body's quadrangles out to the far field (radius rfar). Wall marker 2, far field 4. */
int fvmesh_generate_hybrid(int nsurf, int nwake, int nquad, int nrows, double rfar,
                           double wallspacing, fvmesh_handle* out);
int fvmesh_write_gmsh(fvmesh_handle m, const char* path);
int fvmesh_destroy(fvmesh_handle m);
/** The aggregation multigrid's first coarsening (fvhip_implicit_config::prec_amg) on the mesh's own cell order
 *  (host only): cells aggregate along couplings face length / centre distance of at least `threshold` of both
 *  cells' strongest. *nagg = aggregates, agg [nelem] = each cell's aggregate (may be NULL). The device builds the
 *  same hierarchy over its internal (Hilbert) cell order. */
int fvmesh_amg_aggregates(fvmesh_handle m, double threshold, int* nagg, int* agg);
/** TrivialReplicatedGlobalMeshPartitioner::compute_partition (meshpartitioning.cpp:354-367): cell i
 *  goes to rank i/(nelem/nranks), the remainder to the last rank */
int fvmesh_partition_trivial(int nelem, int nranks, int* elemdist);
/** ReplicatedGlobalMeshPartitioner::restrictMeshToPartitions (meshpartitioning.cpp:24-159) followed by
 *  preprocessMesh (ameshutils.cpp:40-99): rank `rank`'s subdomain of global mesh g under the cell
 *  distribution elemdist [nelem of g], with its connectivity faces; rc has nelem+nconnface rows, the
 *  ghost rows holding the neighbouring cells' centres (the Spatial ctor's ghost scatter, aspatial.cpp:41-66) */
int fvmesh_restrict(fvmesh_handle g, const int* elemdist, int rank, fvmesh_handle* out);
/** UMesh::gglobalElemIndex of a subdomain from fvmesh_restrict: gidx [nelem] */
int fvmesh_global_elem_index(fvmesh_handle m, int* gidx);
/** Fills a fvhip_mesh view whose pointers stay valid until fvmesh_destroy */
int fvmesh_view(fvmesh_handle m, fvhip_mesh* view);
/** Raw (pre-topology) arrays: npoin, nelem, maxnnode, nbface, nbtag */
int fvmesh_raw_info(fvmesh_handle m, int* info5);
int fvmesh_raw_arrays(fvmesh_handle m, double* coords, int* inpoel, int* nnode, int* bface);

#ifdef __cplusplus
}
#endif
#endif
