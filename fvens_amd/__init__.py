"""fvens_amd: MI355X-native FVENS face-flux / residual sweep.

Host-side mirror of the reference's operator interface for the hot path (paths relative to
/root/reference/src):

  FlowPhysicsConfig / FlowNumericsConfig / FlowBCConfig   spatial/flow_spatial.hpp:33-55, abc.hpp
  create_flow_spatial(mesh, pconf, nconf)                 utilities/afactory.cpp:251-276
  FlowFV.compute_residual(u, r, gettimesteps, dtm)        spatial/flow_spatial.cpp:636-816
  FlowFV.getGradients(u)                                  spatial/flow_spatial.cpp:95-112
  UMesh (Gmsh-2 reader + face-indexing contract)          mesh/meshreaders.cpp, mesh/mesh.cpp

Every call goes through libfvhip.so (include/fvhip.h); there is no CPU fallback.
"""
from dataclasses import dataclass, field
import ctypes
from typing import List, Optional

import numpy as np

from . import _ffi
from ._ffi import check, dptr, iptr

# string tables mirror the reference factories (upper-cased control-file strings)
FLUXES = {"LLF": 0, "VANLEER": 1, "AUSM": 2, "AUSMPLUS": 3, "ROE": 4, "HLL": 5, "HLLC": 6}
GRADIENTS = {"NONE": 0, "ZERO": 0, "GREENGAUSS": 1, "LEASTSQUARES": 2}
RECONSTRUCTIONS = {"NONE": 0, "WENO": 1, "VANALBADA": 2, "BARTHJESPERSEN": 3, "VENKATAKRISHNAN": 4}
BCTYPES = {"slipwall": 0, "farfield": 1, "inflowoutflow": 2, "subsonic_inflow": 3, "extrapolation": 4,
           "periodic": 5, "isothermalwall": 6, "adiabaticwall": 7}


@dataclass
class FlowBCConfig:
    """FlowBCConfig (spatial/abc.hpp): bc_type string as in bcTypeMap (abctypemap.cpp:14-28)"""
    bc_type: str
    bc_tag: int
    bc_vals: List[float] = field(default_factory=list)


@dataclass
class FlowPhysicsConfig:
    """spatial/flow_spatial.hpp:33-44. Inviscid runs use Tinf=298, Reinf=inf, Pr=nan like
    controlparser.cpp:133-138."""
    gamma: float = 1.4
    Minf: float = 0.5
    Tinf: float = 298.0
    Reinf: float = float("inf")
    Pr: float = float("nan")
    aoa: float = 0.0            # radians
    viscous_sim: bool = False
    const_visc: bool = False
    bcconf: List[FlowBCConfig] = field(default_factory=list)


@dataclass
class FlowNumericsConfig:
    """spatial/flow_spatial.hpp:47-55 (limiter_param must be given: the reference never parses it)"""
    conv_numflux: str = "ROE"
    conv_numflux_jac: str = "ROE"
    gradientscheme: str = "LEASTSQUARES"
    reconstruction: str = "VANALBADA"
    limiter_param: float = 20.0
    order2: bool = True
    # Not a reference option: contracted FMAs + approximate division/sqrt in the residual sweep
    # (results within a stated tolerance instead of bitwise; include/fvhip.h)
    fast_math: bool = False


@dataclass
class ImplicitConfig:
    """One pseudo-time solve (SteadySolverConfig, ode/aodesolver.hpp; control-file keys
    pseudotime.{main,initialization}.*, controlparser.cpp:150-206) plus the linear-solver options of
    the reference's .solverc files (include/fvhip.h fvhip_implicit_config)."""
    cflinit: float = 50.0
    cflfin: float = 3000.0
    tol: float = 1e-8
    maxiter: int = 100
    matrix_free: bool = False       # -matrix_free_jacobian
    mf_eps: float = 1e-7            # -matrix_free_difference_step
    lin_rtol: float = 1e-2          # -ksp_rtol
    lin_maxit: int = 30             # -ksp_max_it
    restart: int = 30               # -ksp_gmres_restart
    prec_sweeps: int = 1            # block-Jacobi sweeps per preconditioner application
    min_relax: float = 1.0          # nonlinear_update_scheme: >= 1 "full", else "robust_flow" factor
    prec_single: bool = False       # preconditioner blocks / line factors stored in fp32 (operator stays fp64)
    prec_gs: bool = False           # multicolour block Gauss-Seidel sweeps instead of block-Jacobi
    prec_lines: bool = False        # line-implicit (block-tridiagonal along strongly coupled lines)
    line_threshold: float = 0.0     # strongest/weakest coupling ratio for a cell to join a line (0: 4)
    prec_ilu: bool = False          # block ILU(0) in multicolour order (-sub_pc_type ilu)
    cgs_refine: int = 0             # -ksp_gmres_cgs_refinement_type: 0 never (PETSc default), 1 ifneeded, 2 always
    prec_amg: int = 0               # aggregation multigrid levels (mgopts.solverc -pc_mg_levels; 0 off)
    amg_sweeps: int = 2             # smoothing sweeps per level (-mg_levels_ksp_max_it)
    amg_coarse_sweeps: int = 6      # Gauss-Seidel sweeps on the coarsest level (-mg_coarse_ksp_max_it)
    amg_threshold: float = 0.2      # aggregation strength threshold (-pc_gamg_threshold)
    amg_fine_sweeps: int = 0        # finest-level smoothing sweeps (0: amg_sweeps)
    resume: tuple = None            # continue a checkpointed solve: (first residual, last, the one before, last CFL)

    def _struct(self):
        c = _ffi.FvImplicitConfig()
        c.cflinit, c.cflfin, c.tol, c.maxiter = float(self.cflinit), float(self.cflfin), float(self.tol), int(self.maxiter)
        c.matrix_free, c.mf_eps = int(self.matrix_free), float(self.mf_eps)
        c.lin_rtol, c.lin_maxit, c.restart = float(self.lin_rtol), int(self.lin_maxit), int(self.restart)
        c.prec_sweeps, c.min_relax = int(self.prec_sweeps), float(self.min_relax)
        c.prec_single = int(self.prec_single)
        c.prec_gs = int(self.prec_gs)
        c.prec_lines = int(self.prec_lines)
        c.line_threshold = float(self.line_threshold)
        c.prec_ilu = int(self.prec_ilu)
        c.cgs_refine = int(self.cgs_refine)
        c.prec_amg, c.amg_sweeps, c.amg_coarse_sweeps = int(self.prec_amg), int(self.amg_sweeps), int(self.amg_coarse_sweeps)
        c.amg_threshold = float(self.amg_threshold)
        c.amg_fine_sweeps = int(self.amg_fine_sweeps)
        if self.resume is not None:
            c.resume_res0, c.resume_res, c.resume_res_prev, c.resume_cfl = (float(x) for x in self.resume)
        return c


def _solve_stats(st, hist):
    n = int(st.steps)
    return dict(steps=n, converged=bool(st.converged), lin_iters=int(st.lin_iters), resratio=float(st.resratio),
                cfl=float(st.cfl), lin_unconverged=int(st.lin_unconverged), lin_worst=float(st.lin_worst)), hist[:n]


class UMesh:
    """Reference-indexed mesh built natively (mesh/mesh.hpp accessors as numpy arrays)."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle)
        v = _ffi.FvMeshView()
        check(_ffi.lib().fvmesh_view(self._h, ctypes.byref(v)))
        self.view = v
        self.nelem, self.npoin, self.nbface = v.nelem, v.npoin, v.nbface
        self.naface, self.nconnface, self.maxnnode = v.naface, v.nconnface, v.maxnnode
        self.maxnfael, self.nbtag = v.maxnfael, v.nbtag
        self.ninface = self.naface - self.nbface - self.nconnface

        def arr(p, n, dt):
            if n == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True)
        N, F, nb = self.nelem, self.naface, self.nbface
        self.coords = arr(v.coords, 2 * self.npoin, np.float64).reshape(-1, 2)
        self.inpoel = arr(v.inpoel, N * self.maxnnode, np.int32).reshape(N, -1)
        self.nnode = arr(v.nnode, N, np.int32)
        self.esuel = arr(v.esuel, N * self.maxnfael, np.int32).reshape(N, -1)
        self.elemface = arr(v.elemface, N * self.maxnfael, np.int32).reshape(N, -1)
        self.intfac = arr(v.intfac, 4 * F, np.int32).reshape(F, 4)
        self.btags = arr(v.btags, nb * self.nbtag, np.int32).reshape(nb, self.nbtag)
        self.facemetric = arr(v.facemetric, 3 * F, np.float64).reshape(F, 3)
        self.area = arr(v.area, N, np.float64)
        self.rc = arr(v.rc, 2 * (N + self.nconnface), np.float64).reshape(-1, 2)
        self.rcbp = arr(v.rcbp, 2 * nb, np.float64).reshape(-1, 2)
        self.gr = arr(v.gr, 2 * F, np.float64).reshape(F, 2)
        nc = self.nconnface
        self.connface = (arr(v.connface, 5 * nc, np.int32).reshape(nc, 5) if nc > 0
                         else np.zeros((0, 5), np.int32))

    @classmethod
    def read_gmsh(cls, path):
        h = ctypes.c_void_p()
        check(_ffi.lib().fvmesh_read_gmsh(str(path).encode(), ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def naca_ogrid(cls, ntheta, nquad, ntri, rfar=20.0, wallspacing=1e-4, farmap=0):
        """farmap 0: far-field points in the direction of the surface point from mid-chord; 1: far-field
        angles uniform in the surface parameter; + 2: layers leave the body along its normal (blended into
        the straight line to the far field; mesh.cpp generateNacaOgrid)"""
        h = ctypes.c_void_p()
        check(_ffi.lib().fvmesh_generate(0, ntheta, nquad, ntri, rfar, wallspacing, float(farmap), ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def naca_cgrid(cls, nsurf, nwake, nquad, ntri, rfar=20.0, wallspacing=1e-5):
        """C-grid round the NACA 0012: (2 nwake + nsurf) columns x (nquad quadrangle + 2 ntri triangle) rows
        (mesh.cpp generateNacaCgrid; the C5 family)"""
        h = ctypes.c_void_p()
        check(_ffi.lib().fvmesh_generate(3, nsurf, nquad, ntri, rfar, wallspacing, float(nwake), ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def naca_hybrid(cls, nsurf, nwake, nquad, nrows, rfar=20.0, wallspacing=1e-5):
        """hybrid mesh of the visc-naca0012 grids' topology: the C-grid of `naca_cgrid` with quadrangles in the
        body's first nquad rows (boundary layer) and in the wake blocks, near-isotropic triangles above the
        body's quadrangles (mesh.cpp generateNacaHybrid; the C5 family)"""
        h = ctypes.c_void_p()
        check(_ffi.lib().fvmesh_generate_hybrid(nsurf, nwake, nquad, nrows, rfar, wallspacing,
                                                ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def cylinder_ogrid(cls, ntheta, nr, r0=0.5, r1=20.0):
        h = ctypes.c_void_p()
        check(_ffi.lib().fvmesh_generate(1, ntheta, nr, 0, r0, r1, 0.0, ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def flat_plate(cls, nx, ny, xlead=0.25, height=0.5, wallspacing=1e-4):
        h = ctypes.c_void_p()
        check(_ffi.lib().fvmesh_generate(2, nx, ny, 0, xlead, height, wallspacing, ctypes.byref(h)))
        return cls(h.value)

    def amg_aggregates(self, threshold=0.2):
        """the aggregation multigrid's first coarsening on this mesh's cell order (host only): (aggregates, agg per cell)"""
        n = np.zeros(1, np.int32)
        agg = np.zeros(self.nelem, np.int32)
        check(_ffi.lib().fvmesh_amg_aggregates(self._h, float(threshold), iptr(n), iptr(agg)))
        return int(n[0]), agg

    @staticmethod
    def partition_trivial(nelem, nranks):
        """TrivialReplicatedGlobalMeshPartitioner::compute_partition (meshpartitioning.cpp:354-367)"""
        d = np.zeros(nelem, np.int32)
        check(_ffi.lib().fvmesh_partition_trivial(int(nelem), int(nranks), iptr(d)))
        return d

    def restrict(self, elemdist, rank):
        """restrictMeshToPartitions + preprocessMesh (meshpartitioning.cpp:24-159): rank `rank`'s
        subdomain with its connectivity faces (the mesh each MPI rank of the reference holds)"""
        d = np.ascontiguousarray(elemdist, np.int32)
        h = ctypes.c_void_p()
        check(_ffi.lib().fvmesh_restrict(self._h, iptr(d), int(rank), ctypes.byref(h)))
        return UMesh(h.value)

    def global_elem_index(self):
        g = np.zeros(self.nelem, np.int32)
        check(_ffi.lib().fvmesh_global_elem_index(self._h, iptr(g)))
        return g

    def raw(self):
        """Pre-topology arrays (as read/generated): coords, inpoel, nnode, bface, nbtag"""
        info = np.zeros(5, np.int32)
        check(_ffi.lib().fvmesh_raw_info(self._h, iptr(info)))
        npoin, nelem, maxnnode, nbface, nbtag = [int(x) for x in info]
        coords = np.zeros(2 * npoin)
        inpoel = np.zeros(nelem * maxnnode, np.int32)
        nnode = np.zeros(nelem, np.int32)
        bface = np.zeros(nbface * (2 + nbtag), np.int32)
        check(_ffi.lib().fvmesh_raw_arrays(self._h, dptr(coords), iptr(inpoel), iptr(nnode), iptr(bface)))
        return dict(npoin=npoin, nelem=nelem, maxnnode=maxnnode, nbface=nbface, nbtag=nbtag,
                    coords=coords, inpoel=inpoel, nnode=nnode, bface=bface)

    def write_gmsh(self, path):
        check(_ffi.lib().fvmesh_write_gmsh(self._h, str(path).encode()))

    def __del__(self):
        try:
            if self._h:
                _ffi.lib().fvmesh_destroy(self._h)
                self._h = None
        except Exception:
            pass


def _named(table, name, what):
    """the factories' string -> scheme lookup (afactory.cpp:38-81, 178-211; abc.cpp:460-500): an unknown
    name is refused here (the reference prints a warning and returns nullptr, dereferenced later)"""
    try:
        return table[name]
    except KeyError:
        raise ValueError(f"{what} {name!r} not available (one of {', '.join(table)})") from None


def _config_struct(pconf: FlowPhysicsConfig, nconf: FlowNumericsConfig):
    n = len(pconf.bcconf)
    types = np.array([_named(BCTYPES, b.bc_type.lower(), "boundary condition") for b in pconf.bcconf], np.int32)
    tags = np.array([b.bc_tag for b in pconf.bcconf], np.int32)
    vals = np.zeros(2 * max(n, 1))
    for i, b in enumerate(pconf.bcconf):
        for j, x in enumerate(b.bc_vals[:2]):
            vals[2 * i + j] = x
    c = _ffi.FvFlowConfig()
    c.gamma, c.Minf, c.Tinf, c.Reinf, c.Pr, c.aoa = (pconf.gamma, pconf.Minf, pconf.Tinf, pconf.Reinf,
                                                     pconf.Pr, pconf.aoa)
    c.viscous_sim, c.const_visc = int(pconf.viscous_sim), int(pconf.const_visc)
    c.conv_numflux = _named(FLUXES, nconf.conv_numflux.upper(), "inviscid flux")
    c.fast_math = int(getattr(nconf, "fast_math", False))
    c.conv_numflux_jac = _named(FLUXES, nconf.conv_numflux_jac.upper(), "inviscid flux (Jacobian)")
    grad = nconf.gradientscheme.upper()
    c.gradientscheme = GRADIENTS.get(grad, 0)
    c.reconstruction = _named(RECONSTRUCTIONS, nconf.reconstruction.upper(), "reconstruction")
    c.limiter_param = nconf.limiter_param
    c.order2 = int(nconf.order2 and grad != "NONE")       # controlparser.cpp:180-181
    c.nbc = n
    keep = (types, tags, vals)
    c.bc_type, c.bc_tag, c.bc_vals = iptr(types), iptr(tags), dptr(vals)
    return c, keep


class FlowFV:
    """Device-resident FlowFV<freal,order2,constVisc> (spatial/flow_spatial.hpp:174-320)."""

    def __init__(self, mesh: UMesh, pconf: FlowPhysicsConfig, nconf: FlowNumericsConfig, device: int = 0,
                 partition=None, rank: int = 0):
        """partition: per-cell part array (e.g. UMesh.partition_rcb) -> this handle is rank `rank`'s
        piece with one ghost layer (multi-GPU); None -> the whole mesh."""
        self.mesh, self.pconf, self.nconf = mesh, pconf, nconf
        cfg, self._keep = _config_struct(pconf, nconf)
        h = ctypes.c_void_p()
        self.rank, self.nparts = rank, 1
        if partition is None:
            # a per-rank mesh (nconnface > 0) is one MPI rank's subdomain of the reference
            check(_ffi.lib().fvhip_create(ctypes.byref(mesh.view), ctypes.byref(cfg), device, ctypes.byref(h)))
            self.nown, self.nghost = mesh.nelem, mesh.nconnface
        else:
            part = np.ascontiguousarray(partition, np.int32)
            self.nparts = int(part.max()) + 1
            check(_ffi.lib().fvhip_create_partitioned(ctypes.byref(mesh.view), ctypes.byref(cfg), iptr(part),
                                                      self.nparts, rank, device, ctypes.byref(h)))
        self._h = h
        if partition is not None:
            st = self.layout_stats()
            self.nown, self.nghost = st["cells"], st["ghosts"]

    def set_rank(self, rank, nranks):
        """rank of a per-rank-mesh handle (before group use; comm_init implies it)"""
        check(_ffi.lib().fvhip_set_rank(self._h, int(rank), int(nranks)))
        self.rank, self.nparts = rank, nranks

    def comm_init(self, nranks, rank, uid):
        """RCCL communicator of the partition (uid: 128 bytes from comm_unique_id on rank 0)"""
        buf = ctypes.create_string_buffer(bytes(uid), 128)
        check(_ffi.lib().fvhip_comm_init(self._h, nranks, rank, buf))

    def trace_exchange_device(self, d_left, d_right, width=4):
        """L2TraceVector::updateSharedFaces (tracevector.cpp:213-340) of this RCCL rank's per-rank mesh"""
        check(_ffi.lib().fvhip_trace_exchange_device(self._h, ctypes.c_void_p(d_left), ctypes.c_void_p(d_right),
                                                     int(width)))

    # --- reference-ordered host interface -----------------------------------------------------
    def compute_residual(self, u, r, gettimesteps=False, dtm=None):
        """Adds -r(u) into r (flow_spatial.hpp:73-87); fills dtm if gettimesteps."""
        N = self.nown
        assert u.shape[1] == 4 and u.shape[0] >= N and r.shape == (N, 4)
        if gettimesteps:
            assert dtm is not None and dtm.shape == (N,)
        check(_ffi.lib().fvhip_compute_residual(self._h, dptr(u), dptr(r), int(gettimesteps),
                                                dptr(dtm) if gettimesteps else None))
        return r

    def getGradients(self, u):
        """GradBlock_t array [nelem][4 vars][2 dims] of conserved-variable gradients"""
        g = np.zeros((self.mesh.nelem, 4, 2))
        check(_ffi.lib().fvhip_get_gradients(self._h, dptr(u), dptr(g)))
        return g

    def surface_data_device(self, d_u, marker):
        """FlowFV_base::computeSurfaceData (flow_spatial.cpp:130-310) for the device state d_u
        (internal order): ((CL, CDp, CDsf), per-face (x, y, Cp, Cf) of this handle's faces of `marker`)"""
        funcs = np.zeros(3)
        faces = np.zeros((max(self.mesh.nbface, 1), 4))
        nf = np.zeros(1, np.int32)
        check(_ffi.lib().fvhip_surface_data_device(self._h, ctypes.c_void_p(d_u), int(marker), dptr(funcs),
                                                   dptr(faces), iptr(nf)))
        return tuple(float(x) for x in funcs), faces[:int(nf[0])]

    def entropy_error_device(self, d_u):
        """FlowOutput::compute_entropy_cell (aoutput.cpp:28-62): L2 entropy error of the device state"""
        e = np.zeros(1)
        check(_ffi.lib().fvhip_entropy_error_device(self._h, ctypes.c_void_p(d_u), dptr(e)))
        return float(e[0])

    def assemble_jacobian(self, u, diag=None, lower=None, upper=None):
        """Spatial::assemble_jacobian (aspatial.cpp:242-340): blocks are ADDED into diag [nelem][4][4],
        lower/upper [ninface][4][4] (A[R][L] += lower, A[L][R] += upper); zeros if not given."""
        N, Fi = self.mesh.nelem, self.mesh.naface - self.mesh.nbface
        diag = np.zeros((N, 4, 4)) if diag is None else diag
        lower = np.zeros((Fi, 4, 4)) if lower is None else lower
        upper = np.zeros((Fi, 4, 4)) if upper is None else upper
        check(_ffi.lib().fvhip_assemble_jacobian(self._h, dptr(u), dptr(diag), dptr(lower), dptr(upper)))
        return diag, lower, upper

    def jacobian_pattern(self):
        """Block-CSR pattern of the Jacobian (setJacobianPreallocation, alinalg.cpp:42-85)"""
        N, Fi = self.mesh.nelem, self.mesh.naface - self.mesh.nbface
        rowptr = np.zeros(N + 1, np.int32)
        colind = np.zeros(N + 2 * Fi, np.int32)
        check(_ffi.lib().fvhip_jacobian_pattern(self._h, iptr(rowptr), iptr(colind)))
        return rowptr, colind

    def assemble_jacobian_bsr(self, u, rowptr, colind):
        vals = np.zeros((int(rowptr[-1]), 4, 4))
        check(_ffi.lib().fvhip_assemble_jacobian_bsr(self._h, dptr(u), iptr(rowptr), iptr(colind), dptr(vals)))
        return vals

    def matfree_set_state(self, u, r, mdt):
        """MatrixFreeSpatialJacobian::set_state (alinalg.cpp:131-140); r = -r(u), mdt = area/(CFL dt)"""
        self._mf = (np.ascontiguousarray(u), np.ascontiguousarray(r), np.ascontiguousarray(mdt))
        check(_ffi.lib().fvhip_matfree_set_state(self._h, *[dptr(a) for a in self._mf]))

    def matfree_apply(self, x):
        """MatrixFreeSpatialJacobian::apply (alinalg.cpp:142-233)"""
        y = np.zeros((self.mesh.nelem, 4))
        check(_ffi.lib().fvhip_matfree_apply(self._h, dptr(np.ascontiguousarray(x)), dptr(y)))
        return y

    def matfree_set_eps(self, eps):
        check(_ffi.lib().fvhip_matfree_set_eps(self._h, float(eps)))

    # --- device-resident interface (internal cell order) -----------------------------------------
    def assemble_jacobian_device(self, d_u, d_diag, d_lower, d_upper):
        check(_ffi.lib().fvhip_assemble_jacobian_device(self._h, *[ctypes.c_void_p(p) for p in
                                                                   (d_u, d_diag, d_lower, d_upper)]))

    def add_pseudo_time_term_device(self, cfl, d_dtm, d_diag):
        check(_ffi.lib().fvhip_add_pseudo_time_term_device(self._h, float(cfl), ctypes.c_void_p(d_dtm),
                                                           ctypes.c_void_p(d_diag)))

    def block_apply_device(self, d_diag, d_lower, d_upper, d_x, d_y):
        check(_ffi.lib().fvhip_block_apply_device(self._h, *[ctypes.c_void_p(p) for p in
                                                             (d_diag, d_lower, d_upper, d_x, d_y)]))

    def steady_forward_euler_device(self, d_u, cfl, tol, maxiter):
        """SteadyForwardEulerSolver::solve on the device (aodesolver.cpp:170-240); returns
        (steps, final residual ratio, residual-norm history)"""
        steps = np.zeros(1, np.int32)
        ratio = np.zeros(1)
        hist = np.zeros(max(int(maxiter), 1))
        check(_ffi.lib().fvhip_steady_forward_euler_device(self._h, ctypes.c_void_p(d_u), float(cfl), float(tol),
                                                           int(maxiter), iptr(steps), dptr(ratio), dptr(hist)))
        return int(steps[0]), float(ratio[0]), hist[:int(steps[0])]

    def tvdrk_device(self, d_u, order, cfl, finaltime, maxsteps):
        """TVDRKSolver::solve on the device (aodesolver.cpp:669-758); returns (steps, physical time)"""
        steps = np.zeros(1, np.int32)
        t = np.zeros(1)
        check(_ffi.lib().fvhip_tvdrk_device(self._h, ctypes.c_void_p(d_u), int(order), float(cfl), float(finaltime),
                                            int(maxsteps), iptr(steps), dptr(t)))
        return int(steps[0]), float(t[0])

    def steady_backward_euler_device(self, d_u, cfg: ImplicitConfig):
        """SteadyBackwardEulerSolver::solve on the device (aodesolver.cpp:363-638), linear systems by
        device GMRES; returns (stats dict, residual-norm history)"""
        st = _ffi.FvSolveStats()
        hist = np.zeros(max(int(cfg.maxiter), 1))
        c = cfg._struct()
        try:
            check(_ffi.lib().fvhip_steady_backward_euler_device(self._h, ctypes.c_void_p(d_u), ctypes.byref(c),
                                                                ctypes.byref(st), dptr(hist)))
        except RuntimeError as e:
            # a diverged solve: the residual norms of the steps before the failing one travel with the error
            e.history = hist[:int(np.count_nonzero(hist))].copy()
            raise
        return _solve_stats(st, hist)

    def gmres_blocks_device(self, d_diag, d_lower, d_upper, d_b, d_x, rtol, maxit, restart=30, sweeps=1):
        """x = A^-1 b by device GMRES + block-Jacobi sweeps on face blocks; returns (iterations, |b - A x|)"""
        it = np.zeros(1, np.int32)
        rn = np.zeros(1)
        check(_ffi.lib().fvhip_gmres_blocks_device(self._h, *[ctypes.c_void_p(p) for p in
                                                              (d_diag, d_lower, d_upper, d_b, d_x)],
                                                   float(rtol), int(maxit), int(restart), int(sweeps), iptr(it), dptr(rn)))
        return int(it[0]), float(rn[0])

    def line_precondition_device(self, d_diag, d_lower, d_upper, d_v, d_z, line_threshold=0.0, single=False):
        """z = M^-1 v, M the block-tridiagonal line part of the block operator (prec_lines; single: the
        factors in fp32, as prec_single)"""
        check(_ffi.lib().fvhip_line_precondition_device(self._h, *[ctypes.c_void_p(p) for p in (d_diag, d_lower, d_upper)],
                                                        float(line_threshold), int(single), ctypes.c_void_p(d_v),
                                                        ctypes.c_void_p(d_z)))

    def ilu_precondition_device(self, d_diag, d_lower, d_upper, d_v, d_z):
        """z = M^-1 v, M the block ILU(0) of the block operator in colour order (prec_ilu)"""
        check(_ffi.lib().fvhip_ilu_precondition_device(self._h, *[ctypes.c_void_p(p) for p in
                                                                  (d_diag, d_lower, d_upper, d_v, d_z)]))

    def amg_precondition_device(self, d_diag, d_lower, d_upper, levels=5, threshold=0.2, sweeps=2, coarse_sweeps=10,
                                line_threshold=0.0, d_v=None, d_z=None):
        """the aggregation multigrid on the block operator (prec_amg): builds the hierarchy (once per handle) and
        the Galerkin coarse operators, then z = M^-1 v by one V-cycle if d_v / d_z are given; returns the number
        of coarse levels"""
        nl = np.zeros(1, np.int32)
        check(_ffi.lib().fvhip_amg_precondition_device(self._h, *[ctypes.c_void_p(p) for p in (d_diag, d_lower, d_upper)],
                                                       int(levels), float(threshold), int(sweeps), int(coarse_sweeps),
                                                       float(line_threshold), ctypes.c_void_p(d_v), ctypes.c_void_p(d_z),
                                                       iptr(nl)))
        return int(nl[0])

    def amg_level(self, level):
        """coarse level `level` (1 = first) of the multigrid hierarchy: dict(agg, rowptr, col, val[nnz][4][4])"""
        n, nnz = np.zeros(1, np.int32), np.zeros(1, np.int32)
        check(_ffi.lib().fvhip_amg_level(self._h, int(level), iptr(n), iptr(nnz), None, None, None, None))
        nf = self.nown if level == 1 else self.amg_level(level - 1)["n"]
        agg, rowptr = np.zeros(nf, np.int32), np.zeros(int(n[0]) + 1, np.int32)
        col, val = np.zeros(int(nnz[0]), np.int32), np.zeros((int(nnz[0]), 4, 4))
        check(_ffi.lib().fvhip_amg_level(self._h, int(level), iptr(n), iptr(nnz), iptr(agg), iptr(rowptr), iptr(col),
                                         dptr(val)))
        return dict(n=int(n[0]), agg=agg, rowptr=rowptr, col=col, val=val)

    def colouring(self):
        """(colour per owned cell in internal order, number of pairwise-adjacent cell triples)"""
        nc = np.zeros(1, np.int32)
        tr = ctypes.c_longlong(0)
        col = np.zeros(self.nown, np.int32)
        check(_ffi.lib().fvhip_colouring(self._h, iptr(nc), iptr(col), ctypes.byref(tr)))
        return col, int(tr.value)

    def lines(self, line_threshold=0.0):
        """the preconditioner's lines: list of (cells, faces) in line order, internal cell ids; faces[k] =
        interior face fi << 1 | (cells[k-1] is its R) linking cells[k-1] and cells[k] (-1 at k = 0)"""
        nl = np.zeros(1, np.int32)
        check(_ffi.lib().fvhip_lines(self._h, float(line_threshold), iptr(nl), None, None, None))
        n = self.nown
        st = np.zeros(int(nl[0]) + 1, np.int32)
        cells = np.zeros(n, np.int32)
        faces = np.zeros(n, np.int32)
        check(_ffi.lib().fvhip_lines(self._h, float(line_threshold), iptr(nl), iptr(st), iptr(cells), iptr(faces)))
        return [(cells[st[i]:st[i+1]], faces[st[i]:st[i+1]]) for i in range(int(nl[0]))]

    def matfree_set_state_device(self, d_u, d_r, d_mdt):
        check(_ffi.lib().fvhip_matfree_set_state_device(self._h, *[ctypes.c_void_p(p) for p in (d_u, d_r, d_mdt)]))

    def matfree_apply_device(self, d_x, d_y):
        check(_ffi.lib().fvhip_matfree_apply_device(self._h, ctypes.c_void_p(d_x), ctypes.c_void_p(d_y)))

    def compute_residual_device(self, d_u, d_r, d_dtm=None, gettimesteps=False, overwrite=True, staged=False,
                                pipelined=False, halo_ready=False):
        """staged=True forces the gradient + sweep kernels one after the other, pipelined=True the
        gradient chunks overlapped with the sweep groups (FVHIP_RES_STAGED / FVHIP_RES_PIPELINED);
        every path gives the same bits. halo_ready=True (partitioned handles): the ghost rows of d_u
        are current, no exchange runs (FVHIP_RES_HALO_READY)"""
        check(_ffi.lib().fvhip_compute_residual_device(self._h, ctypes.c_void_p(d_u), ctypes.c_void_p(d_r),
                                                       int(gettimesteps), ctypes.c_void_p(d_dtm or 0),
                                                       (1 if overwrite else 0) | (2 if staged else 0) |
                                                       (4 if pipelined else 0) | (8 if halo_ready else 0)))

    def permutation(self):
        p = np.zeros(self.nown, np.int32)
        check(_ffi.lib().fvhip_get_permutation(self._h, iptr(p)))
        return p

    def stream(self):
        return _ffi.lib().fvhip_stream(self._h)

    def synchronize(self):
        check(_ffi.lib().fvhip_synchronize(self._h))

    def profile(self, enable=True):
        check(_ffi.lib().fvhip_profile(self._h, int(enable)))

    def kernel_times(self):
        maxk, nl = 32, 64
        names = ctypes.create_string_buffer(maxk * nl)
        ms = np.zeros(maxk)
        cnt = np.zeros(maxk, np.int32)
        n = _ffi.lib().fvhip_kernel_times(self._h, maxk, names, nl, dptr(ms), iptr(cnt))
        if n < 0:
            raise RuntimeError(_ffi.lib().fvhip_last_error().decode())
        out = {}
        for i in range(n):
            nm = names.raw[i * nl:(i + 1) * nl].split(b"\0")[0].decode()
            out[nm] = (float(ms[i]), int(cnt[i]))
        return out

    def layout_stats(self):
        s = (ctypes.c_longlong * 12)()
        check(_ffi.lib().fvhip_layout_stats(self._h, s))
        return dict(zip(LAYOUT_KEYS[:12], [int(x) for x in s]))

    def close(self):
        if getattr(self, "_h", None):
            _ffi.lib().fvhip_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def create_flow_spatial(mesh, pconf, nconf, device=0):
    """create_const_flowSpatialDiscretization (afactory.cpp:251-276)"""
    return FlowFV(mesh, pconf, nconf, device)


def local_flux(flux, gas, ul, ur, n):
    """InviscidFlux::get_flux on the device for arrays of faces; gas = (g, Minf, Tinf, Reinf, Pr)"""
    ul = np.ascontiguousarray(ul, np.float64)
    ur = np.ascontiguousarray(ur, np.float64)
    n = np.ascontiguousarray(n, np.float64)
    out = np.zeros_like(ul)
    g = np.array(gas, np.float64)
    check(_ffi.lib().fvhip_local_flux(_named(FLUXES, flux.upper(), "inviscid flux") if isinstance(flux, str) else flux, dptr(g),
                                      ul.shape[0], dptr(ul), dptr(ur), dptr(n), dptr(out)))
    return out


def local_flux_jacobian(flux, gas, ul, ur, n):
    """InviscidFlux::get_jacobian on the device: (dfdl, dfdr) [nf][4][4] with dfdl = -dF/dul"""
    ul = np.ascontiguousarray(ul, np.float64)
    ur = np.ascontiguousarray(ur, np.float64)
    n = np.ascontiguousarray(n, np.float64)
    nf = ul.shape[0]
    dl = np.zeros((nf, 4, 4))
    dr = np.zeros((nf, 4, 4))
    g = np.array(gas, np.float64)
    check(_ffi.lib().fvhip_local_flux_jacobian(_named(FLUXES, flux.upper(), "inviscid flux") if isinstance(flux, str) else flux, dptr(g),
                                               nf, dptr(ul), dptr(ur), dptr(n), dptr(dl), dptr(dr)))
    return dl, dr


def comm_unique_id():
    """128-byte RCCL unique id (create on rank 0, broadcast, pass to FlowFV.comm_init)"""
    buf = ctypes.create_string_buffer(128)
    check(_ffi.lib().fvhip_comm_unique_id(buf))
    return bytes(buf.raw)


def cell_face_counts(mesh):
    """faces per cell (3 triangle, 4 quadrangle): the work weights of partition_graph(weights="faces")"""
    return np.ascontiguousarray(mesh.raw()["nnode"], np.int32)


# fused-residual cost of a triangle : quadrangle, measured per rank on C4 split 8 ways
# (profiles/r03/scale_proxy_faces2.jsonl: a quadrangle ~1.44 triangles)
RESIDUAL_COST_WEIGHTS = (7, 10)


def partition_graph(mesh, nparts, weights=None):
    """Graph partition of the cell dual graph (stand-in for the reference's Scotch, absent here).
    weights: None (every cell 1, as the reference's Scotch graph), "faces" (the cell's face count),
    "cost" (RESIDUAL_COST_WEIGHTS: the fused residual's measured cost of a triangle / quadrangle) or an
    int array [nelem]"""
    part = np.zeros(mesh.nelem, np.int32)
    if weights is None:
        check(_ffi.lib().fvhip_partition_graph(ctypes.byref(mesh.view), int(nparts), iptr(part)))
        return part
    if isinstance(weights, str) and weights == "cost":
        weights = np.where(cell_face_counts(mesh) == 4, RESIDUAL_COST_WEIGHTS[1], RESIDUAL_COST_WEIGHTS[0])
    w = cell_face_counts(mesh) if isinstance(weights, str) and weights == "faces" else np.ascontiguousarray(weights, np.int32)
    if w.shape != (mesh.nelem,):
        raise ValueError("partition_graph: weights must be 'faces' or one int per cell")
    check(_ffi.lib().fvhip_partition_graph_weighted(ctypes.byref(mesh.view), int(nparts), iptr(w), iptr(part)))
    return part


def find_lines(mesh, threshold):
    """the reference's line finder (mesh/meshordering.cpp:143-264, findLines): list of int arrays of
    reference cell numbers, in discovery order"""
    nl, nc = np.zeros(1, np.int32), np.zeros(1, np.int32)
    check(_ffi.lib().fvhip_find_lines(ctypes.byref(mesh.view), float(threshold), iptr(nl), iptr(nc), None, None))
    st = np.zeros(int(nl[0]) + 1, np.int32)
    cells = np.zeros(max(int(nc[0]), 1), np.int32)
    check(_ffi.lib().fvhip_find_lines(ctypes.byref(mesh.view), float(threshold), iptr(nl), iptr(nc), iptr(st),
                                      iptr(cells)))
    return [cells[st[i]:st[i + 1]].copy() for i in range(int(nl[0]))]


def partition_edge_cut(mesh, part):
    """interior faces whose cells lie in different parts"""
    p = np.ascontiguousarray(part, np.int32)
    c = _ffi.lib().fvhip_partition_edge_cut(ctypes.byref(mesh.view), iptr(p))
    if c < 0:
        raise RuntimeError(_ffi.lib().fvhip_last_error().decode())
    return int(c)


def partition_rcb(mesh, nparts):
    """Recursive coordinate bisection of the cell centres (Scotch is not available here)"""
    part = np.zeros(mesh.nelem, np.int32)
    check(_ffi.lib().fvhip_partition_rcb(ctypes.byref(mesh.view), int(nparts), iptr(part)))
    return part


def partition_info(mesh, part, rank):
    """Host-side halo description of `rank` (fvhip_partition_info)"""
    part = np.ascontiguousarray(part, np.int32)
    counts = np.zeros(6, np.int32)
    null = ctypes.POINTER(ctypes.c_int)()
    check(_ffi.lib().fvhip_partition_info(ctypes.byref(mesh.view), iptr(part), rank, iptr(counts),
                                          null, null, null, null, null))
    nown, ngh, nb, nf, nnbr, nsend = [int(x) for x in counts]
    cg = np.zeros(nown + ngh, np.int32)
    nbr = np.zeros(max(nnbr, 1), np.int32)
    gs = np.zeros(nnbr + 1, np.int32)
    ss = np.zeros(nnbr + 1, np.int32)
    sg = np.zeros(max(nsend, 1), np.int32)
    check(_ffi.lib().fvhip_partition_info(ctypes.byref(mesh.view), iptr(part), rank, iptr(counts), iptr(cg),
                                          iptr(nbr), iptr(gs), iptr(ss), iptr(sg)))
    g1 = np.zeros(max(nnbr, 1), np.int32)
    s1 = np.zeros(max(nnbr, 1), np.int32)
    check(_ffi.lib().fvhip_partition_halo_layers(ctypes.byref(mesh.view), iptr(part), rank, iptr(g1), iptr(s1)))
    return dict(owned=nown, ghosts=ngh, bfaces=nb, faces=nf, cell_global=cg, nbr_rank=nbr[:nnbr],
                ghost_start=gs, send_start=ss, send_global=sg[:nsend], ghost_l1_end=g1[:nnbr], send_l1_end=s1[:nnbr])


LAYOUT_KEYS = ("cells", "faces", "slots", "patches", "max_slots", "bfaces", "ghosts", "neighbours", "send_rows",
               "interior_patches", "ring1_cells", "patches_over_block", "ring2_cells", "max_staged_cells",
               "slots_per_patch")


def layout_probe(mesh, pconf, nconf):
    """Layout statistics of the device layout a FlowFV would build, computed on the host only
    (fvhip_layout_probe; no device needed)"""
    cfg, keep = _config_struct(pconf, nconf)
    s = (ctypes.c_longlong * 16)()
    check(_ffi.lib().fvhip_layout_probe(ctypes.byref(mesh.view), ctypes.byref(cfg), s))
    del keep
    return dict(zip(LAYOUT_KEYS, [int(x) for x in s]))


class FlowFVGroup:
    """All ranks of one partition driven from one process (device copies instead of RCCL)."""

    def __init__(self, spatials):
        self.sps = list(spatials)
        arr = (ctypes.c_void_p * len(self.sps))(*[s._h.value for s in self.sps])
        g = ctypes.c_void_p()
        check(_ffi.lib().fvhip_group_create(arr, len(self.sps), ctypes.byref(g)))
        self._g = g

    def compute_residual_device(self, d_us, d_rs, d_dts=None, gettimesteps=False, overwrite=True):
        n = len(self.sps)
        P = ctypes.c_void_p * n
        u, r = P(*d_us), P(*d_rs)
        d = P(*(d_dts if d_dts else [0] * n))
        check(_ffi.lib().fvhip_group_compute_residual_device(self._g, u, r, int(gettimesteps), d,
                                                             1 if overwrite else 0))

    def _ptrs(self, ps):
        return (ctypes.c_void_p * len(self.sps))(*ps)

    def steady_forward_euler_device(self, d_us, cfl, tol, maxiter):
        steps = np.zeros(1, np.int32)
        ratio = np.zeros(1)
        hist = np.zeros(max(int(maxiter), 1))
        check(_ffi.lib().fvhip_group_steady_forward_euler_device(self._g, self._ptrs(d_us), float(cfl), float(tol),
                                                                 int(maxiter), iptr(steps), dptr(ratio), dptr(hist)))
        return int(steps[0]), float(ratio[0]), hist[:int(steps[0])]

    def tvdrk_device(self, d_us, order, cfl, finaltime, maxsteps):
        steps = np.zeros(1, np.int32)
        t = np.zeros(1)
        check(_ffi.lib().fvhip_group_tvdrk_device(self._g, self._ptrs(d_us), int(order), float(cfl), float(finaltime),
                                                  int(maxsteps), iptr(steps), dptr(t)))
        return int(steps[0]), float(t[0])

    def steady_backward_euler_device(self, d_us, cfg: ImplicitConfig):
        st = _ffi.FvSolveStats()
        hist = np.zeros(max(int(cfg.maxiter), 1))
        c = cfg._struct()
        check(_ffi.lib().fvhip_group_steady_backward_euler_device(self._g, self._ptrs(d_us), ctypes.byref(c),
                                                                  ctypes.byref(st), dptr(hist)))
        return _solve_stats(st, hist)

    def trace_exchange_device(self, d_lefts, d_rights, width=4):
        """L2TraceVector::updateSharedFaces (tracevector.cpp:213-340) over the per-rank meshes of the
        group: d_lefts[r] [nconnface][width] -> each neighbour's d_rights (device arrays)"""
        check(_ffi.lib().fvhip_group_trace_exchange_device(self._g, self._ptrs(d_lefts), self._ptrs(d_rights),
                                                           int(width)))

    def entropy_error_device(self, d_us):
        e = np.zeros(1)
        check(_ffi.lib().fvhip_group_entropy_error_device(self._g, self._ptrs(d_us), dptr(e)))
        return float(e[0])

    def matfree_set_state_device(self, d_us, d_rs, d_mdts):
        check(_ffi.lib().fvhip_group_matfree_set_state_device(self._g, self._ptrs(d_us), self._ptrs(d_rs),
                                                              self._ptrs(d_mdts)))

    def matfree_apply_device(self, d_xs, d_ys):
        check(_ffi.lib().fvhip_group_matfree_apply_device(self._g, self._ptrs(d_xs), self._ptrs(d_ys)))

    def close(self):
        if getattr(self, "_g", None):
            _ffi.lib().fvhip_group_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
