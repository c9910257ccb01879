"""Per-rank subdomain meshes on the device: every rank of a partition is a handle over its own
restricted mesh (restrictMeshToPartitions, meshpartitioning.cpp:24-159: connectivity faces last,
local outward normals, one ghost row per connectivity face), all ranks driven from one process as a
group (the exchange by device copies in place of RCCL). Bar: each rank's residual and time steps are
BITWISE the oracle's restatement of the reference's multi-rank residual (flow_spatial.cpp:636-816 with
the gradient ghost scatter and the L2TraceVector face-trace exchange, tracevector.cpp:213-340). Ghost
rows start as NaN so that a missed exchange cannot pass."""
import numpy as np
import pytest

import fvens_amd as fa
import _oracle as orc
import cases
from test_rankmesh import rank_states

pytestmark = pytest.mark.gpu

SCHEMES = [("naca", "ROE", "LEASTSQUARES", "VANALBADA", True),
           ("naca", "ROE", "LEASTSQUARES", "NONE", True),
           ("naca", "LLF", "NONE", "NONE", False),
           ("cyl", "HLLC", "GREENGAUSS", "VENKATAKRISHNAN", True),
           ("naca", "ROE", "LEASTSQUARES", "BARTHJESPERSEN", True),
           ("naca", "AUSM", "GREENGAUSS", "WENO", True),
           ("viscconst", "ROE", "LEASTSQUARES", "VANALBADA", True),
           ("visc", "ROE", "LEASTSQUARES", "VANALBADA", True),
           ("plate", "HLLC", "LEASTSQUARES", "NONE", True)]


def _global(kind):
    if kind == "plate":
        return fa.UMesh.flat_plate(48, 32)
    return fa.UMesh.naca_ogrid(96, 6, 18)


def run_ranks(kind, flux, grad, rec, order2, nranks, part=None):
    import torch
    gm = _global(kind)
    ogm = orc.OracleMesh.from_raw(gm.raw())
    p = cases.physics(kind)
    n = cases.numerics(flux, grad, rec, order2=order2)
    u = cases.state(gm, p, seed=11)
    d = fa.UMesh.partition_trivial(gm.nelem, nranks) if part is None else np.ascontiguousarray(part, np.int32)
    lms = [gm.restrict(d, r) for r in range(nranks)]
    us = rank_states(gm, lms, u)
    # oracle: the reference's per-rank residuals with its exchanges
    sps_o = [orc.OracleSpatial(ogm.restrict(d, r), p, n) for r in range(nranks)]
    r0 = [np.zeros((lm.nelem, 4)) for lm in lms]
    t0 = [np.zeros(lm.nelem) for lm in lms]
    orc.residual_ranks(sps_o, us, r0, True, t0)
    # device: one handle per subdomain, ranks from the group
    sps = [fa.FlowFV(lm, p, n) for lm in lms]
    for r, sp in enumerate(sps):
        sp.set_rank(r, nranks)
    dus, drs, dts, perms = [], [], [], []
    for lm, sp, ur in zip(lms, sps, us):
        perm = sp.permutation()
        perms.append(perm)
        du = torch.full((lm.nelem + lm.nconnface, 4), float("nan"), dtype=torch.float64, device="cuda")
        du[:lm.nelem] = torch.tensor(ur[perm], device="cuda")
        dus.append(du)
        drs.append(torch.full((lm.nelem, 4), float("nan"), dtype=torch.float64, device="cuda"))
        dts.append(torch.full((lm.nelem,), float("nan"), dtype=torch.float64, device="cuda"))
    torch.cuda.synchronize()  # torch's stream vs the library's (non-blocking) streams
    grp = fa.FlowFVGroup(sps)
    grp.compute_residual_device([x.data_ptr() for x in dus], [x.data_ptr() for x in drs],
                                [x.data_ptr() for x in dts], True, True)
    torch.cuda.synchronize()
    out = []
    for k in range(nranks):
        r = np.empty((lms[k].nelem, 4))
        t = np.empty(lms[k].nelem)
        r[perms[k]] = drs[k].cpu().numpy()
        t[perms[k]] = dts[k].cpu().numpy()
        out.append((r, t, r0[k], t0[k]))
    stats = [sp.layout_stats() for sp in sps]
    grp.close()
    for sp in sps:
        sp.close()
    return out, stats, lms


@pytest.mark.parametrize("kind,flux,grad,rec,order2", SCHEMES)
@pytest.mark.parametrize("nranks", [3, 8])
def test_rank_meshes_bitwise_vs_oracle(kind, flux, grad, rec, order2, nranks):
    out, stats, lms = run_ranks(kind, flux, grad, rec, order2, nranks)
    # WENO's pow and Sutherland's T^1.5 (device T*sqrt(T)): device libm vs glibc, 1e-12
    tol = 1e-12 if rec == "WENO" or kind in ("plate", "visc") else 0.0
    for k, (r, t, r0, t0) in enumerate(out):
        assert lms[k].nconnface > 0 and stats[k]["ghosts"] == lms[k].nconnface
        if tol == 0.0:
            assert np.array_equal(r, r0), f"rank {k}: max |dr| {np.abs(r - r0).max():.3e}"
            assert np.array_equal(t, t0), f"rank {k}: max |dt| {np.abs(t - t0).max():.3e}"
        else:
            assert (np.abs(r - r0).max(axis=0) <= tol * np.abs(r0).max(axis=0)).all()
            assert np.abs(t - t0).max() <= tol * np.abs(t0).max()


def test_rank_meshes_rcb_partition():
    """a geometric partition (several neighbours per rank, ghosts of one cell appearing once per
    connectivity face) through the reference's restriction: still bitwise"""
    gm = _global("naca")
    part = fa.partition_rcb(gm, 6)
    out, _, _ = run_ranks("naca", "ROE", "LEASTSQUARES", "VANALBADA", True, 6, part=part)
    for r, t, r0, t0 in out:
        assert np.array_equal(r, r0) and np.array_equal(t, t0)


@pytest.mark.parametrize("meshname,nranks", [("testhybrid", 3), ("2dcylinderhybrid", 4)])
def test_trace_exchange_known_answer(meshname, nranks):
    """MPI_TraceVector_Comm_{1,2} (tests/solvers/CMakeLists.txt:23-33, testtracevector.cpp:15-50) on the
    device: every rank fills the left trace of each connectivity face with rank*1000 + global face*10 + j,
    exchanges (L2TraceVector::updateSharedFaces), and finds in the right trace the neighbour's value
    nbdrank*1000 + global face*10 + j. The reference runs it on squareunsquad3 (3 ranks) and 2dcylquad2
    (4 ranks), gmsh-generated meshes absent here; restated on the reference's testhybrid and
    2dcylinderhybrid meshes with the reference's trivial partition (the rank counts of its tests)."""
    import torch
    gm = fa.UMesh.read_gmsh(cases.fixture_mesh(meshname))
    d = fa.UMesh.partition_trivial(gm.nelem, nranks)
    lms = [gm.restrict(d, r) for r in range(nranks)]
    p = cases.physics("cyl")
    p.bcconf = [fa.FlowBCConfig("farfield", int(t)) for t in np.unique(gm.btags[:, 0])]   # the markers it has
    n = cases.numerics("HLLC", "LEASTSQUARES", "NONE")
    sps = [fa.FlowFV(lm, p, n) for lm in lms]
    for r, sp in enumerate(sps):
        sp.set_rank(r, nranks)
    lefts, rights = [], []
    for r, lm in enumerate(lms):
        assert lm.nconnface > 0
        left = r * 1000.0 + lm.connface[:, 4:5] * 10.0 + np.arange(4)[None, :]
        lefts.append(torch.tensor(left, dtype=torch.float64, device="cuda"))
        rights.append(torch.full((lm.nconnface, 4), float("nan"), dtype=torch.float64, device="cuda"))
    grp = fa.FlowFVGroup(sps)
    grp.trace_exchange_device([x.data_ptr() for x in lefts], [x.data_ptr() for x in rights], 4)
    torch.cuda.synchronize()
    for r, lm in enumerate(lms):
        want = lm.connface[:, 2:3] * 1000.0 + lm.connface[:, 4:5] * 10.0 + np.arange(4)[None, :]
        np.testing.assert_array_equal(rights[r].cpu().numpy(), want)
    grp.close()
    for sp in sps:
        sp.close()


def test_entropy_convergence_four_rank_meshes():
    """MPI_SpatialFlow_Euler_Cylinder_LeastSquares_HLLC_Quad_EntropyConvergence (tests/inv-2dcyl/
    CMakeLists.txt:29-35: the entropy test on 4 ranks; its 2dcylquad meshes are gmsh-generated and
    absent) restated on the 2dcylinder0-3 triangle meshes: each mesh restricted to 4 per-rank meshes
    (trivial partition), solved by the group's implicit driver (first-order starter, second-order main
    solve as tests/test_gpu_convergence.py's ls_hllc_implicit case), entropy error over the ranks. The
    multi-rank discretisation is the single-rank one to rounding (connectivity faces evaluated as
    -F(uR, uL, -n)), the solves stop at a 1e-7 residual drop, so every entropy error
    must match the single-rank one to 1e-4 relative and the finest slope lies in [1.65, 2.1]."""
    import torch
    from test_gpu_convergence import CASES, solve_entropy
    grad, flux, implicit, init, main, nmesh, drop, _ = CASES["ls_hllc_implicit"]
    # point-block Jacobi on every rank: the single-rank case's multicolour Gauss-Seidel becomes
    # block-Jacobi across the ranks (as PETSc's bjacobi does) and, on 2dcylinder0, that weaker
    # preconditioner lets the CFL-5000 main solve diverge; with point-block Jacobi the 4-rank and the
    # 1-rank solves run the same preconditioner and their histories agree to rounding
    prec = dict(prec_sweeps=1, lin_rtol=1e-2)
    nranks = 4
    lh, le = [], []
    for i in range(nmesh):
        name = "2dcylinder%d" % i
        gm = fa.UMesh.read_gmsh(cases.fixture_mesh(name))
        d = fa.UMesh.partition_trivial(gm.nelem, nranks)
        lms = [gm.restrict(d, r) for r in range(nranks)]
        p = cases.physics("cyl")
        n1 = cases.numerics(flux, "NONE", "NONE", order2=False)
        n2 = cases.numerics(flux, grad, "NONE")
        starts, mains = [fa.FlowFV(lm, p, n1) for lm in lms], [fa.FlowFV(lm, p, n2) for lm in lms]
        for r in range(nranks):
            starts[r].set_rank(r, nranks)
            mains[r].set_rank(r, nranks)
        dus = []
        for lm, sp in zip(lms, mains):
            u0 = np.tile(cases.freestream(p), (lm.nelem + lm.nconnface, 1))
            du = torch.tensor(u0, device="cuda")
            du[:lm.nelem] = du[:lm.nelem][torch.tensor(sp.permutation(), device="cuda")]
            dus.append(du)
        g1, g2 = fa.FlowFVGroup(starts), fa.FlowFVGroup(mains)
        lin = dict(lin_rtol=1e-1, lin_maxit=30, restart=30, min_relax=0.2)
        lin.update(prec or {})
        g1.steady_backward_euler_device([x.data_ptr() for x in dus], fa.ImplicitConfig(
            cflinit=init[0], cflfin=init[1], tol=init[2], maxiter=init[3], **lin))
        st, _ = g2.steady_backward_euler_device([x.data_ptr() for x in dus], fa.ImplicitConfig(
            cflinit=main[0], cflfin=main[1], tol=main[2], maxiter=main[3], **lin))
        err = g2.entropy_error_device([x.data_ptr() for x in dus])
        nelem1, err1, _, st1, _ = solve_entropy(name, grad, flux, implicit, init, main, drop, prec)
        print(f"{name}: {nranks} ranks {st} entropy {err!r}; 1 rank {st1} entropy {err1!r}")
        assert st["resratio"] <= drop, st
        assert abs(err - err1) <= 1e-4 * err1, (err, err1)
        lh.append(np.log10(1.0 / np.sqrt(gm.nelem)))
        le.append(np.log10(err))
        g1.close()
        g2.close()
        for sp in starts + mains:
            sp.close()
    slopes = [(le[i] - le[i - 1]) / (lh[i] - lh[i - 1]) for i in range(1, nmesh)]
    print("4-rank slopes", slopes)
    assert 1.65 <= slopes[-1] <= 2.1, slopes
