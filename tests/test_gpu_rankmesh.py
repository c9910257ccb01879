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
