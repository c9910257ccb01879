"""Multi-GPU path on one device: all ranks of a partition held by one process (FlowFVGroup, the
halo exchanged by device copies instead of RCCL). Bar: every rank's owned-cell residual and time
step are BITWISE equal to the single-GPU residual of the whole mesh (faces keep global order and
orientation on every rank), with ghost rows starting as NaN so a missed exchange cannot pass."""
import numpy as np
import pytest

import fvens_amd as fa
import cases
from test_gpu_residual import get_mesh

pytestmark = pytest.mark.gpu

CONFIGS = [("naca_small", "naca", "ROE", "LEASTSQUARES", "VANALBADA", True),
           ("naca_small", "naca", "LLF", "NONE", "NONE", False),
           ("2dcylinderhybrid.msh", "cyl", "HLLC", "GREENGAUSS", "VENKATAKRISHNAN", True),
           ("naca_small", "naca", "ROE", "LEASTSQUARES", "BARTHJESPERSEN", True),
           ("naca_small", "naca", "ROE", "LEASTSQUARES", "VENKATAKRISHNAN", True),
           ("naca_small", "naca", "AUSM", "GREENGAUSS", "WENO", True),
           ("naca_small", "viscconst", "ROE", "LEASTSQUARES", "VANALBADA", True),
           ("plate_small", "plate", "HLLC", "LEASTSQUARES", "NONE", True),
           # BASELINE config 5's numerics: Roe + WLS + Van Albada + Sutherland (fused viscous, two-layer halo)
           ("naca_small", "visc", "ROE", "LEASTSQUARES", "VANALBADA", True),
           ("naca_c2", "naca", "ROE", "LEASTSQUARES", "VANALBADA", True),
           # BASELINE config 4's numerics: Roe + WLS + Venkatakrishnan (K = 20)
           ("naca_c2", "naca", "ROE", "LEASTSQUARES", "VENKATAKRISHNAN", True)]


def run_partitioned(meshkey, kind, flux, grad, rec, order2, nparts, fast=False, partitioner="rcb"):
    import torch
    m, _ = get_mesh(meshkey)
    p = cases.physics(kind)
    n = cases.numerics(flux, grad, rec, order2=order2)
    n.fast_math = fast
    u = cases.state(m, p, seed=3)
    # single GPU reference
    one = fa.FlowFV(m, p, n)
    r1 = np.zeros((m.nelem, 4))
    dt1 = np.zeros(m.nelem)
    one.compute_residual(u, r1, True, dt1)
    one.close()
    part = (fa.partition_rcb(m, nparts) if partitioner == "rcb" else
            fa.partition_graph(m, nparts, weights="cost" if partitioner == "graph-cost" else None))
    sps = [fa.FlowFV(m, p, n, partition=part, rank=k) for k in range(nparts)]
    glob = []
    dus, drs, dts = [], [], []
    for k, sp in enumerate(sps):
        owned = np.nonzero(part == k)[0]                 # local reference order = ascending global id
        g_int = owned[sp.permutation()]                  # global id of each internal owned row
        glob.append(g_int)
        du = torch.full((sp.nown + sp.nghost, 4), float("nan"), dtype=torch.float64, device="cuda")
        du[:sp.nown] = torch.tensor(u[g_int], device="cuda")
        dus.append(du)
        drs.append(torch.full((sp.nown, 4), float("nan"), dtype=torch.float64, device="cuda"))
        dts.append(torch.full((sp.nown,), float("nan"), dtype=torch.float64, device="cuda"))
    torch.cuda.synchronize()  # torch's stream vs the library's (non-blocking) streams
    grp = fa.FlowFVGroup(sps)
    grp.compute_residual_device([d.data_ptr() for d in dus], [d.data_ptr() for d in drs],
                                [d.data_ptr() for d in dts], True, True)
    torch.cuda.synchronize()
    r = np.full((m.nelem, 4), np.nan)
    dt = np.full(m.nelem, np.nan)
    for k in range(nparts):
        r[glob[k]] = drs[k].cpu().numpy()
        dt[glob[k]] = dts[k].cpu().numpy()
    stats = [sp.layout_stats() for sp in sps]
    grp.close()
    for sp in sps:
        sp.close()
    return r, dt, r1, dt1, stats


@pytest.mark.parametrize("nparts", [2, 3, 8])
@pytest.mark.parametrize("cfg", CONFIGS[:9], ids=lambda c: f"{c[0]}-{c[1]}-{c[2]}-{c[3]}-{c[4]}")
def test_partitioned_residual_bitwise(cfg, nparts):
    r, dt, r1, dt1, stats = run_partitioned(*cfg, nparts)
    assert sum(s["ghosts"] for s in stats) > 0
    if cfg[1] in ("plate",) or cfg[4] == "WENO":
        # pow() paths: the same device code on both sides, so still bitwise
        pass
    np.testing.assert_array_equal(r, r1)
    np.testing.assert_array_equal(dt, dt1)


def test_partitioned_c2_eight_ranks():
    r, dt, r1, dt1, stats = run_partitioned(*CONFIGS[9], 8)
    np.testing.assert_array_equal(r, r1)
    np.testing.assert_array_equal(dt, dt1)
    # the fused residual runs most patches before the halo arrives (overlapped with the exchange)
    for s in stats:
        assert 0 < s["interior_patches"] < s["patches"]
        assert s["interior_patches"] >= 0.7 * s["patches"], s


@pytest.mark.parametrize("partitioner", ["rcb", "graph", "graph-cost"])
def test_partitioned_c2_eight_ranks_venkatakrishnan(partitioner):
    """config 4's numerics on the partitioned path: ONE exchange of the two-layer halo, the layer-1
    ghosts' gradients AND Venkatakrishnan limiter values computed locally, the fused kernel with
    interior patches ahead of the halo -- every owned row bitwise the single-GPU residual"""
    r, dt, r1, dt1, stats = run_partitioned(*CONFIGS[10], 8, partitioner=partitioner)
    np.testing.assert_array_equal(r, r1)
    np.testing.assert_array_equal(dt, dt1)
    for s in stats:
        assert s["patches"] > 0, s                      # the fused (one-launch) residual
        assert 0 < s["interior_patches"] < s["patches"]
        assert s["interior_patches"] >= 0.7 * s["patches"], s


@pytest.mark.parametrize("rec", ["VANALBADA", "VENKATAKRISHNAN"])
def test_partitioned_c4_eight_ranks(rec):
    """BASELINE config 4 at its full size on the partitioned path the driver's 8-GPU run takes: the
    4,063,232-cell C4 mesh split 8 ways by the cost-weighted graph partitioner (bench.py's default), all
    ranks in one process (device
    copies for RCCL), overlapped schedule (interior patches, one exchange of the two-layer halo, border
    patches on the comm stream) -- every owned row's residual and time step bitwise the single-GPU ones,
    for the headline numerics and config 4's Venkatakrishnan"""
    r, dt, r1, dt1, stats = run_partitioned("naca_c4", "naca", "ROE", "LEASTSQUARES", rec, True, 8,
                                            partitioner="graph-cost")
    np.testing.assert_array_equal(r, r1)
    np.testing.assert_array_equal(dt, dt1)
    for s in stats:
        assert 0 < s["interior_patches"] < s["patches"]
    print("per-rank cells", [s["cells"] for s in stats], "ghosts", [s["ghosts"] for s in stats],
          "interior patch fraction", [round(s["interior_patches"] / s["patches"], 3) for s in stats])


def test_partitioned_c5_eight_ranks():
    """BASELINE config 5 at its full size on the partitioned path: the 8,054,616-cell hybrid C5 mesh (quadrangle
    boundary layer and wakes, 4,122,456 near-isotropic triangles outside, 1e-5 wall spacing), laminar Roe + WLS
    + unlimited linear + Sutherland at alpha 0 (the
    visc-naca0012 deck's numerics, laminar-implicit.ctrl:19,72; the fused viscous kernel on the two-layer
    halo), split 8 ways by the cost-weighted graph partitioner, all ranks in one
    process with the overlapped schedule -- every owned row's residual and time step bitwise the
    single-GPU ones (the same device code evaluates Sutherland's law on both sides)"""
    r, dt, r1, dt1, stats = run_partitioned("naca_c5", "visc", "ROE", "LEASTSQUARES", "NONE", True, 8,
                                            partitioner="graph-cost")
    assert r.shape[0] == 8054616
    np.testing.assert_array_equal(r, r1)
    np.testing.assert_array_equal(dt, dt1)
    for s in stats:
        assert s["patches"] > 0 and 0 < s["interior_patches"] < s["patches"]
    print("per-rank cells", [s["cells"] for s in stats], "ghosts", [s["ghosts"] for s in stats])


def test_partitioned_fast_math_within_tolerance():
    # fast kernels contract FMAs per inlining context (a neighbour converted from LDS or from
    # global memory), so partitioned and single-GPU fast results agree to the fast-mode tolerance
    r, dt, r1, dt1, _ = run_partitioned(*CONFIGS[0], 4, fast=True)
    scale = np.abs(r1).max(axis=0)
    assert np.all(np.abs(r - r1).max(axis=0) <= 1e-11 * scale)
    np.testing.assert_allclose(dt, dt1, rtol=1e-12, atol=0)


@pytest.mark.parametrize("nparts", [3, 8])
def test_overlapped_group_repeated_residuals(nparts):
    """the group's overlapped schedule (pack and halo copies on each rank's comm stream, interior
    patches concurrent, border patches behind the halo event; ONE exchange of the two-layer halo):
    five residuals back to back on different states, each compared bit for bit with one GPU -- a
    send buffer refilled before a receiver copied it, or a border patch ahead of its ghost gradients,
    would show up as a mismatch"""
    import torch
    m, _ = get_mesh("naca_small")
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    one = fa.FlowFV(m, p, n)
    part = fa.partition_rcb(m, nparts)
    sps = [fa.FlowFV(m, p, n, partition=part, rank=k) for k in range(nparts)]
    grp = fa.FlowFVGroup(sps)
    gl = [np.nonzero(part == k)[0][sp.permutation()] for k, sp in enumerate(sps)]
    dus = [torch.full((sp.nown + sp.nghost, 4), float("nan"), dtype=torch.float64, device="cuda") for sp in sps]
    drs = [torch.zeros((sp.nown, 4), dtype=torch.float64, device="cuda") for sp in sps]
    dts = [torch.zeros(sp.nown, dtype=torch.float64, device="cuda") for sp in sps]
    results = []
    for it in range(5):
        u = cases.state(m, p, seed=100 + it)
        for k in range(nparts):
            dus[k][:sps[k].nown] = torch.tensor(u[gl[k]], device="cuda")
        torch.cuda.synchronize()         # torch's stream and the library's streams
        grp.compute_residual_device([d.data_ptr() for d in dus], [d.data_ptr() for d in drs],
                                    [d.data_ptr() for d in dts], True, True)
        torch.cuda.synchronize()
        r = np.full((m.nelem, 4), np.nan)
        dt = np.full(m.nelem, np.nan)
        for k in range(nparts):
            r[gl[k]] = drs[k].cpu().numpy()
            dt[gl[k]] = dts[k].cpu().numpy()
        r1 = np.zeros((m.nelem, 4))
        dt1 = np.zeros(m.nelem)
        one.compute_residual(u, r1, True, dt1)
        results.append((r, dt, r1, dt1))
    grp.close()
    for sp in sps:
        sp.close()
    one.close()
    for r, dt, r1, dt1 in results:
        np.testing.assert_array_equal(r, r1)
        np.testing.assert_array_equal(dt, dt1)


def test_halo_ready_residual_bitwise():
    """FVHIP_RES_HALO_READY (the caller keeps the ghost rows current, as the reference's drivers do with
    VecGhostUpdate): after one group residual has filled every rank's ghost rows, each rank's residual
    with no exchange is bitwise the group's"""
    import torch
    m, _ = get_mesh("naca_c2")
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VENKATAKRISHNAN")
    u = cases.state(m, p, seed=5)
    part = fa.partition_graph(m, 4)
    sps = [fa.FlowFV(m, p, n, partition=part, rank=k) for k in range(4)]
    dus, drs, dts = [], [], []
    for k, sp in enumerate(sps):
        g = np.nonzero(part == k)[0][sp.permutation()]
        x = torch.full((sp.nown + sp.nghost, 4), float("nan"), dtype=torch.float64, device="cuda")
        x[:sp.nown] = torch.tensor(u[g], device="cuda")
        dus.append(x)
        drs.append(torch.zeros((sp.nown, 4), dtype=torch.float64, device="cuda"))
        dts.append(torch.zeros(sp.nown, dtype=torch.float64, device="cuda"))
    torch.cuda.synchronize()  # torch's stream vs the library's (non-blocking) streams
    grp = fa.FlowFVGroup(sps)
    grp.compute_residual_device([x.data_ptr() for x in dus], [x.data_ptr() for x in drs],
                                [x.data_ptr() for x in dts], True, True)
    torch.cuda.synchronize()
    for k, sp in enumerate(sps):
        r2 = torch.zeros_like(drs[k])
        t2 = torch.zeros_like(dts[k])
        torch.cuda.synchronize()
        sp.compute_residual_device(dus[k].data_ptr(), r2.data_ptr(), t2.data_ptr(), True, True, halo_ready=True)
        sp.synchronize()
        assert torch.equal(r2, drs[k]) and torch.equal(t2, dts[k]), k
    grp.close()
    for sp in sps:
        sp.close()
