"""The unsteady explicit driver on the device: TVDRKSolver::solve (aodesolver.cpp:669-758), the
reference's remaining caller of compute_residual (casesolvers.cpp:435).

Restated as written: ustage = u once before the loop; every stage's residual at the step's start
state u (the reference passes uvec to compute_residual, :719); dtmin = min over cells of the first
stage's local time steps; ustage = c0 u + c1 ustage - c2 dtmin cfl / area r; u = ustage; time +=
dtmin cfl while time <= finaltime - 1e-12. Checked bit for bit against a host restatement of that loop
around the oracle's residual (numpy's float64 operations in the reference's order), for temporal
orders 1-3, with the final-time stop, and on a 3-rank in-process partition against one GPU.
"""
import numpy as np
import pytest

import fvens_amd as fa
import _oracle as orc
import cases
from test_gpu_residual import get_mesh

pytestmark = pytest.mark.gpu

COEF = {1: [(1.0, 0.0, 1.0)],
        2: [(1.0, 0.0, 1.0), (0.5, 0.5, 0.5)],
        3: [(1.0, 0.0, 1.0), (0.75, 0.25, 0.25), (0.3333333333333333, 0.6666666666666667, 0.6666666666666667)]}


def host_tvdrk(m, om, p, n, u0, order, cfl, finaltime, maxsteps):
    ref = orc.OracleSpatial(om, p, n)
    N = m.nelem
    area = m.area[:N]
    u = u0.copy()
    us = u0.copy()
    t, step = 0.0, 0
    while t <= finaltime - 1e-12 and step < maxsteps:
        r = np.zeros((N, 4))
        dtm = np.zeros(N)
        ref.compute_residual(u, r, True, dtm)
        dtmin = dtm.min()
        for c0, c1, c2 in COEF[order]:
            us = c0 * u + c1 * us - c2 * dtmin * cfl / area[:, None] * r
        u = us.copy()
        step += 1
        t += dtmin * cfl
    return u, step, t


def _dev(u, perm):
    import torch
    return torch.tensor(np.ascontiguousarray(u[perm]), device="cuda")


@pytest.mark.parametrize("order", [1, 2, 3])
def test_tvdrk_bitwise_vs_host(order):
    m, om = get_mesh("naca_small")
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    u0 = cases.state(m, p, 5)
    cfl = 0.4
    u_ref, steps_ref, t_ref = host_tvdrk(m, om, p, n, u0, order, cfl, 1e9, 6)
    dev = fa.FlowFV(m, p, n)
    perm = dev.permutation()
    du = _dev(u0, perm)
    steps, t = dev.tvdrk_device(du.data_ptr(), order, cfl, 1e9, 6)
    u = np.empty_like(u0)
    u[perm] = du.cpu().numpy()
    dev.close()
    assert steps == steps_ref == 6
    assert t == t_ref
    np.testing.assert_array_equal(u, u_ref)


def test_tvdrk_final_time():
    """the loop stops at the reference's criterion (time <= finaltime - 1e-12), not at maxsteps"""
    m, om = get_mesh("naca_small")
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    u0 = cases.state(m, p, 6)
    # final time a little over three steps
    _, _, t3 = host_tvdrk(m, om, p, n, u0, 2, 0.4, 1e9, 3)
    u_ref, steps_ref, t_ref = host_tvdrk(m, om, p, n, u0, 2, 0.4, t3 * 1.001, 100)
    dev = fa.FlowFV(m, p, n)
    perm = dev.permutation()
    du = _dev(u0, perm)
    steps, t = dev.tvdrk_device(du.data_ptr(), 2, 0.4, t3 * 1.001, 100)
    u = np.empty_like(u0)
    u[perm] = du.cpu().numpy()
    dev.close()
    assert steps == steps_ref and steps < 100 and t == t_ref and t > t3 * 1.001 - 1e-12
    np.testing.assert_array_equal(u, u_ref)
    with pytest.raises(RuntimeError):
        fa.FlowFV(m, p, n).tvdrk_device(du.data_ptr(), 4, 0.4, 1.0, 10)


def test_tvdrk_partitioned_bitwise():
    """3 ranks in one process: the global dtmin and the one-GPU residuals, so the same bits"""
    import torch
    m, _ = get_mesh("naca_small")
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    u0 = cases.state(m, p, 7)
    one = fa.FlowFV(m, p, n)
    perm = one.permutation()
    du = _dev(u0, perm)
    s1, t1 = one.tvdrk_device(du.data_ptr(), 3, 0.4, 1e9, 4)
    u1 = np.empty_like(u0)
    u1[perm] = du.cpu().numpy()
    one.close()
    part = fa.partition_graph(m, 3, weights="cost")
    sps = [fa.FlowFV(m, p, n, partition=part, rank=k) for k in range(3)]
    dus, glob = [], []
    for k, sp in enumerate(sps):
        g = np.nonzero(part == k)[0][sp.permutation()]
        glob.append(g)
        d = torch.full((sp.nown + sp.nghost, 4), float("nan"), dtype=torch.float64, device="cuda")
        d[:sp.nown] = torch.tensor(u0[g], device="cuda")
        dus.append(d)
    torch.cuda.synchronize()  # torch's stream vs the library's (non-blocking) streams
    grp = fa.FlowFVGroup(sps)
    s, t = grp.tvdrk_device([d.data_ptr() for d in dus], 3, 0.4, 1e9, 4)
    u = np.full_like(u0, np.nan)
    for k, sp in enumerate(sps):
        u[glob[k]] = dus[k][:sp.nown].cpu().numpy()
    grp.close()
    for sp in sps:
        sp.close()
    assert s == s1 == 4 and t == t1
    np.testing.assert_array_equal(u, u1)


def test_tvdrk_nan_in_some_cells_diverges():
    """a NaN state in a few cells makes their time steps NaN: the reduction carries it (fmin would skip
    it and keep stepping), so the reference's 'dtmin is Nan or inf' error fires (aodesolver.cpp:730-731);
    on a 3-rank partition too, with the NaN on one rank only"""
    import torch
    m, _ = get_mesh("naca_small")
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    u0 = cases.state(m, p, 8)
    bad = [m.nelem // 3]
    u0[bad, 0] = np.nan
    one = fa.FlowFV(m, p, n)
    du = _dev(u0, one.permutation())
    with pytest.raises(RuntimeError, match="dtmin is Nan or inf"):
        one.tvdrk_device(du.data_ptr(), 3, 0.4, 1e9, 4)
    one.close()
    part = fa.partition_graph(m, 3, weights="cost")
    sps = [fa.FlowFV(m, p, n, partition=part, rank=k) for k in range(3)]
    dus = []
    for k, sp in enumerate(sps):
        g = np.nonzero(part == k)[0][sp.permutation()]
        d = torch.zeros((sp.nown + sp.nghost, 4), dtype=torch.float64, device="cuda")
        d[:sp.nown] = torch.tensor(u0[g], device="cuda")
        dus.append(d)
    torch.cuda.synchronize()  # torch's stream vs the library's (non-blocking) streams
    grp = fa.FlowFVGroup(sps)
    with pytest.raises(RuntimeError, match="dtmin is Nan or inf"):
        grp.tvdrk_device([d.data_ptr() for d in dus], 3, 0.4, 1e9, 4)
    # the group entry points check their per-rank arrays before indexing them
    import ctypes
    import fvens_amd._ffi as ffi
    arr = (ctypes.c_void_p * 3)(*[d.data_ptr() for d in dus])
    nul = (ctypes.c_void_p * 3)(dus[0].data_ptr(), None, dus[2].data_ptr())
    assert ffi.lib().fvhip_group_matfree_set_state_device(grp._g, arr, nul, arr) != 0
    assert ffi.lib().fvhip_last_error().decode() == "null residual"
    assert ffi.lib().fvhip_group_matfree_set_state_device(grp._g, None, arr, arr) != 0
    assert ffi.lib().fvhip_last_error().decode() == "null u"
    grp.close()
    for sp in sps:
        sp.close()
