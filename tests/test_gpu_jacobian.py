"""GPU parity of the Jacobian rows through the C-ABI vs the CPU oracle.

Bar:
  * flux Jacobians (LLF, AUSM, Roe, HLL, HLLC) and assembled blocks (diag / lower / upper) for
    inviscid and constant-viscosity configurations: BITWISE equal to the oracle's restatement of
    Spatial::assemble_jacobian (aspatial.cpp:242-340);
  * Sutherland viscosity (device pow vs glibc pow): |dA| <= 1e-12 * max|A| per block entry;
  * matrix-free operator (alinalg.cpp:142-233): the vector norm is a parallel reduction on the device
    (the reference uses PETSc's VecNorm, itself not a sequential sum), so eps/|x| may differ in the
    last ulp, which the finite difference amplifies by ~|x|/eps:  |dy| <= 1e-6 * max|y|;
  * consistency: the assembled first-order Roe Jacobian times x agrees with the matrix-free product
    to finite-difference accuracy (relative 1e-4), and the pseudo-time term / block apply match
    numpy on the same blocks.
"""
import numpy as np
import pytest

import fvens_amd as fa
import _oracle as orc
import cases
from test_gpu_residual import get_mesh

pytestmark = pytest.mark.gpu

JAC_FLUXES = ["LLF", "AUSM", "ROE", "HLL", "HLLC"]


def random_states(nf, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(2):
        rho = 1.0 + 0.5 * rng.uniform(-1, 1, nf)
        mach = np.where(np.arange(nf) % 4 == 0, 2.5, 1.0)
        vx = mach * rng.uniform(-1, 1, nf)
        vy = mach * rng.uniform(-1, 1, nf)
        vy[::7] = 0.0
        vx[::11] = 0.0
        p = (1.0 + 0.4 * rng.uniform(-1, 1, nf)) / (1.4 * 0.64)
        out.append(np.stack([rho, rho * vx, rho * vy, p / 0.4 + 0.5 * rho * (vx * vx + vy * vy)], 1))
    ul, ur = out
    ur[::13] = ul[::13]
    th = np.pi * rng.uniform(-1, 1, nf)
    n = np.stack([np.cos(th), np.sin(th)], 1)
    return np.ascontiguousarray(ul), np.ascontiguousarray(ur), np.ascontiguousarray(n)


@pytest.mark.parametrize("flux", JAC_FLUXES)
def test_local_flux_jacobian_bitwise(flux):
    gas = (1.4, 0.8, 288.15, 5000.0, 0.72)
    ul, ur, n = random_states(1500, 3)
    dl, dr = fa.local_flux_jacobian(flux, gas, ul, ur, n)
    for f in range(ul.shape[0]):
        a, b = orc.flux_jacobian(flux, gas, ul[f], ur[f], n[f])
        np.testing.assert_array_equal(dl[f], a, err_msg=f"face {f}")
        np.testing.assert_array_equal(dr[f], b, err_msg=f"face {f}")


def test_local_flux_jacobian_unsupported():
    gas = (1.4, 0.8, 288.15, 5000.0, 0.72)
    ul, ur, n = random_states(4, 3)
    for flux in ("VANLEER", "AUSMPLUS"):
        with pytest.raises(RuntimeError, match="Not implemented"):
            fa.local_flux_jacobian(flux, gas, ul, ur, n)


def assemble_both(meshkey, p, n, seed=5):
    m, om = get_mesh(meshkey)
    u = cases.state(m, p, seed)
    dev = fa.FlowFV(m, p, n)
    d, lo, up = dev.assemble_jacobian(u)
    ref = orc.OracleSpatial(om, p, n)
    d0, lo0, up0 = ref.jacobian(u)
    dev.close()
    return (d, lo, up), (d0, lo0, up0)


@pytest.mark.parametrize("flux", JAC_FLUXES)
@pytest.mark.parametrize("meshkey,kind", [("2dcylinderhybrid.msh", "cyl"), ("naca_small", "naca"),
                                          ("plate_small", "plate_inviscid")])
def test_assemble_inviscid_bitwise(flux, meshkey, kind):
    p = cases.physics(kind)
    n = cases.numerics("ROE", jac=flux)
    got, ref = assemble_both(meshkey, p, n)
    for a, b, nm in zip(got, ref, ("diag", "lower", "upper")):
        np.testing.assert_array_equal(a, b, err_msg=nm)


@pytest.mark.parametrize("flux", ["ROE", "HLLC", "LLF"])
@pytest.mark.parametrize("meshkey,kind", [("naca_small", "viscconst"), ("2dcylinder1.msh", "wall")])
def test_assemble_viscous_const_bitwise(flux, meshkey, kind):
    p = cases.physics(kind)
    p.const_visc = True
    n = cases.numerics("ROE", jac=flux)
    got, ref = assemble_both(meshkey, p, n)
    for a, b, nm in zip(got, ref, ("diag", "lower", "upper")):
        np.testing.assert_array_equal(a, b, err_msg=nm)


@pytest.mark.parametrize("flux", ["ROE", "HLL"])
@pytest.mark.parametrize("meshkey,kind", [("naca_small", "visc"), ("plate_small", "plate")])
def test_assemble_sutherland(flux, meshkey, kind):
    p = cases.physics(kind)
    n = cases.numerics("ROE", jac=flux)
    got, ref = assemble_both(meshkey, p, n)
    for a, b, nm in zip(got, ref, ("diag", "lower", "upper")):
        scale = np.abs(b).max(axis=0) + 1e-300
        err = (np.abs(a - b).max(axis=0) / scale).max()
        assert err <= 1e-12, f"{nm}: rel err {err}"


def test_assemble_adds_into_caller_blocks():
    m, _ = get_mesh("naca_small")
    p = cases.physics("naca")
    n = cases.numerics("ROE")
    u = cases.state(m, p, 9)
    dev = fa.FlowFV(m, p, n)
    d1, l1, u1 = dev.assemble_jacobian(u)
    d2, l2, u2 = dev.assemble_jacobian(u, d1.copy(), l1.copy(), u1.copy())
    np.testing.assert_array_equal(d2, 2 * d1)
    np.testing.assert_array_equal(l2, 2 * l1)
    np.testing.assert_array_equal(u2, 2 * u1)
    dev.close()


def test_subsonic_inflow_has_no_jacobian():
    m, _ = get_mesh("plate_small")
    p = cases.physics("plate_inviscid")
    p.bcconf[3] = fa.FlowBCConfig("subsonic_inflow", 5, [1.0 / (1.4 * 0.04) * 1.02, 1.01])
    dev = fa.FlowFV(m, p, cases.numerics("ROE"))
    with pytest.raises(RuntimeError, match="Not implemented"):
        dev.assemble_jacobian(cases.state(m, p, 1))
    dev.close()


def test_bsr_pattern_and_values():
    m, om = get_mesh("2dcylinderhybrid.msh")
    p = cases.physics("cyl")
    n = cases.numerics("HLLC")
    u = cases.state(m, p, 2)
    dev = fa.FlowFV(m, p, n)
    rowptr, colind = dev.jacobian_pattern()
    vals = dev.assemble_jacobian_bsr(u, rowptr, colind)
    d0, lo0, up0 = orc.OracleSpatial(om, p, n).jacobian(u)
    L = m.intfac[m.nbface:, 0]
    R = m.intfac[m.nbface:, 1]
    N = m.nelem
    # dense reference from the oracle's face blocks
    for c in range(N):
        cols = colind[rowptr[c]:rowptr[c + 1]]
        assert np.all(np.diff(cols) > 0)
        assert c in cols
    A = {}
    for c in range(N):
        A[(c, c)] = d0[c]
    for fi in range(len(L)):
        A[(R[fi], L[fi])] = lo0[fi]
        A[(L[fi], R[fi])] = up0[fi]
    assert rowptr[-1] == len(A)
    for c in range(N):
        for k in range(rowptr[c], rowptr[c + 1]):
            np.testing.assert_array_equal(vals[k], A[(c, colind[k])])
    dev.close()


def _torch():
    import torch
    return torch


def test_pseudo_time_and_block_apply_device():
    torch = _torch()
    m, _ = get_mesh("naca_small")
    p = cases.physics("naca")
    n = cases.numerics("ROE", order2=False)
    u = cases.state(m, p, 4)
    dev = fa.FlowFV(m, p, n)
    perm = dev.permutation()
    N, Fi = m.nelem, m.naface - m.nbface
    du = torch.tensor(u[perm], device="cuda")
    dd = torch.zeros((N, 16), dtype=torch.float64, device="cuda")
    dl = torch.zeros((Fi, 16), dtype=torch.float64, device="cuda")
    dup = torch.zeros((Fi, 16), dtype=torch.float64, device="cuda")
    dev.assemble_jacobian_device(du.data_ptr(), dd.data_ptr(), dl.data_ptr(), dup.data_ptr())
    dev.synchronize()
    # device blocks equal the host-path blocks
    d_h, l_h, u_h = dev.assemble_jacobian(u)
    np.testing.assert_array_equal(dd.cpu().numpy().reshape(N, 4, 4), d_h[perm])
    np.testing.assert_array_equal(dl.cpu().numpy().reshape(Fi, 4, 4), l_h)
    np.testing.assert_array_equal(dup.cpu().numpy().reshape(Fi, 4, 4), u_h)
    # pseudo-time term
    r = np.zeros((N, 4))
    dtm = np.zeros(N)
    dev.compute_residual(u, r, True, dtm)
    cfl = 7.5
    ddtm = torch.tensor(dtm[perm], device="cuda")
    dev.add_pseudo_time_term_device(cfl, ddtm.data_ptr(), dd.data_ptr())
    dev.synchronize()
    area = m.area[:N]
    mdt = area / (cfl * dtm)
    np.testing.assert_array_equal(ddtm.cpu().numpy(), mdt[perm])
    dref = d_h + mdt[:, None, None] * np.eye(4)[None]
    np.testing.assert_array_equal(dd.cpu().numpy().reshape(N, 4, 4), dref[perm])
    # block apply vs numpy
    x = np.random.default_rng(0).standard_normal((N, 4))
    dx = torch.tensor(x[perm], device="cuda")
    dy = torch.zeros_like(dx)
    dev.block_apply_device(dd.data_ptr(), dl.data_ptr(), dup.data_ptr(), dx.data_ptr(), dy.data_ptr())
    dev.synchronize()
    L = m.intfac[m.nbface:, 0]
    R = m.intfac[m.nbface:, 1]
    y = np.einsum("cij,cj->ci", dref, x)
    np.add.at(y, R, np.einsum("fij,fj->fi", l_h, x[L]))
    np.add.at(y, L, np.einsum("fij,fj->fi", u_h, x[R]))
    got = np.empty_like(y)
    got[perm] = dy.cpu().numpy()
    np.testing.assert_allclose(got, y, rtol=1e-12, atol=1e-12 * np.abs(y).max())
    dev.close()


@pytest.mark.parametrize("meshkey,kind,order2", [("2dcylinderhybrid.msh", "cyl", False),
                                                 ("naca_small", "naca", True),
                                                 ("naca_small", "viscconst", True)])
def test_matfree_vs_oracle(meshkey, kind, order2):
    m, om = get_mesh(meshkey)
    p = cases.physics(kind)
    n = cases.numerics("ROE", order2=order2)
    u = cases.state(m, p, 6)
    N = m.nelem
    ref = orc.OracleSpatial(om, p, n)
    res = np.zeros((N, 4))
    dtm = np.zeros(N)
    ref.compute_residual(u, res, True, dtm)
    mdt = m.area[:N] / (5.0 * dtm)
    x = np.random.default_rng(1).standard_normal((N, 4))
    y0 = ref.matfree(u, res, mdt, 1e-7, x)
    dev = fa.FlowFV(m, p, n)
    dev.matfree_set_state(u, res, mdt)
    y = dev.matfree_apply(x)
    err = np.abs(y - y0).max() / np.abs(y0).max()
    assert err <= 1e-6, err
    dev.close()


def test_jacobian_matches_matfree_first_order():
    """Assembled analytic first-order Roe Jacobian (the reference's exact linearisation) vs the
    finite-difference operator on the same state; no pseudo-time term."""
    torch = _torch()
    m, _ = get_mesh("2dcylinderhybrid.msh")
    p = cases.physics("cyl")
    n = cases.numerics("ROE", "NONE", "NONE", order2=False)
    u = cases.state(m, p, 8)
    dev = fa.FlowFV(m, p, n)
    perm = dev.permutation()
    N, Fi = m.nelem, m.naface - m.nbface
    du = torch.tensor(u[perm], device="cuda")
    dd = torch.zeros((N, 16), dtype=torch.float64, device="cuda")
    dl = torch.zeros((Fi, 16), dtype=torch.float64, device="cuda")
    dup = torch.zeros((Fi, 16), dtype=torch.float64, device="cuda")
    dev.assemble_jacobian_device(du.data_ptr(), dd.data_ptr(), dl.data_ptr(), dup.data_ptr())
    dr = torch.zeros((N, 4), dtype=torch.float64, device="cuda")
    dev.compute_residual_device(du.data_ptr(), dr.data_ptr())
    mdt = torch.zeros(N, dtype=torch.float64, device="cuda")
    dev.matfree_set_state_device(du.data_ptr(), dr.data_ptr(), mdt.data_ptr())
    dev.matfree_set_eps(1e-6)
    x = torch.tensor(np.random.default_rng(2).standard_normal((N, 4)), device="cuda")
    y1 = torch.zeros_like(x)
    y2 = torch.zeros_like(x)
    dev.block_apply_device(dd.data_ptr(), dl.data_ptr(), dup.data_ptr(), x.data_ptr(), y1.data_ptr())
    dev.matfree_apply_device(x.data_ptr(), y2.data_ptr())
    dev.synchronize()
    a, b = y1.cpu().numpy(), y2.cpu().numpy()
    # J = d(-r)/du with -r as stored: assembled A = -dR/du convention of the reference
    rel = np.abs(a - b).max() / np.abs(a).max()
    assert rel < 1e-4, rel
    dev.close()
