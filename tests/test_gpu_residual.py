"""GPU parity: FlowFV::compute_residual through the C-ABI vs the CPU oracle (restated reference).

Bar (north_star: residuals match the reference to a stated tolerance, indexing bit-exact):
  * inviscid and constant-viscosity sweeps without WENO: BITWISE equal residual and time steps
    (-ffp-contract=off, ordered per-cell accumulation in reference face order);
  * sweeps that call pow() (Sutherland viscosity pow(T,1.5), WENO pow(x,4)): the device libm and
    glibc may differ in the last ulp, so |dr| <= 1e-12 * max|r| per variable (and dt likewise).
"""
import numpy as np
import pytest

import fvens_amd as fa
import _oracle as orc
import cases

pytestmark = pytest.mark.gpu

_mesh_cache = {}


def get_mesh(key):
    if key not in _mesh_cache:
        if key.endswith(".msh"):
            m = fa.UMesh.read_gmsh(cases.fixture_mesh(key[:-4]))
            om = orc.OracleMesh.read(cases.fixture_mesh(key[:-4]))
        elif key == "naca_small":
            m = fa.UMesh.naca_ogrid(96, 6, 18)
            om = orc.OracleMesh.from_raw(m.raw())
        elif key == "naca_c2":
            m = fa.UMesh.naca_ogrid(512, 64, 192)          # C2 of SURVEY.md 8d: 229,376 cells
            om = orc.OracleMesh.from_raw(m.raw())
        elif key == "naca_c4":                               # the bench's C4 mesh (no oracle mesh)
            m, om = fa.UMesh.naca_ogrid(2048, 256, 864, 20.0, 1e-5, farmap=1), None
        elif key == "naca_c5":                               # BASELINE config 5's 8,054,616-cell hybrid mesh
            from bench import c4_mesh
            m, om = c4_mesh(fa, 1, 2)[0], None
        elif key == "c1":                                    # BASELINE config 1's cylinder
            m = fa.UMesh.cylinder_ogrid(64, 40)
            om = orc.OracleMesh.from_raw(m.raw())
        elif key == "plate_small":
            m = fa.UMesh.flat_plate(48, 32)
            om = orc.OracleMesh.from_raw(m.raw())
        else:
            raise KeyError(key)
        _mesh_cache[key] = (m, om)
    return _mesh_cache[key]


def run_both(meshkey, p, n, seed=7, gettimesteps=True):
    m, om = get_mesh(meshkey)
    u = cases.state(m, p, seed)
    dev = fa.FlowFV(m, p, n)
    r = np.zeros((m.nelem, 4))
    dt = np.zeros(m.nelem)
    dev.compute_residual(u, r, gettimesteps, dt)
    ref = orc.OracleSpatial(om, p, n)
    r0 = np.zeros((m.nelem, 4))
    dt0 = np.zeros(m.nelem)
    ref.compute_residual(u, r0, gettimesteps, dt0)
    dev.close()
    return r, dt, r0, dt0


def assert_close(r, r0, dt, dt0, rtol=1e-12):
    """|dr| <= rtol * max|r| per variable; NaNs must coincide"""
    np.testing.assert_array_equal(np.isnan(r), np.isnan(r0))
    fin = np.isfinite(r0)
    scale = np.where(fin, np.abs(r0), 0).max(axis=0) + 1e-300
    err = np.where(fin, np.abs(r - r0), 0).max(axis=0) / scale
    assert np.all(err <= rtol), f"residual rel err per var {err}"
    if dt0 is not None:
        np.testing.assert_array_equal(np.isnan(dt), np.isnan(dt0))
        f = np.isfinite(dt0)
        assert np.all(np.abs(dt[f] - dt0[f]) <= rtol * np.abs(dt0[f])), "time step mismatch"


FIRST_ORDER_FLUXES = ["LLF", "ROE", "HLL", "HLLC", "AUSM", "AUSMPLUS", "VANLEER"]


@pytest.mark.parametrize("flux", FIRST_ORDER_FLUXES)
@pytest.mark.parametrize("meshkey", ["2dcylinderhybrid.msh", "naca_small"])
def test_first_order_bitwise(flux, meshkey):
    p = cases.physics("cyl" if "cyl" in meshkey else "naca")
    n = cases.numerics(flux, "NONE", "NONE", order2=False)
    r, dt, r0, dt0 = run_both(meshkey, p, n)
    np.testing.assert_array_equal(r, r0)
    np.testing.assert_array_equal(dt, dt0)


SECOND_ORDER = [
    ("ROE", "LEASTSQUARES", "VANALBADA"),
    ("HLLC", "LEASTSQUARES", "VANALBADA"),
    ("LLF", "LEASTSQUARES", "VANALBADA"),
    ("ROE", "GREENGAUSS", "VANALBADA"),
    ("HLLC", "LEASTSQUARES", "NONE"),
    ("ROE", "LEASTSQUARES", "VENKATAKRISHNAN"),
    ("ROE", "GREENGAUSS", "BARTHJESPERSEN"),
    ("AUSM", "LEASTSQUARES", "VANALBADA"),
    ("HLL", "GREENGAUSS", "NONE"),
]


@pytest.mark.parametrize("flux,grad,rec", SECOND_ORDER)
@pytest.mark.parametrize("meshkey", ["2dcylinderhybrid.msh", "naca0012luo.msh", "naca_small"])
def test_second_order_inviscid_bitwise(flux, grad, rec, meshkey):
    p = cases.physics("cyl" if "cyl" in meshkey else "naca")
    n = cases.numerics(flux, grad, rec)
    r, dt, r0, dt0 = run_both(meshkey, p, n)
    np.testing.assert_array_equal(r, r0)
    np.testing.assert_array_equal(dt, dt0)


def test_weno_tolerance():
    p = cases.physics("naca")
    n = cases.numerics("HLLC", "LEASTSQUARES", "WENO", K=4.0)
    r, dt, r0, dt0 = run_both("naca0012luo.msh", p, n)
    assert_close(r, r0, dt, dt0)


@pytest.mark.parametrize("order2", [False, True])
@pytest.mark.parametrize("kind", ["visc", "viscconst"])
def test_viscous_naca(kind, order2):
    p = cases.physics(kind)
    n = cases.numerics("ROE", "LEASTSQUARES" if order2 else "NONE", "NONE", order2=order2)
    r, dt, r0, dt0 = run_both("naca_small", p, n)
    if kind == "viscconst":
        np.testing.assert_array_equal(r, r0)
        np.testing.assert_array_equal(dt, dt0)
    else:
        assert_close(r, r0, dt, dt0)


def test_flat_plate_all_bcs():
    p = cases.physics("plate")
    n = cases.numerics("HLLC", "LEASTSQUARES", "NONE")
    r, dt, r0, dt0 = run_both("plate_small", p, n)
    assert_close(r, r0, dt, dt0)


def test_flat_plate_inviscid_bitwise():
    p = cases.physics("plate_inviscid")
    n = cases.numerics("ROE", "GREENGAUSS", "VANALBADA")
    r, dt, r0, dt0 = run_both("plate_small", p, n)
    np.testing.assert_array_equal(r, r0)
    np.testing.assert_array_equal(dt, dt0)


def test_wall_bcs_isothermal():
    p = cases.physics("wall")
    n = cases.numerics("ROE", "LEASTSQUARES", "NONE")
    r, dt, r0, dt0 = run_both("testperiodic.msh", p, n)
    assert_close(r, r0, dt, dt0)


def test_c2_size_roe_muscl_bitwise():
    """The C2 configuration (229,376-cell hybrid NACA0012 O-grid, Roe + WLS + MUSCL/Van Albada)."""
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    r, dt, r0, dt0 = run_both("naca_c2", p, n)
    np.testing.assert_array_equal(r, r0)
    np.testing.assert_array_equal(dt, dt0)


def test_residual_accumulates_into_r():
    """compute_residual ADDS -r(u) into r (flow_spatial.hpp:73-85)"""
    m, om = get_mesh("naca_small")
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    u = cases.state(m, p, 3)
    base = np.random.default_rng(1).standard_normal((m.nelem, 4))
    dev = fa.FlowFV(m, p, n)
    r = base.copy()
    dev.compute_residual(u, r)
    ref = orc.OracleSpatial(om, p, n)
    r0 = base.copy()
    ref.compute_residual(u, r0)
    np.testing.assert_array_equal(r, r0)


def test_device_path_matches_host_path():
    """Device-resident sweep (internal order, overwrite mode) == host API result"""
    import torch
    m, om = get_mesh("naca_small")
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    u = cases.state(m, p, 5)
    dev = fa.FlowFV(m, p, n)
    r = np.zeros((m.nelem, 4))
    dt = np.zeros(m.nelem)
    dev.compute_residual(u, r, True, dt)
    perm = dev.permutation()
    du = torch.tensor(u[perm], device="cuda")
    dr = torch.empty((m.nelem, 4), dtype=torch.float64, device="cuda")
    ddt = torch.empty(m.nelem, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    dev.compute_residual_device(du.data_ptr(), dr.data_ptr(), ddt.data_ptr(), True, True)
    dev.synchronize()
    r2 = np.empty_like(r)
    r2[perm] = dr.cpu().numpy()
    dt2 = np.empty_like(dt)
    dt2[perm] = ddt.cpu().numpy()
    np.testing.assert_array_equal(r, r2)
    np.testing.assert_array_equal(dt, dt2)


def test_gradients_conserved():
    """FlowFV_base::getGradients (conserved gradients with BC ghost states)"""
    m, om = get_mesh("2dcylinderhybrid.msh")
    p = cases.physics("cyl")
    for grad in ["LEASTSQUARES", "GREENGAUSS"]:
        n = cases.numerics("ROE", grad, "VANALBADA")
        u = cases.state(m, p, 11)
        g = fa.FlowFV(m, p, n).getGradients(u)
        g0 = orc.OracleSpatial(om, p, n).getGradients(u)
        np.testing.assert_array_equal(g, g0)


@pytest.mark.parametrize("flux", FIRST_ORDER_FLUXES)
def test_local_flux_bitwise(flux):
    rng = np.random.default_rng(3)
    nf = 2000
    gas = (1.4, 0.8, 298.0, float("inf"), float("nan"))
    ul = np.empty((nf, 4)); ur = np.empty((nf, 4))
    for u in (ul, ur):
        rho = 1 + 0.3 * rng.random(nf)
        vx = 0.8 * rng.standard_normal(nf); vy = 0.8 * rng.standard_normal(nf)
        pr = 1.0 / (1.4 * 0.64) * (1 + 0.3 * rng.random(nf))
        u[:, 0] = rho; u[:, 1] = rho * vx; u[:, 2] = rho * vy; u[:, 3] = pr / 0.4 + 0.5 * rho * (vx**2 + vy**2)
    th = 2 * np.pi * rng.random(nf)
    nn = np.stack([np.cos(th), np.sin(th)], 1)
    f = fa.local_flux(flux, gas, ul, ur, nn)
    f0 = np.array([orc.flux(flux, gas, ul[i], ur[i], nn[i]) for i in range(nf)])
    np.testing.assert_array_equal(f, f0)


# ------------------------------------------------------------------------------------------------
# fast-math mode (not a reference option): contracted FMAs and approximate division/sqrt in the
# sweep. Bar: |dr| <= 1e-11 * max|r| per variable and |d dt| <= 1e-12 |dt| against the oracle.
# ------------------------------------------------------------------------------------------------
FAST_CASES = [("naca_small", "naca", "ROE", "LEASTSQUARES", "VANALBADA"),
              ("naca_c2", "naca", "ROE", "LEASTSQUARES", "VANALBADA"),
              ("2dcylinderhybrid.msh", "cyl", "HLLC", "GREENGAUSS", "VANALBADA"),
              ("naca_small", "naca", "HLLC", "LEASTSQUARES", "VENKATAKRISHNAN"),
              ("naca_small", "viscconst", "ROE", "LEASTSQUARES", "NONE"),
              ("plate_small", "plate", "HLLC", "LEASTSQUARES", "VANALBADA"),
              ("naca_small", "naca", "LLF", "NONE", "NONE")]


@pytest.mark.parametrize("meshkey,kind,flux,grad,rec", FAST_CASES)
def test_fast_math_within_tolerance(meshkey, kind, flux, grad, rec):
    p = cases.physics(kind)
    n = cases.numerics(flux, grad, rec, order2=grad != "NONE")
    n.fast_math = True
    r, dt, r0, dt0 = run_both(meshkey, p, n)
    assert_close(r, r0, None, None, rtol=1e-11)
    np.testing.assert_allclose(dt, dt0, rtol=1e-12, atol=0)


# ------------------------------------------------------------------------------------------------
# one-launch fused residual (WLS + MUSCL / unlimited linear, inviscid or viscous; Barth-Jespersen /
# Venkatakrishnan inviscid) vs the staged kernels
# (same device arithmetic, Sutherland's T*sqrt(T) included: bitwise)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("flux", ["ROE", "HLLC", "LLF", "AUSMPLUS"])
@pytest.mark.parametrize("rec", ["VANALBADA", "NONE", "VENKATAKRISHNAN", "BARTHJESPERSEN"])
@pytest.mark.parametrize("meshkey,kind", [("naca_small", "naca"), ("2dcylinderhybrid.msh", "cyl"),
                                          ("plate_small", "plate_inviscid"), ("naca_c2", "naca"),
                                          ("naca_small", "visc"), ("naca_small", "viscconst"),
                                          ("plate_small", "plate")])
def test_fused_equals_staged_bitwise(flux, rec, meshkey, kind):
    import torch
    m, _ = get_mesh(meshkey)
    p = cases.physics(kind)
    n = cases.numerics(flux, "LEASTSQUARES", rec)
    u = cases.state(m, p, 5)
    dev = fa.FlowFV(m, p, n)
    perm = dev.permutation()
    du = torch.tensor(u[perm], device="cuda")
    out = []
    for staged in (False, True):
        dr = torch.full((m.nelem, 4), float("nan"), dtype=torch.float64, device="cuda")
        dt = torch.full((m.nelem,), float("nan"), dtype=torch.float64, device="cuda")
        dev.compute_residual_device(du.data_ptr(), dr.data_ptr(), dt.data_ptr(), True, True, staged=staged)
        dev.synchronize()
        out.append((dr.cpu().numpy(), dt.cpu().numpy()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    kt = dev.kernel_times() if False else None
    dev.close()


# ------------------------------------------------------------------------------------------------
# pipelined staged residual (gradient chunks overlapped with sweep groups on a second stream) vs
# the serial staged path: same kernels, so bitwise; viscous configurations take it by default
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("meshkey,kind,flux,rec", [("naca_small", "naca", "ROE", "VANALBADA"),
                                                   ("naca_c2", "naca", "ROE", "VANALBADA"),
                                                   ("naca_small", "visc", "ROE", "NONE"),
                                                   ("naca_small", "viscconst", "HLLC", "VANALBADA"),
                                                   ("plate_small", "plate", "HLLC", "NONE"),
                                                   ("2dcylinderhybrid.msh", "cyl", "LLF", "NONE")])
def test_pipelined_equals_staged_bitwise(meshkey, kind, flux, rec):
    import torch
    m, _ = get_mesh(meshkey)
    p = cases.physics(kind)
    n = cases.numerics(flux, "LEASTSQUARES", rec)
    u = cases.state(m, p, 9)
    dev = fa.FlowFV(m, p, n)
    perm = dev.permutation()
    du = torch.tensor(u[perm], device="cuda")
    out = []
    for mode in ("staged", "pipelined"):
        dr = torch.full((m.nelem, 4), float("nan"), dtype=torch.float64, device="cuda")
        dt = torch.full((m.nelem,), float("nan"), dtype=torch.float64, device="cuda")
        for _ in range(2):      # the second call reuses the streams and events
            dev.compute_residual_device(du.data_ptr(), dr.data_ptr(), dt.data_ptr(), True, True,
                                        staged=mode == "staged", pipelined=mode == "pipelined")
        dev.synchronize()
        out.append((dr.cpu().numpy(), dt.cpu().numpy()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    assert np.all(np.isfinite(out[1][0]))
    dev.close()
