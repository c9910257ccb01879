"""Edge cases on the device: degenerate and ragged meshes (a single cell with only boundary faces, one
row of cells, no interior faces), compared with the oracle bit for bit -- including where the
reference's arithmetic itself yields NaN (a least-squares system with collinear neighbours is
singular; the positions of the NaNs must coincide).
"""
import numpy as np
import pytest

import fvens_amd as fa
import _oracle as orc
import cases

pytestmark = pytest.mark.gpu

MESHES = [(1, 1), (2, 1), (1, 3), (3, 2)]
SCHEMES = [("LLF", "NONE", "NONE", False), ("ROE", "LEASTSQUARES", "VANALBADA", True),
           ("HLLC", "GREENGAUSS", "VENKATAKRISHNAN", True)]


@pytest.mark.parametrize("nx,ny", MESHES)
@pytest.mark.parametrize("flux,grad,rec,o2", SCHEMES)
def test_tiny_mesh_residual_bitwise(nx, ny, flux, grad, rec, o2):
    m = fa.UMesh.flat_plate(nx, ny)
    om = orc.OracleMesh.from_raw(m.raw())
    p = cases.physics("plate_inviscid")
    n = cases.numerics(flux, grad, rec, order2=o2)
    u = cases.state(m, p, 3)
    dev = fa.FlowFV(m, p, n)
    r = np.zeros((m.nelem, 4))
    dt = np.zeros(m.nelem)
    dev.compute_residual(u, r, True, dt)
    dev.close()
    ref = orc.OracleSpatial(om, p, n)
    r0 = np.zeros((m.nelem, 4))
    dt0 = np.zeros(m.nelem)
    ref.compute_residual(u, r0, True, dt0)
    np.testing.assert_array_equal(r, r0)
    np.testing.assert_array_equal(dt, dt0)


@pytest.mark.parametrize("nx,ny", [(1, 1), (2, 1)])
def test_tiny_mesh_jacobian_bitwise(nx, ny):
    """no or one interior face: the face-block arrays are empty or a single block"""
    m = fa.UMesh.flat_plate(nx, ny)
    om = orc.OracleMesh.from_raw(m.raw())
    p = cases.physics("plate_inviscid")
    n = cases.numerics("ROE", "NONE", "NONE", order2=False)
    u = cases.state(m, p, 5)
    dev = fa.FlowFV(m, p, n)
    D, lo, up = dev.assemble_jacobian(u)
    dev.close()
    D0, lo0, up0 = orc.OracleSpatial(om, p, n).jacobian(u)
    np.testing.assert_array_equal(D, D0)
    np.testing.assert_array_equal(lo, lo0)
    np.testing.assert_array_equal(up, up0)


def _divsqrt(a, b):
    import fvens_amd._ffi as ffi
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    out = np.zeros((len(a), 4))
    fa.check(ffi.lib().fvhip_divsqrt_probe(len(a), fa.dptr(a), fa.dptr(b), fa.dptr(out)))
    return out


def test_div_sqrt_rn_domain():
    """gasdyn.hpp's div_rn / sqrt_rn are the compiler's IEEE sequences without their range scaling and
    special-value fix-ups. Their bitwise claim, checked against the device's own IEEE operations and
    numpy, holds on a stated domain:
      * div_rn: bitwise on 2e5 random pairs with |a|, |b| and |a/b| in [2^-1000, 2^1000] (mantissas at
        both ends of the binade included);
      * sqrt_rn: bitwise for x in [2^-766, 2^1000]; below 2^-767 the IEEE sequence scales x by 2^256
        first and sqrt_rn, which does not, can be off by one ulp (found by this test: one of 2e5
        draws at x ~ 1e-297);
      * outside: overflowing quotients give NaN instead of inf.
    The sweep's operands lie far inside (densities, pressures, sound speeds, eps-shifted limiter sums,
    squared centre distances of 1e-5-spaced cells: 1e-12 .. 1e12)."""
    rng = np.random.default_rng(7)
    n = 200000
    ea = rng.integers(-1000, 1000, n)
    eb = rng.integers(-1000, 1000, n)
    keep = np.abs(ea - eb) < 998
    ea, eb = ea[keep], eb[keep]
    ma = rng.uniform(1.0, 2.0, len(ea))
    mb = rng.uniform(1.0, 2.0, len(eb))
    ma[:500] = np.nextafter(2.0, 1.0)           # mantissas at the ends of the binade
    mb[500:1000] = np.nextafter(1.0, 2.0)
    a = np.ldexp(ma, ea) * np.where(rng.random(len(ea)) < 0.5, -1.0, 1.0)
    b = np.ldexp(mb, eb) * np.where(rng.random(len(eb)) < 0.5, -1.0, 1.0)
    out = _divsqrt(a, b)
    np.testing.assert_array_equal(out[:, 0], out[:, 1])          # div_rn == device IEEE division
    np.testing.assert_array_equal(out[:, 1], a / b)              # == host IEEE division
    es = rng.integers(-766, 1000, n)
    x = np.ldexp(rng.uniform(1.0, 2.0, n), es)
    x[:500] = np.ldexp(np.nextafter(2.0, 1.0), es[:500])
    out_s = _divsqrt(x, np.ones(n))
    np.testing.assert_array_equal(out_s[:, 2], out_s[:, 3])      # sqrt_rn == device IEEE sqrt
    np.testing.assert_array_equal(out_s[:, 3], np.sqrt(x))
    # outside the domain: tiny square-root operands, subnormal and overflowing quotients
    xt = np.ldexp(rng.uniform(1.0, 2.0, n), rng.integers(-1020, -767, n))
    t = _divsqrt(xt, np.ones(n))
    off = np.count_nonzero(t[:, 2] != t[:, 3])
    ulp = np.abs(t[:, 2] - t[:, 3]) / np.spacing(t[:, 3])
    print(f"sqrt_rn below 2^-767: {off} of {n} differ from IEEE sqrt, at most {ulp.max():.0f} ulp")
    assert ulp.max() <= 1.0
    a_e = np.array([1e-300, 1.0, 1.7e308, 1.0])
    b_e = np.array([1e10, 1e308 * 1.5, 0.5, 1e-310])
    e = _divsqrt(a_e, b_e)
    print("edge operands: div_rn", e[:, 0], "IEEE", e[:, 1])
    assert np.isnan(e[2, 0]) and np.isinf(e[2, 1])               # overflow: NaN instead of inf


def test_null_device_pointers_refused_handle_survives():
    """a null device array is refused by name before any launch (it would fault the GPU), and the
    handle still computes the oracle's residual afterwards"""
    import torch
    m = fa.UMesh.flat_plate(8, 4)
    p = cases.physics("plate_inviscid")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    dev = fa.FlowFV(m, p, n)
    u = cases.state(m, p, 3)
    du = torch.tensor(u[dev.permutation()], device="cuda")
    dr = torch.zeros((m.nelem, 4), dtype=torch.float64, device="cuda")
    dt = torch.zeros(m.nelem, dtype=torch.float64, device="cuda")
    for args, what in [((0, dr.data_ptr(), dt.data_ptr(), True), "null u"),
                       ((du.data_ptr(), 0, dt.data_ptr(), True), "null residual"),
                       ((du.data_ptr(), dr.data_ptr(), 0, True), "null dtm")]:
        with pytest.raises(RuntimeError, match=what):
            dev.compute_residual_device(*args)
    with pytest.raises(RuntimeError, match="null u"):
        fa.FlowFVGroup([dev]).compute_residual_device([0], [dr.data_ptr()])
    dev.compute_residual_device(du.data_ptr(), dr.data_ptr(), dt.data_ptr(), True)
    dev.synchronize()
    inv = np.empty_like(dev.permutation())
    inv[dev.permutation()] = np.arange(m.nelem)
    r = dr.cpu().numpy()[inv]
    dev.close()
    ref = orc.OracleSpatial(orc.OracleMesh.from_raw(m.raw()), p, n)
    r0 = np.zeros((m.nelem, 4))
    ref.compute_residual(u, r0, True, np.zeros(m.nelem))
    np.testing.assert_array_equal(r, r0)
