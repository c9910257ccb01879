"""Host logic of tools/visc_converge.py (no GPU): the mirror map behind the full-size solve's symmetry projection
(--symmetrize) and the nearest-centre carry-over of mesh sequencing, on small members of the hybrid C5 family."""
import os
import sys

import numpy as np

import fvens_amd as fa

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from visc_converge import carry_over, mirror_map   # noqa: E402
from bench import c4_mesh                            # noqa: E402


def test_mirror_map_is_a_fixed_point_free_involution():
    m, dims = c4_mesh(fa, 16, 2)
    assert dims["topology"] == "hybrid"
    rc = np.asarray(m.rc[:m.nelem])
    mir = mirror_map(rc)
    assert np.array_equal(mir[mir], np.arange(m.nelem)) and not np.any(mir == np.arange(m.nelem))
    assert np.abs(rc[mir] * [1.0, -1.0] - rc).max() <= 1e-12 * np.abs(rc).max()
    area = np.asarray(m.area[:m.nelem])
    assert np.abs(area[mir] - area).max() <= 1e-12 * area.max()
    # the projection (u + S u)/2 is exactly mirror-symmetric
    u = np.random.default_rng(1).standard_normal((m.nelem, 4))
    sgn = np.array([1.0, 1.0, -1.0, 1.0])
    p = 0.5 * (u + u[mir] * sgn)
    assert np.array_equal(p, p[mir] * sgn)


def test_mirror_map_refuses_an_asymmetric_mesh():
    m = fa.UMesh.naca_ogrid(64, 8, 8, 20.0, 1e-4)
    rc = np.asarray(m.rc[:m.nelem]) + np.array([0.0, 1e-3])       # shifted off the chord line
    try:
        mirror_map(rc)
    except AssertionError:
        return
    raise AssertionError("an asymmetric set of centres was accepted")


def test_carry_over_between_members():
    mc, _ = c4_mesh(fa, 16, 2)
    mf, _ = c4_mesh(fa, 8, 2)
    rcc, rcf = np.asarray(mc.rc[:mc.nelem]), np.asarray(mf.rc[:mf.nelem])
    u = np.column_stack([rcc[:, 0], rcc[:, 1], np.hypot(rcc[:, 0], rcc[:, 1]), np.ones(mc.nelem)])
    uf = carry_over(rcc, u, rcf)
    assert uf.shape == (mf.nelem, 4)
    # every fine cell takes a coarse cell's state, the one whose centre is nearest
    d = np.hypot(uf[:, 0] - rcf[:, 0], uf[:, 1] - rcf[:, 1])
    j = np.random.default_rng(0).integers(0, mf.nelem, 200)
    best = np.array([np.hypot(*(rcc - rcf[i]).T).min() for i in j])
    np.testing.assert_allclose(d[j], best, rtol=0, atol=1e-15)
