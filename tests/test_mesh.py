"""The native mesh builder reproduces the reference's face-indexing contract bit for bit
(mesh.cpp:55-82, 290-365, 425-762; aspatial.cpp:50-119): checked against the oracle's literal
restatement on the reference's own test meshes and on every synthetic generator."""
import numpy as np
import pytest

import fvens_amd as fa
import _oracle as orc
import cases

FIXTURES = ["testperiodic", "2dcylinderhybrid", "testhybrid", "squareunsquad0", "2dcylinder0",
            "2dcylinder1", "2dcylinder2", "naca0012luo"]
ARRAYS = ["intfac", "btags", "facemetric", "area", "rc", "gr", "rcbp"]


def compare(m, om):
    assert (m.nelem, m.naface, m.nbface) == (om.nelem, om.naface, om.nbface)
    for name in ARRAYS:
        a = getattr(m, name)
        if name == "rc":
            a = a[:m.nelem]
        b = om.get(name)
        assert a.shape == b.shape, name
        assert np.array_equal(a, b), name
    # esuel/elemface entries beyond a cell's face count are unspecified in the reference
    mask = np.arange(m.maxnfael)[None, :] < m.nnode[:, None]
    assert np.array_equal(m.esuel[mask], om.get("esuel")[mask])
    assert np.array_equal(m.elemface[mask], om.get("elemface")[mask])


@pytest.mark.parametrize("name", FIXTURES)
def test_gmsh_fixture_indexing(name):
    p = cases.fixture_mesh(name)
    compare(fa.UMesh.read_gmsh(p), orc.OracleMesh.read(p))


@pytest.mark.parametrize("gen", [
    lambda: fa.UMesh.naca_ogrid(64, 4, 12),
    lambda: fa.UMesh.naca_ogrid(200, 10, 30, 15.0, 1e-3),
    lambda: fa.UMesh.naca_ogrid(256, 16, 54, 20.0, 1e-5, farmap=3),
    lambda: fa.UMesh.naca_cgrid(96, 16, 8, 24, 20.0, 1e-5),
    lambda: fa.UMesh.naca_cgrid(96, 16, 62, 0, 20.0, 1e-5),
    lambda: fa.UMesh.cylinder_ogrid(48, 12),
    lambda: fa.UMesh.flat_plate(40, 24),
])
def test_generated_mesh_indexing(gen):
    m = gen()
    compare(m, orc.OracleMesh.from_raw(m.raw()))
    assert (m.area > 0).all()


def test_face_structure_contract():
    """Face order: physical boundary [0,nb) with R = N+i; interior faces with L<R; normals point L->R
    (mesh.cpp:680-733, 354-359); each face appears in elemface of both neighbours."""
    m = fa.UMesh.read_gmsh(cases.fixture_mesh("2dcylinderhybrid"))
    N, nb = m.nelem, m.nbface
    assert np.array_equal(m.intfac[:nb, 1], N + np.arange(nb))
    assert (m.intfac[nb:, 0] < m.intfac[nb:, 1]).all()
    # unit normals, positive lengths
    assert np.allclose(np.hypot(m.facemetric[:, 0], m.facemetric[:, 1]), 1.0)
    assert (m.facemetric[:, 2] > 0).all()
    # normal points from L centre towards R centre (or outwards at the boundary)
    d = m.rc[m.intfac[nb:, 1]] - m.rc[m.intfac[nb:, 0]]
    assert ((d * m.facemetric[nb:, :2]).sum(1) > 0).all()
    dout = m.gr[:nb] - m.rc[m.intfac[:nb, 0]]
    assert ((dout * m.facemetric[:nb, :2]).sum(1) > 0).all()
    # closed cells: sum of n*len over faces of each cell = 0
    acc = np.zeros((N, 2))
    nl = m.facemetric[:, :2] * m.facemetric[:, 2:3]
    np.add.at(acc, m.intfac[:, 0], nl)
    np.add.at(acc, m.intfac[nb:, 1], -nl[nb:])
    assert np.abs(acc).max() < 1e-12


def test_testhybrid_counts():
    """tests/common-input/testhybrid.msh: 12 tris + 6 quads; the partition golden files list the
    same 18 global cells (testhybrid-distb.dat)"""
    m = fa.UMesh.read_gmsh(cases.fixture_mesh("testhybrid"))
    assert m.nelem == 18 and (m.nnode == 3).sum() == 12 and (m.nnode == 4).sum() == 6


def test_c1_cylinder_size():
    """C1 of SURVEY.md 8(d): Ntheta=64 x Nr=40 triangle-split O-grid, 5120 cells, 7744 faces"""
    m = fa.UMesh.cylinder_ogrid(64, 40)
    assert (m.nelem, m.naface) == (5120, 7744)


def test_c2_naca_size():
    """C2: NACA0012 O-grid Ntheta=512, 64 quad + 192 triangle layers: 229,376 cells, 360,960 faces"""
    m = fa.UMesh.naca_ogrid(512, 64, 192)
    assert (m.nelem, m.naface) == (229376, 360960)


def _quad_skew(m):
    """largest |corner angle - 90 degrees| of each quadrangle"""
    q = np.where(m.nnode == 4)[0]
    P = m.coords[m.inpoel[q, :4]]
    dev = np.zeros(len(q))
    for i in range(4):
        a, b = P[:, i - 1] - P[:, i], P[:, (i + 1) % 4] - P[:, i]
        c = (a * b).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(b, axis=1)
        dev = np.maximum(dev, np.abs(np.degrees(np.arccos(np.clip(c, -1, 1))) - 90.0))
    return q, dev


def test_naca_wall_normal_layers():
    """generateNacaOgrid farmap bit 2 (the C5 family): the layers leave the body along its normal. On C5/8
    (512 x (32 + 108) layers, 1e-5 wall spacing) straight lines to the far field leave 4,922 of the 16,384
    boundary-layer quadrangles skewed by more than 45 degrees (the aft surface: 8-9 degree parallelograms);
    normal layers leave only the trailing-edge fan's 28, every cell stays positive, the first layer's
    normal spacing is the wall spacing, and the cells three chords out are those of farmap 1."""
    m1 = fa.UMesh.naca_ogrid(512, 32, 108, 20.0, 1e-5, farmap=1)
    m3 = fa.UMesh.naca_ogrid(512, 32, 108, 20.0, 1e-5, farmap=3)
    assert (m1.nelem, m1.naface) == (m3.nelem, m3.naface) and np.array_equal(m1.intfac, m3.intfac)
    assert (m3.area > 0).all()
    _, d1 = _quad_skew(m1)
    _, d3 = _quad_skew(m3)
    assert (d1 > 45).sum() > 4000 and (d3 > 45).sum() <= 28, ((d1 > 45).sum(), (d3 > 45).sum())
    # first-layer points: distance from the surface point ~ 1e-5 * |f - s| / 20, along the normal
    s, p1 = m3.coords[:512], m3.coords[512:1024]
    d = np.linalg.norm(p1 - s, axis=1)
    assert np.all((d > 0.97e-5) & (d < 1.03e-5))
    own = np.tile(m1.coords[:512], (141, 1))          # each point's surface point (point j*512 + i)
    far = np.linalg.norm(m1.coords - own, axis=1) >= 3.0
    assert far.sum() > 10000 and np.array_equal(m1.coords[far], m3.coords[far])


def test_naca_cgrid():
    """generateNacaCgrid, the C5 family (BASELINE config 5's viscous case): (2 nwake + nsurf) columns x
    (nquad + 2 ntri) rows of cells; the wake cut is interior (the two wakes' row-0 points are shared), the
    wall is the body's row 0 (marker 2), the far field the outer row and both outflow columns (marker 4).
    On C5/8 every cell is positive and no boundary-layer quadrangle is skewed by more than 10 degrees
    (the straight-line O-grid's: 82, with 4,922 above 45)."""
    ns, nw, nq, nt = 384, 64, 32, 108
    m = fa.UMesh.naca_cgrid(ns, nw, nq, nt, 20.0, 1e-5)
    cols, rows = 2 * nw + ns, nq + 2 * nt
    assert m.nelem == cols * rows == 126976
    tags = m.btags[:, 0] if m.btags.ndim > 1 else m.btags
    assert (tags == 2).sum() == ns and (tags == 4).sum() == cols + 2 * (nq + nt)
    assert (m.area > 0).all()
    # interior faces: every cell edge not on the boundary is shared (Euler: 4-sided cells, 3-sided cells)
    assert m.naface == (4 * (m.nnode == 4).sum() + 3 * (m.nnode == 3).sum() + m.nbface) // 2
    _, d = _quad_skew(m)
    assert d.max() < 10.0, d.max()
    # the first row's points lie ~1e-5 off the wall, the cut's cells are thin (row 1 at 1e-5 above the cut)
    wall = np.where(tags == 2)[0]
    assert np.abs(m.gr[wall] - m.rc[m.intfac[wall, 0]]).max() < 1e-4


def test_gmsh_roundtrip(tmp_path):
    m = fa.UMesh.naca_ogrid(64, 4, 12)
    p = tmp_path / "o.msh"
    m.write_gmsh(p)
    m2 = fa.UMesh.read_gmsh(p)
    assert np.array_equal(m.intfac, m2.intfac)
    assert np.array_equal(m.facemetric, m2.facemetric)


def test_flatplate_struct_stretched_meshes(tmp_path):
    """tests/flatplate_meshes.py restates flatplatestructstretched.geo: 28 x 19 quads on mesh 0, each
    RefineMesh quadruples them; the domain [-0.5, 1] x [0, 1] is covered; markers 2 (plate) / 3 / 4 / 5
    on the right boundary pieces; first wall-normal spacing (1.4 progression, 20 points) halves per level"""
    from flatplate_meshes import write_flatplate_msh, flatplate_points
    for level, cells in enumerate((532, 2128, 8512)):
        path = str(tmp_path / f"fp{level}.msh")
        assert write_flatplate_msh(path, level) == cells
        m = fa.UMesh.read_gmsh(path)
        assert m.nelem == cells
        assert abs(m.area.sum() - 1.5) < 1e-12
        x, y = flatplate_points(level)
        assert abs(y[1] - 0.4 / (1.4 ** 19 - 1.0) / 2 ** level) < 1e-15
        tags = m.btags.reshape(m.nbface, -1)[:, 0]
        fm = m.facemetric.reshape(-1, 3)[:m.nbface]
        lens = {t: fm[tags == t, 2].sum() for t in (2, 3, 4, 5)}
        assert abs(lens[2] - 1.0) < 1e-12 and abs(lens[3] - 0.5) < 1e-12
        assert abs(lens[4] - 2.5) < 1e-12 and abs(lens[5] - 1.0) < 1e-12
