"""Per-rank subdomain meshes (the mesh each MPI rank of the reference holds): the oracle's literal
restatement of restrictMeshToPartitions + preprocessMesh (meshpartitioning.cpp:24-159) against the
product's, index for index, and the oracle's multi-rank residual (flow_spatial.cpp:636-816 with the
ghost-gradient and face-trace exchanges, tracevector.cpp:213-340) against its single-domain residual.
CPU only; the device path is tests/test_gpu_rankmesh.py."""
import numpy as np
import pytest

import fvens_amd as fa
import _oracle as orc
import cases

MESHES = {
    "testhybrid": (lambda: fa.UMesh.read_gmsh(cases.fixture_mesh("testhybrid")),
                   lambda: orc.OracleMesh.read(cases.fixture_mesh("testhybrid"))),
    "2dcylinderhybrid": (lambda: fa.UMesh.read_gmsh(cases.fixture_mesh("2dcylinderhybrid")),
                         lambda: orc.OracleMesh.read(cases.fixture_mesh("2dcylinderhybrid"))),
}


def _pair(key):
    if key in MESHES:
        return MESHES[key][0](), MESHES[key][1]()
    m = fa.UMesh.naca_ogrid(64, 4, 10)
    return m, orc.OracleMesh.from_raw(m.raw())


def rank_states(gm, lms, u):
    """per-rank conserved state with the ghost rows a VecGhostUpdate leaves: row nelem+ic holds the
    global neighbour cell connface(ic,3)"""
    out = []
    for lm in lms:
        g = lm.global_elem_index()
        ur = np.zeros((lm.nelem + lm.nconnface, 4))
        ur[:lm.nelem] = u[g]
        if lm.nconnface:
            ur[lm.nelem:] = u[lm.connface[:, 3]]
        out.append(ur)
    return out


@pytest.mark.parametrize("key,nranks", [("testhybrid", 3), ("2dcylinderhybrid", 4), ("naca", 5), ("naca", 1)])
def test_oracle_restriction_matches_product(key, nranks):
    gm, ogm = _pair(key)
    d = fa.UMesh.partition_trivial(gm.nelem, nranks)
    np.testing.assert_array_equal(d, orc.partition_trivial(gm.nelem, nranks))
    for r in range(nranks):
        lm = gm.restrict(d, r)
        olm = ogm.restrict(d, r)
        assert (lm.nelem, lm.nbface, lm.naface, lm.nconnface) == (olm.nelem, olm.nbface, olm.naface, olm.nconnface)
        np.testing.assert_array_equal(lm.intfac, olm.get("intfac"))
        valid = np.arange(lm.maxnfael)[None, :] < lm.nnode[:, None]     # padding of triangles differs
        np.testing.assert_array_equal(lm.esuel[valid], olm.get("esuel")[valid])
        np.testing.assert_array_equal(lm.elemface[valid], olm.get("elemface")[valid])
        np.testing.assert_array_equal(lm.connface, olm.get("connface"))
        np.testing.assert_array_equal(lm.global_elem_index(), olm.get("globalElemIndex"))
        for name in ("facemetric", "area", "rc", "gr", "rcbp"):
            np.testing.assert_array_equal(getattr(lm, name), olm.get(name), err_msg=name)


SCHEMES = [("naca", "ROE", "LEASTSQUARES", "VANALBADA", True),
           ("naca", "LLF", "NONE", "NONE", False),
           ("cyl", "HLLC", "GREENGAUSS", "VENKATAKRISHNAN", True),
           ("naca", "ROE", "LEASTSQUARES", "NONE", True),
           ("naca", "AUSM", "GREENGAUSS", "WENO", True),
           ("viscconst", "ROE", "LEASTSQUARES", "VANALBADA", True)]


@pytest.mark.parametrize("kind,flux,grad,rec,order2", SCHEMES)
def test_oracle_ranks_close_to_single_domain(kind, flux, grad, rec, order2):
    """the reference's multi-rank residual differs from its one-rank residual only by the order of
    each cell's sum and by the connectivity faces' local orientation (-F(uR,uL,-n) on one side), so
    they agree to rounding; a wrong exchange would be O(1)"""
    gm = fa.UMesh.naca_ogrid(64, 4, 10)
    ogm = orc.OracleMesh.from_raw(gm.raw())
    p = cases.physics(kind)
    n = cases.numerics(flux, grad, rec, order2=order2)
    u = cases.state(gm, p, seed=5)
    one = orc.OracleSpatial(ogm, p, n)
    r1 = np.zeros((gm.nelem, 4))
    dt1 = np.zeros(gm.nelem)
    one.compute_residual(u, r1, True, dt1)
    nranks = 4
    d = orc.partition_trivial(gm.nelem, nranks)
    olms = [ogm.restrict(d, r) for r in range(nranks)]
    lms = [gm.restrict(d, r) for r in range(nranks)]
    sps = [orc.OracleSpatial(om, p, n) for om in olms]
    us = rank_states(gm, lms, u)
    rs = [np.zeros((om.nelem, 4)) for om in olms]
    dts = [np.zeros(om.nelem) for om in olms]
    orc.residual_ranks(sps, us, rs, True, dts)
    r = np.zeros_like(r1)
    dt = np.zeros_like(dt1)
    for lm, rr, dd in zip(lms, rs, dts):
        g = lm.global_elem_index()
        r[g] = rr
        dt[g] = dd
    scale = np.abs(r1).max(axis=0)
    assert (np.abs(r - r1).max(axis=0) <= 1e-12 * scale).all()      # measured <= 3e-15
    assert np.abs(dt - dt1).max() <= 1e-12 * np.abs(dt1).max()
