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
