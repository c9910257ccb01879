"""Surface functionals on the device: FlowFV_base::computeSurfaceData
(flow_spatial.cpp:130-310) through fvhip_surface_data_device, against the oracle's restatement on the
same state and gradients.

Bars: CL and CDp bitwise (same operations in the same face order; the wind vector and free-stream
pressure are formed on the host as the reference does); CDsf to 1e-12 relative (Sutherland's
T^1.5 is the device pow, which may differ from the host's in the last bit); per-face Cp bitwise
against a numpy restatement of getPressureFromConserved, face centres equal to the mesh's gr.
"""
import numpy as np
import pytest

import fvens_amd as fa
import _oracle as orc
import cases
from test_gpu_residual import get_mesh

pytestmark = pytest.mark.gpu


def _run(kind, seed):
    import torch
    m, om = get_mesh("naca_small")
    p = cases.physics(kind)
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    u = cases.state(m, p, seed)
    dev = fa.FlowFV(m, p, n)
    perm = dev.permutation()
    dU = torch.tensor(np.ascontiguousarray(u[perm]), device="cuda")
    (cl, cdp, cdf), faces = dev.surface_data_device(dU.data_ptr(), 2)
    ref = orc.OracleSpatial(om, p, n)
    rcl, rcdp, rcdf = ref.surface(u, ref.getGradients(u), 2)
    dev.close()
    return m, p, u, (cl, cdp, cdf), faces, (rcl, rcdp, rcdf)


@pytest.mark.parametrize("kind,seed", [("naca", 3), ("visc", 5)])
def test_surface_functionals_match_oracle(kind, seed):
    m, p, u, (cl, cdp, cdf), faces, (rcl, rcdp, rcdf) = _run(kind, seed)
    assert cl == rcl and cdp == rcdp, (cl, rcl, cdp, rcdp)
    assert abs(cdf - rcdf) <= 1e-12 * abs(rcdf), (cdf, rcdf)
    if kind == "visc":
        assert rcdf != 0.0
    # per face, reference boundary-face order: centre and Cp
    nb = m.nbface
    wall = np.nonzero(np.asarray(m.btags).reshape(nb, -1)[:, 0] == 2)[0]
    assert faces.shape == (len(wall), 4)
    L = m.intfac[wall, 0]
    uc = u[L]
    pr = (p.gamma - 1.0) * (uc[:, 3] - (0.5 * (uc[:, 1] * uc[:, 1] + uc[:, 2] * uc[:, 2])) / uc[:, 0])
    pinf = 1.0 / (p.gamma * p.Minf * p.Minf)
    assert np.array_equal(faces[:, 2], (pr - pinf) * 2.0)
    assert np.array_equal(faces[:, :2], np.asarray(m.gr).reshape(-1, 2)[wall])
