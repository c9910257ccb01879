"""Known-answer pin of the whole residual path against the reference's own functional regression:
testcases/naca0012 SpatialFlow_Euler_NACA0012_MUSCL_LeastSquares_HLLC_FunctionalRegression
(transonic-sanity-test-muscl.ctrl on grids/naca0012luo.msh: M 0.8, 1.25 deg, HLLC + least squares +
Van Albada) stores CL = 0.154112792928976, CDp = 0.0115814414408097 (regr-MUSCL_LeastSquares_HLLC.txt)
and checks CL to 1e-6 and CDp to 1e-8 relative (tests/flow_solve.cpp:89-126) after an implicit solve to a
1e-7 residual drop. Here the device explicit pseudo-time driver converges the same discretisation to
the same 1e-7 drop (28,168 steps on MI355X; the cap is 300,000) and the oracle evaluates the surface
functionals (flow_spatial.cpp:130-310).

The reference's 1e-8 CDp bar is not reachable by a different solver path, and the measured gap says
why (tools/experiments/regr_probe.py, in git history up to f4c3eb0, MI355X): converged to a 1e-11 drop -- implicitly, or explicitly to the
800,000-step cap -- this discretisation (bitwise the reference's residual) gives CL 9.07e-8 and CDp
4.65e-8 relative to the file, so the file's own values carry ~5e-8 of the reference's 1e-7-drop
convergence error. At the 1e-7 drop the explicit run sits at CL 9.1e-8 / CDp 4.65e-8, the implicit
one (test_gpu_implicit.py) at 8.2e-8 / 3.3e-8. Bars: CL 1e-6 (the reference's), CDp 1e-7 (twice the
measured converged gap)."""
import numpy as np
import pytest

import fvens_amd as fa
import _oracle as orc
import cases

pytestmark = pytest.mark.gpu

CL_REF, CDP_REF = 0.154112792928976, 0.0115814414408097


def test_naca0012_muscl_hllc_functionals():
    import torch
    m = fa.UMesh.read_gmsh(cases.fixture_mesh("naca0012luo"))
    om = orc.OracleMesh.read(cases.fixture_mesh("naca0012luo"))
    p = cases.physics("naca")
    n = cases.numerics("HLLC", "LEASTSQUARES", "VANALBADA")
    dev = fa.FlowFV(m, p, n)
    perm = dev.permutation()
    u0 = np.tile(cases.freestream(p), (m.nelem, 1))
    du = torch.tensor(u0[perm], device="cuda")
    steps, ratio, hist = dev.steady_forward_euler_device(du.data_ptr(), 0.8, 1e-7, 300000)
    u = np.empty_like(u0)
    u[perm] = du.cpu().numpy()
    ref = orc.OracleSpatial(om, p, n)
    cl, cdp, cdsf = ref.surface(u, ref.getGradients(u), 2)
    print(f"steps {steps} ratio {ratio:.3e} CL {cl!r} CDp {cdp!r}")
    assert ratio <= 1e-7
    assert abs(cl - CL_REF) / abs(CL_REF) <= 1e-6        # the reference's CL tolerance
    assert abs(cdp - CDP_REF) / abs(CDP_REF) <= 1e-7     # reference: 1e-8 (see the docstring for the gap)
    dev.close()
