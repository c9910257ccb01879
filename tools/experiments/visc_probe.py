"""probe: the visc-naca0012 regression (laminar-implicit.ctrl) with the device implicit solver under
several preconditioners"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases
from test_gpu_viscous import REGR, _visc_naca_physics

m = fa.UMesh.read_gmsh(cases.fixture_mesh("NACA0012_lam_hybrid_1"))
p = _visc_naca_physics()
for mf in (False, True):
    for prec in (dict(prec_lines=True, prec_sweeps=1), dict(prec_lines=True, prec_sweeps=2),
                 dict(prec_lines=True, prec_sweeps=3, lin_maxit=60, restart=60)):
        start = fa.FlowFV(m, p, cases.numerics("ROE", "NONE", "NONE", order2=False))
        main = fa.FlowFV(m, p, cases.numerics("ROE", "LEASTSQUARES", "NONE"))
        perm = main.permutation()
        du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[perm], device="cuda")
        lin = dict(lin_rtol=1e-1, lin_maxit=30, restart=30, min_relax=1.0)
        lin.update(prec)
        t0 = time.time()
        st0, _ = start.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(cflinit=200.0, cflfin=1000.0,
                                                                                    tol=1e-1, maxiter=50, **lin))
        st, _ = main.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(cflinit=500.0, cflfin=5000.0,
                                                                                  tol=1e-6, maxiter=300,
                                                                                  matrix_free=mf, **lin))
        (cl, cdp, cdsf), _ = main.surface_data_device(du.data_ptr(), 2)
        print("mf", mf, prec, "starter", st0["steps"], "%.2e" % st0["resratio"], "main", st["steps"],
              "%.2e" % st["resratio"], "lin/step %.1f" % (st["lin_iters"] / max(1, st["steps"])),
              "%.1fs" % (time.time() - t0), "CL %.6e CDp %.10f CDsf %.10f" % (cl, cdp, cdsf),
              "rel %.1e %.1e %.1e" % (abs(cl / REGR[0] - 1), abs(cdp / REGR[1] - 1), abs(cdsf / REGR[2] - 1)), flush=True)
        start.close(); main.close()
