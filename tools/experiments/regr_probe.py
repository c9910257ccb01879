"""probe: how close the NACA0012 MUSCL/LS/HLLC functionals get to regr-MUSCL_LeastSquares_HLLC.txt as
the device implicit solve is converged further (tol 1e-7 .. 1e-11), and the explicit run at 1e-7"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

CL_REF, CDP_REF = 0.154112792928976, 0.0115814414408097
m = fa.UMesh.read_gmsh(cases.fixture_mesh("naca0012luo"))
p = cases.physics("naca")
n1 = cases.numerics("HLLC", "NONE", "NONE", order2=False)
n2 = cases.numerics("HLLC", "LEASTSQUARES", "VANALBADA")
start, main = fa.FlowFV(m, p, n1), fa.FlowFV(m, p, n2)
perm = main.permutation()
u0 = np.tile(cases.freestream(p), (m.nelem, 1))[perm]
for sweeps, rtol in ((4, 1e-1), (4, 1e-3)):
    for tol in (1e-7, 1e-8, 1e-9, 1e-10, 1e-11):
        du = torch.tensor(u0, device="cuda")
        lin = dict(lin_rtol=rtol, lin_maxit=30, restart=30, prec_sweeps=sweeps, min_relax=0.2)
        start.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(cflinit=50.0, cflfin=1000.0, tol=1e-1,
                                                                           maxiter=20, **lin))
        t0 = time.time()
        st, hist = main.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(cflinit=500.0, cflfin=5000.0,
                                                                                     tol=tol, maxiter=3000, **lin))
        (cl, cdp, _), _ = main.surface_data_device(du.data_ptr(), 2)
        print(f"implicit sweeps {sweeps} rtol {rtol} tol {tol:.0e}: steps {st['steps']} ratio {st['resratio']:.2e} "
              f"conv {st['converged']} CL rel {abs(cl-CL_REF)/CL_REF:.2e} CDp rel {abs(cdp-CDP_REF)/CDP_REF:.2e} "
              f"{time.time()-t0:.1f}s", flush=True)
for tol in (1e-7, 1e-9):
    du = torch.tensor(u0, device="cuda")
    t0 = time.time()
    steps, ratio, hist = main.steady_forward_euler_device(du.data_ptr(), 0.8, tol, 800000)
    (cl, cdp, _), _ = main.surface_data_device(du.data_ptr(), 2)
    print(f"explicit tol {tol:.0e}: steps {steps} ratio {ratio:.2e} CL rel {abs(cl-CL_REF)/CL_REF:.2e} "
          f"CDp rel {abs(cdp-CDP_REF)/CDP_REF:.2e} {time.time()-t0:.1f}s", flush=True)
