"""probe: step-by-step implicit iterations on the C4-family O-grid to find where the solve blows up"""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases
from bench import c4_mesh

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 4
cfl = float(sys.argv[2]) if len(sys.argv) > 2 else 25.0
lines = len(sys.argv) > 3 and sys.argv[3] == "lines"
m, _ = c4_mesh(fa, scale)
p = cases.physics("naca")
for order2 in (False, True):
    n = cases.numerics("ROE", "LEASTSQUARES" if order2 else "NONE", "VENKATAKRISHNAN" if order2 else "NONE", order2=order2)
    sp = fa.FlowFV(m, p, n)
    if not order2:
        du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[sp.permutation()], device="cuda")
    lin = dict(lin_rtol=1e-2, lin_maxit=60, restart=60, min_relax=0.2, prec_lines=lines, prec_sweeps=2 if lines else 4)
    for k in range(30):
        try:
            st, hist = sp.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(cflinit=cfl, cflfin=cfl, tol=0.0,
                                                                                        maxiter=1, **lin))
            u = du.cpu().numpy()
            print("order2" if order2 else "order1", k, "res %.3e" % hist[0], "lin", st["lin_iters"],
                  "rho [%.3e, %.3e]" % (u[:, 0].min(), u[:, 0].max()), flush=True)
        except RuntimeError as e:
            print("order2" if order2 else "order1", k, "FAILED", e, flush=True)
            sys.exit(0)
    sp.close()
