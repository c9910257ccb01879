"""probe: implicit solve of the C4-family O-grid (1e-5 wall spacing) from free stream: first-order start at a
fixed CFL, then the second-order solve with a capped CFL ramp; line-implicit vs block-Jacobi"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases
from bench import c4_mesh

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 4
maxit = int(sys.argv[2]) if len(sys.argv) > 2 else 100
m, _ = c4_mesh(fa, scale)
p = cases.physics("naca")
n1 = cases.numerics("ROE", "NONE", "NONE", order2=False)
n2 = cases.numerics("ROE", "LEASTSQUARES", "VENKATAKRISHNAN")
for (c0, c1, c2), prec in (((25.0, 25.0, 200.0), dict(prec_lines=True, prec_sweeps=2)),
                           ((25.0, 100.0, 1000.0), dict(prec_lines=True, prec_sweeps=2)),
                           ((25.0, 25.0, 200.0), dict(prec_sweeps=4))):
    start, main = fa.FlowFV(m, p, n1), fa.FlowFV(m, p, n2)
    du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[main.permutation()], device="cuda")
    lin = dict(lin_rtol=1e-2, lin_maxit=60, restart=60, min_relax=0.2)
    lin.update(prec)
    t0 = time.time()
    try:
        st0, h0 = start.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(
            cflinit=c0, cflfin=c0, tol=1e-1, maxiter=30, **lin))
        st, hist = main.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(
            cflinit=c1, cflfin=c2, tol=1e-6, maxiter=maxit, **lin))
        torch.cuda.synchronize()
        print(scale, (c0, c1, c2), prec, "start", st0["steps"], "%.2e" % st0["resratio"], "main",
              {k: (round(v, 4) if isinstance(v, float) else v) for k, v in st.items()}, "%.1fs" % (time.time() - t0),
              np.array2string(hist[:st["steps"]:max(1, st["steps"] // 12)], precision=2), flush=True)
    except RuntimeError as e:
        print(scale, (c0, c1, c2), prec, "FAILED", e, flush=True)
    start.close(); main.close()
