"""probe: cost of the line-implicit preconditioner (first-order LLF on the C4 family, 1e-5 wall
spacing): the wall time per implicit step with lines against point-block Jacobi"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 8
p = cases.physics("naca")
m = fa.UMesh.naca_ogrid(2048 // scale, 256 // scale, 864 // scale, 20.0, 1e-5)
sp = fa.FlowFV(m, p, cases.numerics("LLF", "NONE", "NONE", order2=False))
u0 = np.tile(cases.freestream(p), (m.nelem, 1))[sp.permutation()]
for sett in (dict(prec_sweeps=1), dict(prec_lines=True, prec_sweeps=1), dict(prec_lines=True, prec_sweeps=2)):
    du = torch.tensor(u0, device="cuda")
    t0 = time.time()
    st, h = sp.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(cflinit=5.0, cflfin=200.0, tol=1e-12,
                                            maxiter=400, lin_rtol=1e-2, lin_maxit=40, restart=40, min_relax=0.2, **sett))
    dt = time.time() - t0
    hh = h[:st["steps"]]
    print(sett, f"steps {st['steps']} lin/step {st['lin_iters']/st['steps']:.1f} ms/step {1e3*dt/st['steps']:.2f} "
          f"ms/lin-iter {1e3*dt/max(1,st['lin_iters']):.3f} drop-from-peak {hh[-1]/hh.max():.2e}", flush=True)
