"""probe: does the first-order discretisation on the C4-family O-grid reach a steady state? Explicit
forward Euler (local time steps) against implicit with tight linear solves and full updates"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ws = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-3
p = cases.physics("naca")
m = fa.UMesh.naca_ogrid(2048 // scale, 256 // scale, 864 // scale, 20.0, ws)
print("cells", m.nelem, "ws", ws, flush=True)
n1 = cases.numerics("ROE", "NONE", "NONE", order2=False)
sp = fa.FlowFV(m, p, n1)
perm = sp.permutation()
u0 = np.tile(cases.freestream(p), (m.nelem, 1))[perm]
du = torch.tensor(u0, device="cuda")
t0 = time.time()
steps, ratio, hist = sp.steady_forward_euler_device(du.data_ptr(), 0.8, 1e-10, 200000)
h = np.asarray(hist)[:steps]
print(f"explicit: steps {steps} ratio {ratio:.3e} {time.time()-t0:.1f}s", flush=True)
print("   hist", " ".join("%.2e" % x for x in h[::max(1, steps // 25)]), flush=True)
uex = du.cpu().numpy().copy()
for sett in (dict(lin_rtol=1e-4, lin_maxit=200, restart=100, min_relax=1.0, prec_sweeps=4),
             dict(lin_rtol=1e-4, lin_maxit=200, restart=100, min_relax=0.2, prec_sweeps=4),
             dict(lin_rtol=1e-4, lin_maxit=200, restart=100, min_relax=1.0, prec_lines=True, prec_sweeps=2)):
    for cfl in ((5.0, 5.0), (20.0, 20.0), (5.0, 200.0)):
        du = torch.tensor(u0, device="cuda")
        t0 = time.time()
        try:
            st, hist = sp.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(
                cflinit=cfl[0], cflfin=cfl[1], tol=1e-8, maxiter=300, **sett))
            h = hist[:st["steps"]]
            d = np.abs(du.cpu().numpy() - uex).max()
            print(f"implicit {sett} cfl {cfl}: steps {st['steps']} ratio {st['resratio']:.3e} lin {st['lin_iters']} "
                  f"|u - u_explicit| {d:.2e} {time.time()-t0:.1f}s", flush=True)
            print("   hist", " ".join("%.2e" % x for x in h[::15]), flush=True)
        except RuntimeError as e:
            print(f"implicit {sett} cfl {cfl}: FAILED {e}", flush=True)
