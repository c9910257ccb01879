"""probe: first-order then second-order implicit solves on the C4-family NACA0012 O-grid (reduced
scale) with several wall spacings / fluxes / CFL schedules: residual history, where the density peaks"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 8
p = cases.physics("naca")
print("physics: M", p.Minf, "aoa", p.aoa, flush=True)
for ws in (1e-5, 1e-3):
    m = fa.UMesh.naca_ogrid(2048 // scale, 256 // scale, 864 // scale, 20.0, ws)
    rc = m.rc
    for flux, cfl in (("ROE", (5.0, 100.0)), ("HLLC", (5.0, 100.0)), ("ROE", (1.0, 20.0))):
        n1 = cases.numerics(flux, "NONE", "NONE", order2=False)
        sp = fa.FlowFV(m, p, n1)
        perm = sp.permutation()
        du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[perm], device="cuda")
        lin = dict(lin_rtol=1e-2, lin_maxit=60, restart=60, min_relax=0.2, prec_sweeps=4)
        t0 = time.time()
        try:
            st, hist = sp.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(
                cflinit=cfl[0], cflfin=cfl[1], tol=1e-6, maxiter=400, **lin))
            h = hist[:st["steps"]]
            u = np.empty((m.nelem, 4)); u[perm] = du.cpu().numpy()
            i = int(np.argmax(u[:, 0]))
            print(f"ws {ws} {flux} cfl {cfl}: steps {st['steps']} ratio {st['resratio']:.3e} peak {h.max():.3e}@{int(np.argmax(h))} "
                  f"last {h[-1]:.3e} rho [{u[:,0].min():.3f},{u[:,0].max():.3f}] at ({rc[i,0]:.4f},{rc[i,1]:.4f}) "
                  f"{time.time()-t0:.1f}s", flush=True)
            print("   hist", " ".join("%.2e" % x for x in h[::20]), flush=True)
        except RuntimeError as e:
            print(f"ws {ws} {flux} cfl {cfl}: FAILED {e}", flush=True)
        sp.close()
