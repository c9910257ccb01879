"""probe: CFL schedules and preconditioners for the first-order start on the C4-family O-grid at the
C4 wall spacing (1e-5) and coarser ones; each run reports where the residual peaks and how far it
falls from the peak"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 8
wss = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1e-5, 1e-4]
nit = int(sys.argv[3]) if len(sys.argv) > 3 else 1500
p = cases.physics("naca")
RUNS = [("LLF", dict(prec_sweeps=1, min_relax=0.2), (5.0, 200.0)),
        ("LLF", dict(prec_lines=True, prec_sweeps=1, min_relax=0.2), (5.0, 200.0)),
        ("LLF", dict(prec_lines=True, prec_sweeps=1, min_relax=0.2), (20.0, 1000.0)),
        ("ROE", dict(prec_lines=True, prec_sweeps=1, min_relax=0.2), (5.0, 200.0)),
        ("ROE", dict(prec_sweeps=1, min_relax=0.2), (5.0, 200.0))]
for ws in wss:
    m = fa.UMesh.naca_ogrid(2048 // scale, 256 // scale, 864 // scale, 20.0, ws)
    print("cells", m.nelem, "ws", ws, flush=True)
    for flux, sett, cfl in RUNS:
        n1 = cases.numerics(flux, "NONE", "NONE", order2=False)
        sp = fa.FlowFV(m, p, n1)
        perm = sp.permutation()
        du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[perm], device="cuda")
        t0 = time.time()
        try:
            st, hist = sp.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(
                cflinit=cfl[0], cflfin=cfl[1], tol=1e-12, maxiter=nit, lin_rtol=1e-2, lin_maxit=40, restart=40, **sett))
            h = hist[:st["steps"]]
            k = int(np.argmax(h))
            print(f"  {flux} {sett} cfl {cfl}: steps {st['steps']} peak {h[k]:.2e}@{k} last {h[-1]:.2e} "
                  f"drop-from-peak {h[-1]/h[k]:.1e} cfl_end {st['cfl']:.0f} lin/step {st['lin_iters']/max(1,st['steps']):.1f} "
                  f"{time.time()-t0:.1f}s", flush=True)
            print("     hist", " ".join("%.1e" % x for x in h[::max(1, len(h) // 15)]), flush=True)
        except RuntimeError as e:
            print(f"  {flux} {sett} cfl {cfl}: FAILED {e} {time.time()-t0:.1f}s", flush=True)
        sp.close()
