"""probe: does Venkatakrishnan's differentiable limiter (BASELINE config 4's reconstruction) take the
C4 family to a steady state where Van Albada limit-cycles? Explicit driver (local time steps), from the
free stream, per limiter parameter K (eps^2 = (K clength)^3) and wall spacing.
usage: python tools/c4_venkat_probe.py SCALE STEPS K1 K2 ..."""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

scale, nsteps = int(sys.argv[1]), int(sys.argv[2])
Ks = [float(k) for k in sys.argv[3:]] or [5.0]
p = cases.physics("naca")
for wall in (1e-3, 1e-5):
    m = fa.UMesh.naca_ogrid(2048 // scale, 256 // scale, 864 // scale, 20.0, wall, farmap=1)
    for K in Ks:
        for cfl in (0.5,):
            sp = fa.FlowFV(m, p, cases.numerics("ROE", "LEASTSQUARES", "VENKATAKRISHNAN", K=K))
            du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[sp.permutation()], device="cuda")
            t0 = time.time()
            try:
                steps, ratio, hist = sp.steady_forward_euler_device(du.data_ptr(), cfl, 1e-10, nsteps)
            except RuntimeError as e:
                print(f"wall {wall} K {K} cfl {cfl}: {e}", flush=True)
                sp.close()
                continue
            h = np.asarray(hist)[:steps]
            k = int(np.argmax(h))
            (cl, cdp, _), _ = sp.surface_data_device(du.data_ptr(), 2)
            print(f"wall {wall} K {K} cfl {cfl} cells {m.nelem}: steps {steps} ratio {ratio:.2e} peak {h[k]:.2e}@{k} "
                  f"last {h[-1]:.2e} drop-from-peak {h[-1]/h[k]:.1e} CL {cl:.5f} CDp {cdp:.5f} {time.time()-t0:.1f}s", flush=True)
            print("   hist", " ".join("%.1e" % x for x in h[::max(1, steps // 20)]), flush=True)
            sp.close()
