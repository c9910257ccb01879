"""probe: does the SECOND-order discretisation on the C4 family reach a steady state at all? The explicit
driver (local time steps, no linearisation) on reduced-scale members, per reconstruction"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 8
p = cases.physics("naca")
for wall in (1e-3, 1e-5):
    m = fa.UMesh.naca_ogrid(2048 // scale, 256 // scale, 864 // scale, 20.0, wall)
    for rec, cfl in (("VANALBADA", 0.5), ("WENO", 0.5)):
        sp = fa.FlowFV(m, p, cases.numerics("ROE", "LEASTSQUARES", rec))
        du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[sp.permutation()], device="cuda")
        t0 = time.time()
        steps, ratio, hist = sp.steady_forward_euler_device(du.data_ptr(), cfl, 1e-10, 400000)
        h = np.asarray(hist)[:steps]
        k = int(np.argmax(h))
        print(f"wall {wall} {rec} cfl {cfl}: steps {steps} ratio {ratio:.2e} peak {h[k]:.2e}@{k} last {h[-1]:.2e} "
              f"drop-from-peak {h[-1]/h[k]:.1e} {time.time()-t0:.1f}s", flush=True)
        print("   hist", " ".join("%.1e" % x for x in h[::max(1, steps // 20)]), flush=True)
        sp.close()
