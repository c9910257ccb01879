"""probe: explicit second-order solves (local time steps, from the free stream) on C4-family grids
with the far-field angles uniform in the surface parameter (generateNacaOgrid farmap 1), per
reconstruction and wall spacing. usage: python tools/c4_farmap_probe.py SCALE STEPS FARMAP"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

scale, nsteps, farmap = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
p = cases.physics("naca")
for wall in (1e-3, 1e-5):
    m = fa.UMesh.naca_ogrid(2048 // scale, 256 // scale, 864 // scale, 20.0, wall, farmap=farmap)
    for rec, K, cfl in (("VANALBADA", 5.0, 0.5), ("VENKATAKRISHNAN", 5.0, 0.5), ("NONE", 5.0, 0.5)):
        sp = fa.FlowFV(m, p, cases.numerics("ROE", "LEASTSQUARES", rec, K=K))
        du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[sp.permutation()], device="cuda")
        t0 = time.time()
        try:
            steps, ratio, hist = sp.steady_forward_euler_device(du.data_ptr(), cfl, 1e-10, nsteps)
        except RuntimeError as e:
            print(f"farmap {farmap} wall {wall} {rec} K {K} cfl {cfl}: {e}", flush=True)
            sp.close()
            continue
        h = np.asarray(hist)[:steps]
        k = int(np.argmax(h))
        (cl, cdp, _), _ = sp.surface_data_device(du.data_ptr(), 2)
        print(f"farmap {farmap} wall {wall} {rec} K {K} cfl {cfl} cells {m.nelem}: steps {steps} peak {h[k]:.2e}@{k} "
              f"last {h[-1]:.2e} drop-from-peak {h[-1]/h[k]:.1e} CL {cl:.5f} CDp {cdp:.5f} {time.time()-t0:.1f}s", flush=True)
        print("   hist", " ".join("%.1e" % x for x in h[::max(1, steps // 20)]), flush=True)
        sp.close()
