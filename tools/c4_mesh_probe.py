"""probe: which O-grid parameters let the SECOND-order (Roe + WLS + Van Albada) explicit solve at M 0.8,
1.25 deg reach a steady state: variants of the C4 generator at reduced size"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

p = cases.physics("naca")
VARIANTS = [(256, 32, 108, 20.0, 1e-3), (256, 32, 108, 20.0, 1e-5)]
CFL = float(sys.argv[1]) if len(sys.argv) > 1 else 0.5
NSTEP = int(sys.argv[2]) if len(sys.argv) > 2 else 300000
for (nt, nq, ntri, rfar, ws) in VARIANTS:
    m = fa.UMesh.naca_ogrid(nt, nq, ntri, rfar, ws)
    sp = fa.FlowFV(m, p, cases.numerics("ROE", "LEASTSQUARES", "VANALBADA"))
    du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[sp.permutation()], device="cuda")
    t0 = time.time()
    try:
        steps, ratio, hist = sp.steady_forward_euler_device(du.data_ptr(), CFL, 1e-9, NSTEP)
        h = np.asarray(hist)[:steps]
        k = int(np.argmax(h))
        print(f"cfl {CFL} {(nt, nq, ntri, rfar, ws)} cells {m.nelem}: steps {steps} peak {h[k]:.2e} last {h[-1]:.2e} "
              f"drop-from-peak {h[-1]/h[k]:.1e} {time.time()-t0:.1f}s", flush=True)
        print("   hist", " ".join("%.1e" % x for x in h[::max(1, steps // 15)]), flush=True)
    except RuntimeError as e:
        print(f"{(nt, nq, ntri, rfar, ws)}: {e}", flush=True)
    sp.close()
