"""probe: explicit second-order solves (local time steps, from the free stream) on the reference's
naca0012luo grid per reconstruction -- is a limiter's steady state reachable on a grid where the
reference's own regression converges?  usage: python tools/limiter_probe.py STEPS"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

nsteps = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
p = cases.physics("naca")
m = fa.UMesh.read_gmsh("tests/fixtures/meshes/naca0012luo.msh")
for rec, K, cfl in (("VANALBADA", 5.0, 0.5), ("VENKATAKRISHNAN", 5.0, 0.5), ("VENKATAKRISHNAN", 5.0, 0.2),
                    ("VENKATAKRISHNAN", 0.5, 0.2), ("BARTHJESPERSEN", 5.0, 0.5), ("NONE", 5.0, 0.5)):
    sp = fa.FlowFV(m, p, cases.numerics("ROE", "LEASTSQUARES", rec, K=K))
    du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[sp.permutation()], device="cuda")
    t0 = time.time()
    try:
        steps, ratio, hist = sp.steady_forward_euler_device(du.data_ptr(), cfl, 1e-10, nsteps)
    except RuntimeError as e:
        print(f"{rec} K {K} cfl {cfl}: {e}", flush=True)
        sp.close()
        continue
    h = np.asarray(hist)[:steps]
    k = int(np.argmax(h))
    (cl, cdp, _), _ = sp.surface_data_device(du.data_ptr(), 2)
    print(f"{rec} K {K} cfl {cfl}: steps {steps} peak {h[k]:.2e}@{k} last {h[-1]:.2e} drop-from-peak {h[-1]/h[k]:.1e} "
          f"CL {cl:.5f} CDp {cdp:.5f} {time.time()-t0:.1f}s", flush=True)
    print("   hist", " ".join("%.1e" % x for x in h[::max(1, steps // 20)]), flush=True)
    sp.close()
