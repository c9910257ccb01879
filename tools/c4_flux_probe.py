"""probe: is the second-order stall on the C4 family the Roe flux? Explicit second-order solves with
Roe and HLLC on a C4-family member and on the reference's naca0012luo grid"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

p = cases.physics("naca")
meshes = [("c4 family 256x140 ws1e-3", fa.UMesh.naca_ogrid(256, 32, 108, 20.0, 1e-3)),
          ("naca0012luo", fa.UMesh.read_gmsh(cases.fixture_mesh("naca0012luo")))]
for name, m in meshes:
    for flux, rec in (("HLLC", "VANALBADA"), ("ROE", "VANALBADA"), ("HLL", "VANALBADA"), ("LLF", "VANALBADA")):
        sp = fa.FlowFV(m, p, cases.numerics(flux, "LEASTSQUARES", rec))
        du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[sp.permutation()], device="cuda")
        t0 = time.time()
        try:
            steps, ratio, hist = sp.steady_forward_euler_device(du.data_ptr(), 0.5, 1e-9, 300000)
            h = np.asarray(hist)[:steps]
            k = int(np.argmax(h))
            print(f"{name} {flux}/{rec}: cells {m.nelem} steps {steps} peak {h[k]:.2e} last {h[-1]:.2e} "
                  f"drop-from-peak {h[-1]/h[k]:.1e} {time.time()-t0:.1f}s", flush=True)
        except RuntimeError as e:
            print(f"{name} {flux}/{rec}: {e}", flush=True)
        sp.close()
