"""probe: implicit backward Euler at small fixed CFL on the C4-family O-grid (first order, Roe): does
it follow the explicit solver (which converges) when the pseudo-time step is as small?"""
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
for flux, jflux in (("ROE", "ROE"), ("ROE", "LLF"), ("LLF", "LLF")):
    n1 = cases.numerics(flux, "NONE", "NONE", order2=False)
    n1.conv_numflux_jac = jflux
    sp = fa.FlowFV(m, p, n1)
    perm = sp.permutation()
    u0 = np.tile(cases.freestream(p), (m.nelem, 1))[perm]
    for cfl, nit in ((0.8, 3000), (2.0, 2000), (5.0, 2000), (20.0, 1000)):
        du = torch.tensor(u0, device="cuda")
        t0 = time.time()
        try:
            st, hist = sp.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(
                cflinit=cfl, cflfin=cfl, tol=1e-9, maxiter=nit, lin_rtol=1e-3, lin_maxit=100, restart=100,
                min_relax=1.0, prec_sweeps=4))
            h = hist[:st["steps"]]
            print(f"{flux}/{jflux} cfl {cfl}: steps {st['steps']} ratio {st['resratio']:.3e} lin/step "
                  f"{st['lin_iters']/max(1,st['steps']):.1f} {time.time()-t0:.1f}s", flush=True)
            print("   hist", " ".join("%.2e" % x for x in h[::max(1, len(h) // 20)]), flush=True)
        except RuntimeError as e:
            print(f"{flux}/{jflux} cfl {cfl}: FAILED {e}", flush=True)
    sp.close()
