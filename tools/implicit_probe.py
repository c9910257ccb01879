"""probe: implicit solves of BASELINE configs 2/3 (C3 flat plate 1024^2, HLLC + WLS + viscous) and
4 (C4 NACA0012 O-grid, Roe + WLS + Venkatakrishnan / MUSCL) with the line-implicit preconditioner"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases
from bench import c4_mesh

which = sys.argv[1] if len(sys.argv) > 1 else "c4"
maxit = int(sys.argv[2]) if len(sys.argv) > 2 else 200


def run(m, p, n1, n2, start_cfg, main_cfg, label):
    start = fa.FlowFV(m, p, n1) if n1 is not None else None
    main = fa.FlowFV(m, p, n2)
    perm = main.permutation()
    du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[perm], device="cuda")
    t0 = time.time()
    if start is not None:
        st0, h0 = start.steady_backward_euler_device(du.data_ptr(), start_cfg)
        torch.cuda.synchronize()
        print(label, "starter", {k: (round(v, 4) if isinstance(v, float) else v) for k, v in st0.items()},
              "%.1fs" % (time.time() - t0), flush=True)
    t1 = time.time()
    st, hist = main.steady_backward_euler_device(du.data_ptr(), main_cfg)
    torch.cuda.synchronize()
    dt = time.time() - t1
    print(label, "main", st, "%.1fs" % dt, "ms/step %.1f" % (1e3 * dt / max(1, st["steps"])), flush=True)
    print(label, "history", np.array2string(hist[:st["steps"]:max(1, st["steps"] // 20)], precision=3), flush=True)
    if start is not None:
        start.close()
    main.close()


if which == "c3":
    m = fa.UMesh.flat_plate(1024, 1024)
    p = cases.physics("plate")
    n2 = cases.numerics("HLLC", "LEASTSQUARES", "NONE")
    for mf in (False, True):
        lin = dict(lin_rtol=1e-1, lin_maxit=60, restart=60, prec_lines=True, prec_sweeps=2, min_relax=0.2)
        run(m, p, None, n2, None, fa.ImplicitConfig(cflinit=10.0, cflfin=2000.0, tol=1e-6, maxiter=maxit,
                                                    matrix_free=mf, **lin), "c3 mf=%d" % mf)
else:
    m, _ = c4_mesh(fa, 1)
    p = cases.physics("naca")
    n1 = cases.numerics("ROE", "NONE", "NONE", order2=False)
    for rec in ("VENKATAKRISHNAN", "VANALBADA"):
        n2 = cases.numerics("ROE", "LEASTSQUARES", rec)
        lin = dict(lin_rtol=1e-1, lin_maxit=60, restart=60, prec_lines=True, prec_sweeps=2, min_relax=0.2)
        run(m, p, n1, n2, fa.ImplicitConfig(cflinit=50.0, cflfin=1000.0, tol=1e-1, maxiter=50, **lin),
            fa.ImplicitConfig(cflinit=50.0, cflfin=5000.0, tol=1e-6, maxiter=maxit, **lin), "c4 " + rec)
