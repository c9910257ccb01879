"""probe: implicit convergence of the cylinder entropy cases on the finest mesh under several linear-solver
settings (device GMRES + block-Jacobi / multicolour GS / line-implicit)"""
import sys
import time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import fvens_amd as fa
import cases

SETTINGS = [dict(prec_sweeps=2, prec_gs=True), dict(prec_sweeps=1), dict(prec_sweeps=4),
            dict(prec_sweeps=4, prec_gs=True), dict(prec_sweeps=2, prec_lines=True),
            dict(prec_sweeps=1, prec_lines=True), dict(prec_sweeps=2, prec_gs=True, cflfin=2500.0),
            dict(prec_sweeps=1, cflfin=2500.0)]
mesh = sys.argv[1] if len(sys.argv) > 1 else "2dcylinder3"
grads = sys.argv[2].split(",") if len(sys.argv) > 2 else ["LEASTSQUARES", "GREENGAUSS"]
CFL = {"LEASTSQUARES": (250.0, 5000.0), "GREENGAUSS": (250.0, 1000.0)}
for grad in grads:
    for sett in SETTINGS:
        sett = dict(sett)
        cfl = (CFL[grad][0], sett.pop("cflfin", CFL[grad][1]))
        m = fa.UMesh.read_gmsh(cases.fixture_mesh(mesh))
        p = cases.physics("cyl")
        start = fa.FlowFV(m, p, cases.numerics("HLLC", "NONE", "NONE", order2=False))
        sp = fa.FlowFV(m, p, cases.numerics("HLLC", grad, "NONE"))
        perm = sp.permutation()
        du = torch.tensor(np.tile(cases.freestream(p), (m.nelem, 1))[perm], device="cuda")
        lin = dict(lin_rtol=1e-1, lin_maxit=30, restart=30, min_relax=0.2)
        lin.update(sett)
        start.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(cflinit=25.0, cflfin=500.0, tol=1e-1,
                                                                            maxiter=150, **lin))
        t0 = time.time()
        st, hist = sp.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(cflinit=cfl[0], cflfin=cfl[1],
                                                                                    tol=1e-8, maxiter=1500, **lin))
        print(grad, sett, cfl, "steps", st["steps"], "ratio %.3e" % st["resratio"], "cfl %.0f" % st["cfl"],
              "lin/step %.1f" % (st["lin_iters"] / max(st["steps"], 1)), "%.1fs" % (time.time() - t0),
              "err %.6f" % np.log10(sp.entropy_error_device(du.data_ptr())), flush=True)
        start.close(); sp.close()
