"""GPU probe: implicit solves on 4 per-rank meshes (group) vs one rank, residual histories side by side
(diagnoses test_gpu_rankmesh.py::test_entropy_convergence_four_rank_meshes)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import fvens_amd as fa  # noqa: E402
import cases  # noqa: E402


def run(name, nranks, init, main, lin):
    gm = fa.UMesh.read_gmsh(cases.fixture_mesh(name))
    p = cases.physics("cyl")
    n1 = cases.numerics("HLLC", "NONE", "NONE", order2=False)
    n2 = cases.numerics("HLLC", "LEASTSQUARES", "NONE")
    out = {}
    # one rank
    s1, s2 = fa.FlowFV(gm, p, n1), fa.FlowFV(gm, p, n2)
    du = torch.tensor(np.tile(cases.freestream(p), (gm.nelem, 1)), device="cuda")
    a = s1.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(cflinit=init[0], cflfin=init[1], tol=init[2],
                                                                         maxiter=init[3], **lin))
    try:
        b = s2.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(cflinit=main[0], cflfin=main[1], tol=main[2],
                                                                             maxiter=main[3], **lin))
    except RuntimeError as e:
        b = ({"error": str(e)}, np.zeros(0))
    out[1] = (a, b)
    s1.close()
    s2.close()
    d = fa.UMesh.partition_trivial(gm.nelem, nranks)
    lms = [gm.restrict(d, r) for r in range(nranks)]
    starts, mains = [fa.FlowFV(lm, p, n1) for lm in lms], [fa.FlowFV(lm, p, n2) for lm in lms]
    for r in range(nranks):
        starts[r].set_rank(r, nranks)
        mains[r].set_rank(r, nranks)
    dus = [torch.tensor(np.tile(cases.freestream(p), (lm.nelem + lm.nconnface, 1)), device="cuda") for lm in lms]
    g1, g2 = fa.FlowFVGroup(starts), fa.FlowFVGroup(mains)
    a = g1.steady_backward_euler_device([x.data_ptr() for x in dus], fa.ImplicitConfig(
        cflinit=init[0], cflfin=init[1], tol=init[2], maxiter=init[3], **lin))
    try:
        b = g2.steady_backward_euler_device([x.data_ptr() for x in dus], fa.ImplicitConfig(
            cflinit=main[0], cflfin=main[1], tol=main[2], maxiter=main[3], **lin))
    except RuntimeError as e:
        b = ({"error": str(e)}, np.zeros(0))
    out[nranks] = (a, b)
    g1.close()
    g2.close()
    for sp in starts + mains:
        sp.close()
    return out


def show(tag, out):
    for k, (a, b) in out.items():
        print(tag, "ranks", k, "start", a[0], "main", b[0])
        print("   start hist", np.array2string(a[1][:12], precision=3))
        print("   main hist ", np.array2string(b[1][:40], precision=3))


if __name__ == "__main__":
    lin_gs = dict(lin_rtol=1e-2, lin_maxit=30, restart=30, min_relax=0.2, prec_sweeps=2, prec_gs=True)
    lin_j = dict(lin_rtol=1e-2, lin_maxit=30, restart=30, min_relax=0.2, prec_sweeps=1)
    for name in ("2dcylinder0", "2dcylinder1"):
        show(name + " fixed cfl 25 gs", run(name, 4, (25.0, 25.0, 1e-1, 10), (25.0, 25.0, 1e-7, 15), lin_gs))
        show(name + " test schedule gs", run(name, 4, (25.0, 500.0, 1e-1, 150), (250.0, 5000.0, 1e-7, 1500), lin_gs))
        show(name + " test schedule jacobi", run(name, 4, (25.0, 500.0, 1e-1, 150), (250.0, 5000.0, 1e-7, 1500), lin_j))
        sys.stdout.flush()
