#!/usr/bin/env python3
"""Probe: which start and CFL make the bench's timed second-order implicit steps reduce the residual
(VERDICT r3 item 6). For each schedule: a first-order start of `init` steps (expResidualRamp from
cfl0 to cfl1, aodesolver.cpp:110-120, 462), then `main` second-order steps at a fixed or ramped CFL;
prints the residual history of both stages as one JSON line per schedule. One GPU, C4 mesh.
usage: python tools/implicit_probe.py [--scale S]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--case", default="naca")
    ap.add_argument("--schedules", default="")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    mesh, dims = c4_mesh(fa, args.scale)
    p = cases.physics("naca")
    n2 = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    n1 = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA", order2=False)
    sp1 = fa.FlowFV(mesh, p, n1, device=0)
    sp2 = fa.FlowFV(mesh, p, n2, device=0)
    perm = sp1.permutation()
    u0 = np.tile(cases.freestream(p), (mesh.nelem, 1))[perm]
    lin = dict(lin_rtol=1e-2, lin_maxit=30, restart=30, prec_sweeps=1, prec_lines=True)
    # (init steps, init cfl0, init cfl1, main steps, main cfl0, main cfl1)
    scheds = [(5, 25, 25, 6, 25, 25), (20, 5, 200, 6, 25, 25), (50, 5, 500, 6, 25, 25), (50, 5, 500, 6, 5, 5),
              (50, 5, 500, 6, 10, 10), (100, 5, 1000, 6, 25, 25), (20, 25, 25, 6, 10, 10), (10, 25, 25, 6, 5, 5)]
    if args.schedules:
        scheds = [tuple(float(x) for x in s.split(":")) for s in args.schedules.split(",")]
    for (ni, c0, c1, nm, m0, m1) in scheds:
        du = torch.tensor(u0, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()      # torch's stream vs the library's (non-blocking) streams
        try:
            t0 = time.perf_counter()
            st1, h1 = ({"cfl": None}, []) if int(ni) == 0 else sp1.steady_backward_euler_device(
                du.data_ptr(), fa.ImplicitConfig(cflinit=c0, cflfin=c1, tol=0.0, maxiter=int(ni), **lin))
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            st2, h2 = sp2.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(
                cflinit=m0, cflfin=m1, tol=0.0, maxiter=int(nm), **lin))
            torch.cuda.synchronize()
            t2 = time.perf_counter()
        except Exception as e:       # a diverging schedule (the solver's own error)
            print(json.dumps({"init": [ni, c0, c1], "main": [nm, m0, m1], "error": str(e)}), flush=True)
            continue
        print(json.dumps({"init": [ni, c0, c1], "main": [nm, m0, m1], "init_hist": [float(x) for x in h1],
                          "init_cfl": st1["cfl"], "main_hist": [float(x) for x in h2], "main_lin": st2["lin_iters"],
                          "main_resratio": st2["resratio"], "init_s": round(t1 - t0, 2),
                          "main_ms_per_step": round((t2 - t1) / max(st2["steps"], 1) * 1e3, 2)}), flush=True)
    sp1.close()
    sp2.close()


if __name__ == "__main__":
    main()
