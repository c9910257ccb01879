#!/usr/bin/env python3
"""Probe: what cutting the line-implicit preconditioner's lines at rank boundaries costs in GMRES
iterations. The C4 mesh split N ways by bench.py's cost-weighted graph partitioner,
all ranks in one process on one GPU (FlowFVGroup: the same solver, block-Jacobi across ranks); for
each N the same start (first-order implicit steps on one GPU) and then `steps` second-order
backward-Euler steps with GMRES(30), rtol 1e-2, line-implicit preconditioner. Prints one JSON line per
N: linear iterations per step, residual history, and the share of one-GPU line links cut.
usage: python tools/partitioned_lines_probe.py [--scale S] [--parts 1,2,4,8] [--steps K]
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
    ap.add_argument("--parts", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--init-steps", type=int, default=5)
    ap.add_argument("--cfl", type=float, default=25.0)
    ap.add_argument("--case", default="naca", choices=["naca", "visc-c5"])
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    mesh, dims = c4_mesh(fa, args.scale, 2 if args.case == "visc-c5" else 1)
    p = cases.physics("visc" if args.case == "visc-c5" else "naca")
    n2 = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    n1 = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA", order2=False)
    lin = dict(lin_rtol=1e-2, lin_maxit=30, restart=30, prec_sweeps=1, prec_lines=True)
    # common start: first-order implicit steps on one GPU, in the global numbering
    one1 = fa.FlowFV(mesh, p, n1, device=0)
    perm = one1.permutation()
    du = torch.tensor(np.tile(cases.freestream(p), (mesh.nelem, 1))[perm], dtype=torch.float64, device="cuda")
    one1.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(cflinit=args.cfl, cflfin=args.cfl, tol=0.0,
                                                                       maxiter=args.init_steps, **lin))
    u0 = np.empty((mesh.nelem, 4))
    u0[perm] = du.cpu().numpy()
    one1.close()
    del du
    cfg = fa.ImplicitConfig(cflinit=args.cfl, cflfin=args.cfl, tol=0.0, maxiter=args.steps, **lin)
    links = None
    for nparts in [int(x) for x in args.parts.split(",")]:
        if nparts == 1:
            sp = fa.FlowFV(mesh, p, n2, device=0)
            pm = sp.permutation()
            if links is None:
                links = [(pm[c], f) for c, f in sp.lines()]
            d = torch.tensor(u0[pm], dtype=torch.float64, device="cuda")
            t0 = time.perf_counter()
            st, hist = sp.steady_backward_euler_device(d.data_ptr(), cfg)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            sp.close()
            cut = 0.0
            nl = [len(links)]
        else:
            part = fa.partition_graph(mesh, nparts, weights="cost")
            sps = [fa.FlowFV(mesh, p, n2, device=0, partition=part, rank=k) for k in range(nparts)]
            dus = []
            for k, s_ in enumerate(sps):
                g = np.nonzero(part == k)[0][s_.permutation()]
                d = torch.zeros((s_.nown + s_.nghost, 4), dtype=torch.float64, device="cuda")
                d[:s_.nown] = torch.tensor(u0[g], device="cuda")
                dus.append(d)
            torch.cuda.synchronize()  # torch's stream vs the library's (non-blocking) streams
            grp = fa.FlowFVGroup(sps)
            t0 = time.perf_counter()
            st, hist = grp.steady_backward_euler_device([d.data_ptr() for d in dus], cfg)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            nl = [len(s_.lines()) for s_ in sps]
            grp.close()
            for s_ in sps:
                s_.close()
            del dus
            tot = sum(len(g) - 1 for g, _ in links)
            cut = sum(int(np.count_nonzero(part[g[1:]] != part[g[:-1]])) for g, _ in links) / max(tot, 1)
        print(json.dumps({"case": args.case, "cells": mesh.nelem, "ranks": nparts, "steps": st["steps"],
                          "lin_iters_per_step": round(st["lin_iters"] / max(st["steps"], 1), 2),
                          "resratio": st["resratio"], "hist": [float(x) for x in hist],
                          "cut_line_link_fraction": round(cut, 5), "lines_per_rank": nl,
                          "ms_per_step_one_gpu_group": round(dt / max(st["steps"], 1) * 1e3, 1),
                          "cfl": args.cfl, "init_steps": args.init_steps}), flush=True)


if __name__ == "__main__":
    main()
