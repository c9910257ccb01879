#!/usr/bin/env python3
"""Single-GPU proxy of the multi-GPU strong-scaling run (BASELINE config 4 at 2/4/8 GPUs): the C4
mesh split N ways by the graph partitioner (bench.py --gpus N's default), every rank's handle built on
this one GPU, the ghost rows filled once by the in-process group exchange, then each rank's residual
timed ALONE with its halo already current (FVHIP_RES_HALO_READY: layer-1 ghost gradients + every
patch, no exchange). Reports per rank: owned / ghost cells, patches and interior-patch fraction, ms
per residual and its kernels; per N: the edge cut, the slowest rank (the compute floor of an N-GPU
step if the exchange is hidden) and the speed-up that floor implies over the 1-GPU residual.
    python tools/scale_proxy.py [--parts 2 4 8] [--rec VANALBADA|VENKATAKRISHNAN] [--steps 200] [--weights faces|none]
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


def timed(sp, du, dr, ddt, steps, preheat_s, halo_ready):
    def step():
        sp.compute_residual_device(du.data_ptr(), dr.data_ptr(), ddt.data_ptr(), True, True, halo_ready=halo_ready)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < preheat_s:
        for _ in range(20):
            step()
        sp.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sp.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    sp.profile(True)
    for _ in range(steps):
        step()
    kt = sp.kernel_times()
    sp.profile(False)
    return ms, {k: round(v[0] / steps, 5) for k, v in kt.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--rec", default="VANALBADA")
    ap.add_argument("--config5", action="store_true", help="BASELINE config 5: the hybrid C5 mesh, laminar viscous")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--preheat", type=float, default=0.3, help="seconds of untimed residuals before each timing")
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--weights", choices=["cost", "faces", "none"], default="cost",
                    help="graph partition weights: measured cost (bench.py's default), face counts or none (equal cells)")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    mesh, dims = c4_mesh(fa, args.scale, 2 if args.config5 else 1)
    p = cases.physics("visc" if args.config5 else "naca")
    # config 5: the visc-naca0012 deck's limiter none (laminar-implicit.ctrl:72)
    n = cases.numerics("ROE", "LEASTSQUARES", "NONE" if args.config5 else args.rec)
    u = cases.state(mesh, p, seed=42)
    N = mesh.nelem
    one = fa.FlowFV(mesh, p, n)
    du = torch.tensor(u[one.permutation()], device="cuda")
    dr = torch.empty((N, 4), dtype=torch.float64, device="cuda")
    ddt = torch.empty(N, dtype=torch.float64, device="cuda")
    t1, k1 = timed(one, du, dr, ddt, args.steps, args.preheat, False)
    one.close()
    print(json.dumps({"parts": 1, "cells": N, "ms_per_residual": round(t1, 5), "kernels_ms": k1, "numerics": args.rec}),
          flush=True)
    for nparts in args.parts:
        tp = time.time()
        part = fa.partition_graph(mesh, nparts, weights=None if args.weights == "none" else args.weights)
        tp = time.time() - tp
        sps = [fa.FlowFV(mesh, p, n, partition=part, rank=k) for k in range(nparts)]
        dus, drs, dts = [], [], []
        for k, sp in enumerate(sps):
            g = np.nonzero(part == k)[0][sp.permutation()]
            x = torch.full((sp.nown + sp.nghost, 4), float("nan"), dtype=torch.float64, device="cuda")
            x[:sp.nown] = torch.tensor(u[g], device="cuda")
            dus.append(x)
            drs.append(torch.empty((sp.nown, 4), dtype=torch.float64, device="cuda"))
            dts.append(torch.empty(sp.nown, dtype=torch.float64, device="cuda"))
        torch.cuda.synchronize()  # torch's stream vs the library's (non-blocking) streams
        grp = fa.FlowFVGroup(sps)
        grp.compute_residual_device([x.data_ptr() for x in dus], [x.data_ptr() for x in drs],
                                    [x.data_ptr() for x in dts], True, True)     # fills the ghost rows
        torch.cuda.synchronize()
        ranks = []
        for k, sp in enumerate(sps):
            ms, kt = timed(sp, dus[k], drs[k], dts[k], args.steps, args.preheat, True)
            st = sp.layout_stats()
            ranks.append({"rank": k, "cells": st["cells"], "ghosts": st["ghosts"], "neighbours": st["neighbours"],
                          "patches": st["patches"], "interior_patch_frac": round(st["interior_patches"] / st["patches"], 4),
                          "ms_per_residual": round(ms, 5), "kernels_ms": kt})
        grp.close()
        for sp in sps:
            sp.close()
        worst = max(r["ms_per_residual"] for r in ranks)
        print(json.dumps({"parts": nparts, "partitioner": "graph", "weights": args.weights, "partition_s": round(tp, 2),
                          "edge_cut": fa.partition_edge_cut(mesh, part),
                          "edge_cut_rcb": fa.partition_edge_cut(mesh, fa.partition_rcb(mesh, nparts)),
                          "slowest_rank_ms": worst, "mean_rank_ms": round(float(np.mean([r["ms_per_residual"] for r in ranks])), 5),
                          "compute_floor_speedup": round(t1 / worst, 3), "efficiency_floor": round(t1 / worst / nparts, 3),
                          "ranks": ranks, "numerics": args.rec}), flush=True)


if __name__ == "__main__":
    main()
