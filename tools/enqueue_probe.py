#!/usr/bin/env python3
"""Host enqueue cost of a partitioned rank's residual step against its kernel time (VERDICT r3
item 8): the C4 mesh split N ways (bench.py's cost-weighted graph partition); for each rank, its
handle on this one GPU runs tools/probes/enqueue_probe.cpp's loop -- the rank's exchange (event
record/wait, pack, one ncclGroupStart..End with a send/recv pair per neighbour of the rank's own row
counts, over a 1-rank RCCL communicator: RCCL refuses two ranks on one device) and the library's
residual launches (k_grad_ghost + fused) -- and reports host enqueue time per step against the wall
time per step (GPU-bound when the enqueue is shorter). One JSON line per rank.
usage: python tools/enqueue_probe.py [--parts 8] [--iters 200] [--build-only]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
LIB = os.path.join(ROOT, "tools", "bin", "libenqprobe.so")


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    src = os.path.join(ROOT, "tools", "probes", "enqueue_probe.cpp")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-fPIC", "-shared", "--offload-arch=gfx950", src, "-o", LIB,
                    "-L" + os.path.join(ROOT, "fvens_amd"), "-lfvhip", "-L/opt/rocm/lib", "-lrccl",
                    "-Wl,-rpath," + os.path.join(ROOT, "fvens_amd")], check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--ranks", default="", help="comma list (default all)")
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    if args.build_only or not os.path.exists(LIB):
        build()
        if args.build_only:
            return
    import torch
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    lib = ctypes.CDLL(LIB)
    mesh, _ = c4_mesh(fa, args.scale)
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    u = cases.state(mesh, p, seed=42)
    part = fa.partition_graph(mesh, args.parts, weights="cost")
    ranks = [int(x) for x in args.ranks.split(",")] if args.ranks else range(args.parts)
    for r in ranks:
        sp = fa.FlowFV(mesh, p, n, device=0, partition=part, rank=r)
        info = fa.partition_info(mesh, part, r)
        g = np.nonzero(part == r)[0][sp.permutation()]
        du = torch.zeros((sp.nown + sp.nghost, 4), dtype=torch.float64, device="cuda")
        du[:sp.nown] = torch.tensor(u[g], device="cuda")
        dr = torch.empty((sp.nown, 4), dtype=torch.float64, device="cuda")
        dt = torch.empty(sp.nown, dtype=torch.float64, device="cuda")
        ss = np.asarray(info["send_start"])
        counts = np.ascontiguousarray(np.diff(ss), np.int32)
        tot = int(counts.sum())
        sb = torch.zeros((max(tot, 1), 4), dtype=torch.float64, device="cuda")
        rb = torch.zeros((max(tot, 1), 4), dtype=torch.float64, device="cuda")
        out = np.zeros(6)
        torch.cuda.synchronize()  # torch's stream vs the library's (non-blocking) streams
        rc = lib.enq_probe(sp._h, ctypes.c_void_p(du.data_ptr()), ctypes.c_void_p(dr.data_ptr()),
                           ctypes.c_void_p(dt.data_ptr()), int(len(counts)),
                           counts.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), ctypes.c_void_p(sb.data_ptr()),
                           ctypes.c_void_p(rb.data_ptr()), int(args.iters),
                           out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        if rc != 0:
            raise SystemExit("enq_probe failed with %d" % rc)
        print(json.dumps({"rank": r, "parts": args.parts, "cells": sp.nown, "ghosts": sp.nghost,
                          "neighbours": int(len(counts)), "send_rows": tot, "iters": args.iters,
                          "full_step": {"host_enqueue_us": round(out[0], 2), "wall_us": round(out[1], 2)},
                          "residual_only": {"host_enqueue_us": round(out[2], 2), "wall_us": round(out[3], 2)},
                          "exchange_only": {"host_enqueue_us": round(out[4], 2), "wall_us": round(out[5], 2)},
                          "host_bound": bool(out[0] > out[1] * 0.9)}), flush=True)
        sp.close()


if __name__ == "__main__":
    main()
