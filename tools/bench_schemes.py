#!/usr/bin/env python3
"""Secondary benchmark: device residual (compute_residual with local time steps) for the scheme
combinations of BASELINE.json's configs on one MI355X, each on its own synthetic mesh:

  C2/C4 NACA0012 O-grid (bench.py's generator) -- Roe + WLS + MUSCL/Van Albada (the headline path),
        Roe + WLS + Venkatakrishnan (config 4), Roe + WLS + unlimited linear, HLLC + Green-Gauss +
        Barth-Jespersen, first-order LLF;
  flat plate (config 3) -- laminar, HLLC + WLS + unlimited linear + Sutherland viscous flux;
  laminar NACA0012 on the O-grid -- Roe + WLS + Van Albada + viscous (config 5 itself, on its C-grid with the
  deck's unlimited reconstruction: bench.py --numerics config5).

Prints one JSON line per case: ms per residual, Gfaces/s, the kernels and their per-call times.
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

CASES = [  # name, mesh kind, physics, flux, gradients, reconstruction
    ("roe-wls-muscl", "naca", "naca", "ROE", "LEASTSQUARES", "VANALBADA"),
    ("roe-wls-venkatakrishnan", "naca", "naca", "ROE", "LEASTSQUARES", "VENKATAKRISHNAN"),
    ("roe-wls-linear", "naca", "naca", "ROE", "LEASTSQUARES", "NONE"),
    ("hllc-gg-barthjespersen", "naca", "naca", "HLLC", "GREENGAUSS", "BARTHJESPERSEN"),
    ("llf-first-order", "naca", "naca", "LLF", "NONE", "NONE"),
    ("roe-wls-muscl-viscous", "naca", "visc", "ROE", "LEASTSQUARES", "VANALBADA"),
    ("plate-hllc-wls-viscous", "plate", "plate", "HLLC", "LEASTSQUARES", "NONE"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=1, help="divide the mesh dimensions by this")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--only", default=None, help="comma-separated case names")
    ap.add_argument("--staged", action="store_true", help="force the staged (gradient + sweep) path")
    args = ap.parse_args()

    import torch
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from bench import c4_mesh

    meshes = {}
    for name, mk, phys, flux, grad, rec in CASES:
        if args.only and name not in args.only.split(","):
            continue
        if mk not in meshes:
            if mk == "plate":
                nx = 2048 // args.scale
                meshes[mk] = (fa.UMesh.flat_plate(nx, nx // 2), dict(nx=nx, ny=nx // 2))
            else:
                meshes[mk] = c4_mesh(fa, args.scale)
        mesh, dims = meshes[mk]
        p = cases.physics(phys)
        n = cases.numerics(flux, grad, rec, order2=grad != "NONE")
        sp = fa.FlowFV(mesh, p, n, device=0)
        perm = sp.permutation()
        u = cases.state(mesh, p, seed=42)[perm]
        du = torch.tensor(np.ascontiguousarray(u), device="cuda")
        dr = torch.empty_like(du)
        ddt = torch.empty(mesh.nelem, dtype=torch.float64, device="cuda")

        def step():
            sp.compute_residual_device(du.data_ptr(), dr.data_ptr(), ddt.data_ptr(), True, True, staged=args.staged)
        for _ in range(args.warmup):
            step()
        sp.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        sp.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
        sp.profile(True)
        for _ in range(args.steps):
            step()
        kt = sp.kernel_times()
        sp.profile(False)
        sp.close()
        print(json.dumps({"case": name, "path": "staged" if args.staged else "default", "cells": mesh.nelem, "faces": mesh.naface, "dims": dims,
                          "ms_per_residual": round(ms, 4), "gfaces_per_s": round(mesh.naface / (ms * 1e-3) / 1e9, 2),
                          "kernels_ms": {k: round(v[0] / args.steps, 4) for k, v in kt.items()}}), flush=True)


if __name__ == "__main__":
    main()
