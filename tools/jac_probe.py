#!/usr/bin/env python3
"""Probe: the C4 Jacobian assembly (k_jac_interior / k_jac_boundary / k_jac_diag) launched `reps`
times on a perturbed state, with the library's HIP-event kernel times; for rocprofv3 trace and PMC
passes of the assembly kernels.
usage: python tools/jac_probe.py [--reps R] [--scale S] [--case naca|visc-c5]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--case", default="naca", choices=["naca", "visc-c5"])
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    mesh, dims = c4_mesh(fa, args.scale, 2 if args.case == "visc-c5" else 1)
    kind = "visc" if args.case == "visc-c5" else "naca"
    p = cases.physics(kind)
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    sp = fa.FlowFV(mesh, p, n, device=0)
    perm = sp.permutation()
    u = cases.state(mesh, p, seed=42)[perm]
    N, Fi = mesh.nelem, mesh.ninface
    du = torch.tensor(u, dtype=torch.float64, device="cuda")
    dd = torch.empty((N, 16), dtype=torch.float64, device="cuda")
    dl = torch.empty((max(Fi, 1), 16), dtype=torch.float64, device="cuda")
    dup = torch.empty((max(Fi, 1), 16), dtype=torch.float64, device="cuda")
    for _ in range(5):
        sp.assemble_jacobian_device(du.data_ptr(), dd.data_ptr(), dl.data_ptr(), dup.data_ptr())
    sp.synchronize()
    sp.profile(True)
    for _ in range(args.reps):
        sp.assemble_jacobian_device(du.data_ptr(), dd.data_ptr(), dl.data_ptr(), dup.data_ptr())
    kt = sp.kernel_times()
    sp.profile(False)
    sp.synchronize()
    ms = {k: round(v[0] / args.reps, 5) for k, v in kt.items()}
    rb = 32 * mesh.naface + 32 * N          # state of both cells + face geometry read
    wb = 128 * (N + 2 * Fi)
    out = {"case": args.case, "cells": N, "interior_faces": Fi, "reps": args.reps, "kernels_ms": ms}
    ki = [k for k in ms if k.startswith("k_jac_interior")]
    if ki:
        fb = Fi * (96 + 256)
        out["k_jac_interior_algorithmic_bytes"] = fb
        out["k_jac_interior_GBs"] = round(fb / (ms[ki[0]] * 1e-3) / 1e9, 1)
    out["assembly_bytes"] = rb + wb
    print(json.dumps(out), flush=True)
    sp.close()


if __name__ == "__main__":
    main()
