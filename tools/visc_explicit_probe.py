#!/usr/bin/env python3
"""Does the C5-family laminar case (visc-naca0012 deck numerics) have a steady state on a given member of
the family? The explicit device driver (SteadyForwardEulerSolver, aodesolver.cpp:135-282: local time
steps, forward Euler) from the free stream, first order then second order, in chunks with progress lines;
one JSON line per chunk (residual drop, min / max of the chunk's residual history).
usage: python tools/visc_explicit_probe.py [--scale 8] [--wall 1e-5] [--cfl 0.5] [--steps1 20000] [--steps2 100000]"""
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
    ap.add_argument("--scale", type=int, default=8)
    ap.add_argument("--wall", type=float, default=None)
    ap.add_argument("--cfl", type=float, default=0.5)
    ap.add_argument("--steps1", type=int, default=20000)
    ap.add_argument("--steps2", type=int, default=100000)
    ap.add_argument("--chunk", type=int, default=10000)
    ap.add_argument("--mesh", default="c5", help="c5: the C5 family (--scale, --wall); ref: the reference's "
                    "NACA0012_lam_hybrid_1.msh; cgrid-quads: the C5 C-grid without triangle rows")
    ap.add_argument("--physics", default="visc", help="visc (the deck) or naca0 (inviscid M 0.5, alpha 0)")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    if args.mesh == "ref":
        mesh, dims = fa.UMesh.read_gmsh(cases.fixture_mesh("NACA0012_lam_hybrid_1")), {"wall_spacing": "ref"}
    elif args.mesh == "cgrid-quads":             # the C5/scale C-grid with quadrangles in every row
        s = args.scale
        mesh = fa.UMesh.naca_cgrid(3072 // s, 512 // s, 1984 // s, 0, 20.0, args.wall or 1e-5)
        dims = {"topology": "C-grid, quadrangles only", "wall_spacing": args.wall or 1e-5}
    else:
        mesh, dims = c4_mesh(fa, args.scale, 2, wall=args.wall)
    if args.physics == "naca0":
        p = cases.physics("naca", Minf=0.5)
        p.aoa = 0.0
        p.bcconf = [fa.FlowBCConfig("slipwall", 2), fa.FlowBCConfig("farfield", 4)]
    else:
        p = cases.physics("visc")
    h1 = fa.FlowFV(mesh, p, cases.numerics("ROE", "NONE", "NONE", order2=False))
    h2 = fa.FlowFV(mesh, p, cases.numerics("ROE", "LEASTSQUARES", "NONE"))
    du = torch.tensor(np.tile(cases.freestream(p), (mesh.nelem, 1))[h2.permutation()], device="cuda")
    torch.cuda.synchronize()
    first = None
    for name, h, nsteps in (("first-order", h1, args.steps1), ("second-order", h2, args.steps2)):
        done = 0
        r0 = None
        while done < nsteps:
            k = min(args.chunk, nsteps - done)
            t0 = time.time()
            try:
                steps, ratio, hist = h.steady_forward_euler_device(du.data_ptr(), args.cfl, 0.0, k)
            except RuntimeError as e:
                print(json.dumps({"stage": name, "steps_before": done, "error": str(e)}), flush=True)
                break
            if r0 is None:
                r0 = float(hist[0])
            done += steps
            (cl, cdp, cdsf), _ = h2.surface_data_device(du.data_ptr(), 2)
            print(json.dumps({"stage": name, "cells": mesh.nelem, "wall": dims["wall_spacing"], "cfl": args.cfl,
                              "steps": done, "res_first": r0, "res_last": float(hist[-1]),
                              "drop": float(hist[-1]) / r0, "chunk_min": float(hist.min()), "chunk_max": float(hist.max()),
                              "CL": cl, "CDp": cdp, "CDsf": cdsf, "seconds": round(time.time() - t0, 1)}), flush=True)
            if not np.isfinite(hist[-1]):
                break
            # where the residual sits: the cells with the largest |r_energy| / area
            dr = torch.zeros((mesh.nelem, 4), dtype=torch.float64, device="cuda")
            ddt = torch.zeros(mesh.nelem, dtype=torch.float64, device="cuda")
            h.compute_residual_device(du.data_ptr(), dr.data_ptr(), ddt.data_ptr(), True, True)
            h.synchronize()
            perm = h.permutation()
            r = np.empty((mesh.nelem, 4))
            r[perm] = dr.cpu().numpy()
            q = np.abs(r[:, 3]) / mesh.area
            top = np.argsort(-q)[:6]
            print(json.dumps({"top_cells": [[int(c), float("%.3e" % q[c]), [round(float(x), 6) for x in mesh.rc[c]],
                                             float("%.2e" % mesh.area[c])] for c in top]}), flush=True)
    h1.close()
    h2.close()


if __name__ == "__main__":
    main()
