#!/usr/bin/env python3
"""Converged implicit solve of the C4 configuration (NACA0012 O-grid, M 0.8, 1.25 deg,
Roe + WLS + MUSCL/Van Albada, implicit with point-block Jacobi on the assembled first-order Jacobian):
the reference's two-stage start (transonic-implicit.ctrl: first-order initialisation, then the
second-order main solve, casesolvers.cpp:225-314) on the device drivers. Prints per stage the steps,
the residual history (every ~1/15), the drop from the stage's first residual and from its peak, and
the wall time; the last line is a JSON summary.

usage: python tools/c4_converge.py [--scale S] [--wall W] [--init-flux ROE|LLF] ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np


def converge(scale=1, wall=None, init_flux="ROE", init_steps=600, init_cfl=(5.0, 200.0), main_cfl=(5.0, 200.0),
             main_tol=1e-6, main_steps=3000, rec="VANALBADA", lin_maxit=40, sweeps=1, min_relax=0.2, verbose=True,
             lines=False, init_tol=0.0, lin_rtol=1e-2):
    import torch
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    mesh, dims = c4_mesh(fa, scale, wall=wall)
    p = cases.physics("naca")
    n1 = cases.numerics(init_flux, "NONE", "NONE", order2=False)
    n2 = cases.numerics("ROE", "LEASTSQUARES", rec)
    dev = torch.cuda.current_device()
    sp1, sp2 = fa.FlowFV(mesh, p, n1, device=dev), fa.FlowFV(mesh, p, n2, device=dev)
    perm = sp2.permutation()
    du = torch.tensor(np.tile(cases.freestream(p), (mesh.nelem, 1))[perm], device="cuda")
    lin = dict(lin_rtol=lin_rtol, lin_maxit=lin_maxit, restart=lin_maxit, prec_sweeps=sweeps, min_relax=min_relax,
               prec_lines=lines)
    out = {"cells": mesh.nelem, "dims": dims, "wall_spacing": wall, "stages": []}
    for name, sp, cfl, tol, nit in (("init", sp1, init_cfl, init_tol, init_steps), ("main", sp2, main_cfl, main_tol, main_steps)):
        if nit <= 0:
            continue
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st, hist = sp.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(
            cflinit=cfl[0], cflfin=cfl[1], tol=tol, maxiter=nit, **lin))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        h = np.asarray(hist[:st["steps"]])
        k = int(np.argmax(h))
        rec_ = {"stage": name, "flux": sp is sp1 and init_flux or "ROE", "steps": st["steps"],
                "converged": bool(st["converged"]), "resratio": st["resratio"], "first": float(h[0]),
                "peak": float(h[k]), "peak_step": k, "last": float(h[-1]), "drop_from_peak": float(h[-1] / h[k]),
                "cfl": list(cfl), "cfl_end": st["cfl"], "lin_iters_per_step": round(st["lin_iters"] / max(1, st["steps"]), 2),
                "seconds": round(dt, 2), "ms_per_step": round(1e3 * dt / max(1, st["steps"]), 2)}
        out["stages"].append(rec_)
        if verbose:
            print(name, json.dumps(rec_), flush=True)
            print("   hist", " ".join("%.2e" % x for x in h[::max(1, len(h) // 15)]), flush=True)
    (cl, cdp, cdsf), _ = sp2.surface_data_device(du.data_ptr(), 2)
    out["CL"], out["CDp"] = cl, cdp
    sp1.close(); sp2.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--wall", type=float, default=None, help="wall spacing (default: bench.py's C4)")
    ap.add_argument("--init-flux", default="ROE")
    ap.add_argument("--init-steps", type=int, default=600)
    ap.add_argument("--main-steps", type=int, default=3000)
    ap.add_argument("--main-cfl", type=float, nargs=2, default=(5.0, 200.0))
    ap.add_argument("--init-cfl", type=float, nargs=2, default=(5.0, 200.0))
    ap.add_argument("--rec", default="VANALBADA")
    ap.add_argument("--sweeps", type=int, default=1)
    ap.add_argument("--lines", action="store_true", help="line-implicit preconditioner")
    ap.add_argument("--lin-maxit", type=int, default=40)
    ap.add_argument("--lin-rtol", type=float, default=1e-2)
    ap.add_argument("--init-tol", type=float, default=0.0, help="stop the first-order stage at this residual ratio")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    r = converge(args.scale, args.wall, args.init_flux, args.init_steps, tuple(args.init_cfl), tuple(args.main_cfl),
                 1e-6, args.main_steps, args.rec, lin_maxit=args.lin_maxit, sweeps=args.sweeps, lines=args.lines,
                 init_tol=args.init_tol, lin_rtol=args.lin_rtol)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
