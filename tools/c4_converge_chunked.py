#!/usr/bin/env python3
"""Full-size C4 implicit convergence run with progress output: the device backward-Euler driver called
in chunks of --chunk steps, each chunk starting at the CFL the previous one reached (the reference's
expResidualRamp, aodesolver.cpp:110-120, carried across chunks), first-order initialisation then the
second-order main solve; prints one line per chunk and a JSON summary per stage."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--wall", type=float, default=None)
    ap.add_argument("--init-flux", default="LLF")
    ap.add_argument("--init-steps", type=int, default=3000)
    ap.add_argument("--init-drop", type=float, default=1e-6, help="stop the first stage at this drop from its peak")
    ap.add_argument("--main-steps", type=int, default=1000)
    ap.add_argument("--chunk", type=int, default=100)
    ap.add_argument("--cfl", type=float, nargs=2, default=(5.0, 200.0))
    ap.add_argument("--rec", default="VANALBADA")
    ap.add_argument("--seconds", type=float, default=800.0, help="wall-time budget")
    ap.add_argument("--lines", action="store_true", help="line-implicit preconditioner")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    mesh, dims = c4_mesh(fa, args.scale, wall=args.wall)
    p = cases.physics("naca")
    sp1 = fa.FlowFV(mesh, p, cases.numerics(args.init_flux, "NONE", "NONE", order2=False))
    sp2 = fa.FlowFV(mesh, p, cases.numerics("ROE", "LEASTSQUARES", args.rec))
    du = torch.tensor(np.tile(cases.freestream(p), (mesh.nelem, 1))[sp2.permutation()], device="cuda")
    torch.cuda.synchronize()      # torch's stream vs the library's (non-blocking) streams
    lin = dict(lin_rtol=1e-2, lin_maxit=40, restart=40, prec_sweeps=1, min_relax=0.2, prec_lines=args.lines)
    print("cells", mesh.nelem, dims, flush=True)
    t_start = time.perf_counter()
    summary = []
    for name, sp, nmax in (("init", sp1, args.init_steps), ("main", sp2, args.main_steps)):
        if nmax <= 0:
            continue
        cfl = args.cfl[0]
        hist_all = []
        t0 = time.perf_counter()
        lin_its = 0
        while len(hist_all) < nmax and time.perf_counter() - t_start < args.seconds:
            st, h = sp.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(
                cflinit=cfl, cflfin=args.cfl[1], tol=0.0, maxiter=args.chunk, **lin))
            cfl = st["cfl"]
            lin_its += st["lin_iters"]
            hist_all.extend(h[:st["steps"]].tolist())
            hh = np.asarray(hist_all)
            pk = hh.max()
            print(f"{name} steps {len(hh)} res {hh[-1]:.3e} peak {pk:.3e} drop {hh[-1]/pk:.2e} cfl {cfl:.1f} "
                  f"lin/step {st['lin_iters']/max(1,st['steps']):.1f} {time.perf_counter()-t0:.1f}s", flush=True)
            if name == "init" and len(hh) > 50 and hh[-1] / pk <= args.init_drop:
                break
        torch.cuda.synchronize()
        hh = np.asarray(hist_all)
        dt = time.perf_counter() - t0
        rec = {"stage": name, "steps": len(hh), "first": hh[0], "peak": hh.max(), "last": hh[-1],
               "drop_from_first": hh[-1] / hh[0], "drop_from_peak": hh[-1] / hh.max(), "cfl_end": cfl,
               "seconds": round(dt, 1), "ms_per_step": round(1e3 * dt / max(1, len(hh)), 2),
               "lin_iters_per_step": round(lin_its / max(1, len(hh)), 2)}
        summary.append(rec)
        print(name, json.dumps(rec), flush=True)
    (cl, cdp, _), _ = sp2.surface_data_device(du.data_ptr(), 2)
    print(json.dumps({"cells": mesh.nelem, "dims": dims, "stages": summary, "CL": cl, "CDp": cdp}), flush=True)
    sp1.close(); sp2.close()


if __name__ == "__main__":
    main()
