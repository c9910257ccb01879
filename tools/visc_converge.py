#!/usr/bin/env python3
"""BASELINE config 5 solved to the visc-naca0012 deck's tolerance on the C5 family (the quadrangle C-grid of
bench.c4_mesh; --quads: the same grid built here) with the device
solver: testcases/visc-naca0012/laminar-implicit.ctrl's schedule -- first-order initialisation (CFL 200 ->
1000, tolerance 1e-1, 50 steps), then the second-order main solve (Roe, least squares, limiter none,
Sutherland; CFL 500 -> 5000 by expResidualRamp, tolerance 1e-6), 'full' nonlinear update -- with the
matrix-free operator (BASELINE config 5) or the assembled one, preconditioned by the line-implicit
preconditioner on the assembled first-order Jacobian (the deck's bjacobi/ILU), GMRES rtol 1e-1.
Prints a heartbeat while the device runs, then one JSON line: the stages' steps, linear iterations,
residual histories, wall times, and CL / CDp / CDsf on the wall (marker 2).
usage: python tools/visc_converge.py [--scale S] [--assembled] [--main-steps N] [--lin-maxit K]"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

T0 = time.time()

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(scale=1, matrix_free=True, main_steps=400, init_steps=50, lin_maxit=60, restart=60, sweeps=3,
        tol=1e-6, heartbeat=None, cfl_init=(200.0, 1000.0), cfl_main=(500.0, 5000.0), min_relax=1.0, lin_rtol=1e-1,
        wall=None, mf_eps=None, quads=False, amg=0, amg_sweeps=2, amg_coarse=6, amg_thr=0.2, lines=True, amg_fine=0, single=False,
        u0=None, want_state=False, chunk=0, deadline=None, symmetrize=False):
    """the deck's two stages on the C5 mesh divided by `scale` in both directions; returns the record (a stage
    that diverges is recorded with its history and the error; the later stage is then skipped). u0: a start
    state in the mesh's cell order (mesh sequencing: a coarser member's solution carried over) -- the main
    stage then starts from it, without the first-order stage; want_state: the final state (cell order) and
    the cell centres go into rec["_state"], rec["_rc"]. chunk > 0: the main stage runs in pieces of `chunk`
    steps, each a fresh call resumed from the last one's residuals and CFL (fvhip_implicit_config resume_*: the
    same iterates as one call), so that it can stop at the wall-clock `deadline` (time.time()) with its record.
    symmetrize (with chunk > 0): between chunks the state is projected onto the mirror-symmetric states of the
    (exactly mirrored) hybrid mesh, u <- (u + S u)/2 with S the reflection y -> -y (rho v negated); the deck's
    flow is at alpha 0, so its steady state is symmetric, and the projection removes the antisymmetric mode that
    the unprojected pseudo-time iteration grows at the full size. The record carries the
    antisymmetric part's norm removed by each projection"""
    import torch
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    if symmetrize and chunk <= 0:
        raise ValueError("symmetrize projects between chunks: chunk must be > 0")
    mesh, dims = c4_mesh(fa, scale, 2, wall=wall, topology="cgrid" if quads else "hybrid")
    p = cases.physics("visc")                                   # alpha 0 (laminar-implicit.ctrl:19)
    n1 = cases.numerics("ROE", "NONE", "NONE", order2=False)
    n2 = cases.numerics("ROE", "LEASTSQUARES", "NONE")          # limiter none (:72)
    start, main = fa.FlowFV(mesh, p, n1), fa.FlowFV(mesh, p, n2)
    perm = main.permutation()
    if mf_eps:
        main.matfree_set_eps(mf_eps)          # -matrix_free_difference_step (alinalg.cpp:127)
    ustart = np.tile(cases.freestream(p), (mesh.nelem, 1)) if u0 is None else np.asarray(u0, np.float64)
    if u0 is not None:
        init_steps = 0
    du = torch.tensor(ustart[perm], device="cuda")
    if symmetrize:
        mir = mirror_map(np.asarray(mesh.rc[:mesh.nelem]))
        inv = np.empty_like(perm)
        inv[perm] = np.arange(len(perm))
        dmir = torch.tensor(inv[mir[perm]], device="cuda")     # device row of each device row's mirror cell
        sgn = torch.tensor([1.0, 1.0, -1.0, 1.0], device="cuda", dtype=torch.float64)
    torch.cuda.synchronize()      # torch's stream vs the library's (non-blocking) streams
    lin = dict(lin_rtol=lin_rtol, lin_maxit=lin_maxit, restart=restart, prec_lines=lines, prec_sweeps=sweeps,
               min_relax=min_relax, prec_amg=amg, amg_sweeps=amg_sweeps, amg_coarse_sweeps=amg_coarse,
               amg_threshold=amg_thr, amg_fine_sweeps=amg_fine, prec_single=single)
    rec = {"library": fa._ffi.build_info()["lib_src_hash"], "cells": mesh.nelem, "faces": mesh.naface, "dims": dims, "operator": "matrix-free" if matrix_free else "assembled",
           "linear": dict(lin, gmres="GMRES(%d) right-preconditioned" % restart), "cfl_init": list(cfl_init),
           "cfl_main": list(cfl_main)}
    done = threading.Event()

    def beat():
        t0 = time.time()
        while not done.wait(20.0):
            if heartbeat:
                heartbeat("running %.0f s" % (time.time() - t0))
    th = threading.Thread(target=beat, daemon=True)
    th.start()
    def stage(h, cfg):
        t0 = time.perf_counter()
        try:
            st, hh = h.steady_backward_euler_device(du.data_ptr(), cfg)
            torch.cuda.synchronize()
            return {**st, "seconds": round(time.perf_counter() - t0, 2),
                    "ms_per_step": round((time.perf_counter() - t0) / max(st["steps"], 1) * 1e3, 2),
                    "history": [float(x) for x in hh]}
        except RuntimeError as e:
            hh = getattr(e, "history", [])
            return {"error": str(e), "steps": len(hh), "converged": False, "seconds": round(time.perf_counter() - t0, 2),
                    "history": [float(x) for x in hh]}
    try:
        if init_steps > 0:
            rec["init"] = stage(start, fa.ImplicitConfig(cflinit=cfl_init[0], cflfin=cfl_init[1], tol=1e-1,
                                                        maxiter=init_steps, **lin))
        if "error" not in rec.get("init", {}) and chunk <= 0:
            rec["main"] = stage(main, fa.ImplicitConfig(cflinit=cfl_main[0], cflfin=cfl_main[1], tol=tol,
                                                        maxiter=main_steps, matrix_free=matrix_free, **lin))
        elif "error" not in rec.get("init", {}):
            agg = {"steps": 0, "lin_iters": 0, "lin_unconverged": 0, "lin_worst": 0.0, "seconds": 0.0, "history": [],
                   "chunks": 0, "converged": False}
            if symmetrize:
                agg["antisym_removed"] = []
            t_stage = time.perf_counter()
            while agg["steps"] < main_steps:
                hh = agg["history"]
                res = None if len(hh) < 2 else (hh[0], hh[-1], hh[-2], agg["cfl"])
                n = min(chunk, main_steps - agg["steps"])
                st = stage(main, fa.ImplicitConfig(cflinit=cfl_main[0], cflfin=cfl_main[1], tol=tol, maxiter=n,
                                                   matrix_free=matrix_free, resume=res, **lin))
                agg["chunks"] += 1
                agg["history"] = hh + st["history"]
                for k in ("steps", "lin_iters", "lin_unconverged"):
                    agg[k] += st.get(k, 0)
                agg["lin_worst"] = max(agg["lin_worst"], st.get("lin_worst", 0.0))
                agg["cfl"] = st.get("cfl", agg.get("cfl"))
                if "error" in st:
                    agg["error"] = st["error"]
                    break
                agg["resratio"] = agg["history"][-1] / agg["history"][0]
                if heartbeat:
                    heartbeat("main: %d steps, resratio %.3e, %.0f s" % (agg["steps"], agg["resratio"],
                                                                         time.perf_counter() - t_stage))
                if st["converged"]:
                    agg["converged"] = True
                    break
                if deadline is not None and time.time() + 1.5*st["seconds"]*chunk/max(n, 1) > deadline:
                    agg["stopped"] = "wall-clock deadline"
                    break
                if symmetrize:
                    us = du[dmir] * sgn
                    agg["antisym_removed"].append(float((0.5*(du - us)).norm() / du.norm()))
                    du.copy_(0.5*(du + us))
                    torch.cuda.synchronize()
            agg["seconds"] = round(time.perf_counter() - t_stage, 2)
            agg["ms_per_step"] = round(agg["seconds"]/max(agg["steps"], 1)*1e3, 2)
            rec["main"] = agg
    finally:
        done.set()
    if "main" not in rec or "error" in rec["main"]:
        start.close()
        main.close()
        rec["finite"] = False
        return rec
    (cl, cdp, cdsf), _ = main.surface_data_device(du.data_ptr(), 2)
    finite = bool(torch.isfinite(du).all().item())
    if want_state:
        us = np.empty((mesh.nelem, 4))
        us[perm] = du.cpu().numpy()
        rec["_state"], rec["_rc"] = us, np.asarray(mesh.rc[:mesh.nelem]).copy()
    start.close()
    main.close()
    rec.update({"CL": cl, "CDp": cdp, "CDsf": cdsf, "finite": finite})
    return rec


def mirror_map(rc):
    """the mirror cell (y -> -y) of every cell of a mirror-symmetric mesh, by its centre; an involution
    without fixed points, checked"""
    from scipy.spatial import cKDTree
    d, mir = cKDTree(rc).query(rc * np.array([1.0, -1.0]), workers=16)
    scale = np.abs(rc).max()
    assert d.max() <= 1e-12 * scale, "the mesh is not mirror-symmetric (%g)" % d.max()
    assert (mir[mir] == np.arange(len(rc))).all() and (mir != np.arange(len(rc))).all()
    return mir


def carry_over(rc_from, u_from, rc_to):
    """mesh sequencing: each cell of the finer mesh takes the state of the coarser mesh's cell whose centre is
    nearest to its own (piecewise-constant prolongation; the meshes share their geometry, not their cells)"""
    from scipy.spatial import cKDTree
    _, idx = cKDTree(rc_from).query(rc_to, workers=16)
    return u_from[idx]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--assembled", action="store_true")
    ap.add_argument("--main-steps", type=int, default=400)
    ap.add_argument("--init-steps", type=int, default=50, help="0: no first-order start (main from the free stream)")
    ap.add_argument("--lin-maxit", type=int, default=60)
    ap.add_argument("--restart", type=int, default=60)
    ap.add_argument("--sweeps", type=int, default=3)
    ap.add_argument("--cfl-init", type=float, nargs=2, default=(200.0, 1000.0))
    ap.add_argument("--cfl-main", type=float, nargs=2, default=(500.0, 5000.0))
    ap.add_argument("--min-relax", type=float, default=1.0, help=">= 1: full update (the deck), else robust_flow")
    ap.add_argument("--lin-rtol", type=float, default=1e-1)
    ap.add_argument("--wall", type=float, default=None, help="first-cell wall spacing (default: the C5 mesh's 1e-5)")
    ap.add_argument("--quads", action="store_true", help="round 5's quadrangle C-grid instead of the hybrid mesh")
    ap.add_argument("--mf-eps", type=float, default=None, help="matrix-free difference step (default 1e-7)")
    ap.add_argument("--amg", type=int, default=0, help="aggregation multigrid levels (0: the one-level preconditioner)")
    ap.add_argument("--amg-sweeps", type=int, default=2)
    ap.add_argument("--amg-coarse", type=int, default=6)
    ap.add_argument("--amg-thr", type=float, default=0.2)
    ap.add_argument("--amg-fine", type=int, default=0, help="finest-level sweeps (0: --amg-sweeps)")
    ap.add_argument("--single", action="store_true", help="preconditioner blocks / line factors in fp32 (prec_single)")
    ap.add_argument("--no-lines", action="store_true", help="point-block Jacobi instead of the line-implicit preconditioner")
    ap.add_argument("--sequence", type=int, nargs="+", default=None,
                    help="mesh sequencing: solve these scales in turn (coarsest first, the deck's schedule), each finer "
                         "one starting from the previous solution carried over (no first-order stage); the last is --scale")
    ap.add_argument("--save-state", default=None, help="with --sequence: the last stage's converged state to this "
                    ".npz (compressed, float64, the mesh's cell order)")
    ap.add_argument("--load-state", default=None, help="with --sequence: start the first stage from this .npz "
                    "(carried over to its mesh) instead of the deck's first-order stage")
    ap.add_argument("--load-scale", type=int, default=None, help="the member (scale) the loaded state belongs to")
    ap.add_argument("--final-lin-rtol", type=float, default=None, help="with --sequence: the last stage's linear tolerance")
    ap.add_argument("--final-lin-maxit", type=int, default=None, help="with --sequence: the last stage's GMRES "
                    "iteration cap and restart length")
    ap.add_argument("--final-cfl-main", type=float, nargs=2, default=None, help="with --sequence: the last stage's CFL "
                    "ramp (start, cap)")
    ap.add_argument("--final-amg-sweeps", type=int, nargs=2, default=None, help="with --sequence: the last stage's "
                    "multigrid sweeps per level and coarsest-level sweeps")
    ap.add_argument("--chunk", type=int, default=0, help="run the main stage in resumed pieces of this many steps")
    ap.add_argument("--deadline", type=float, default=None, help="seconds from start after which a chunked main "
                    "stage stops (and its record is printed)")
    ap.add_argument("--symmetrize", action="store_true", help="with --chunk: project the state onto the "
                    "mirror-symmetric states between chunks (alpha 0)")
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    if args.symmetrize and args.chunk <= 0:
        ap.error("--symmetrize projects between chunks: give --chunk")
    import torch
    torch.cuda.set_device(0)
    if args.sequence:
        import fvens_amd as fa
        from bench import c4_mesh
        u0, prev, recs = None, None, []
        if args.load_state:
            z = np.load(args.load_state)
            mz, _ = c4_mesh(fa, args.load_scale, 2, wall=args.wall, topology="cgrid" if args.quads else "hybrid")
            prev = {"_state": z["u"], "_rc": np.asarray(mz.rc[:mz.nelem]).copy()}
            assert prev["_state"].shape == (mz.nelem, 4), "the loaded state is not of that member"
            del mz
        for sc in args.sequence:
            kw = dict(matrix_free=not args.assembled, main_steps=args.main_steps, init_steps=args.init_steps,
                      lin_maxit=args.lin_maxit, restart=args.restart, sweeps=args.sweeps,
                      heartbeat=lambda s: print(s, flush=True), cfl_init=args.cfl_init, cfl_main=args.cfl_main,
                      min_relax=args.min_relax, lin_rtol=args.lin_rtol, wall=args.wall, mf_eps=args.mf_eps,
                      quads=args.quads, amg=args.amg, amg_sweeps=args.amg_sweeps, amg_coarse=args.amg_coarse,
                      amg_thr=args.amg_thr, lines=not args.no_lines, amg_fine=args.amg_fine, single=args.single,
                      chunk=args.chunk, symmetrize=args.symmetrize and sc == args.sequence[-1],
                      deadline=None if args.deadline is None else T0 + args.deadline)
            if sc == args.sequence[-1] and args.final_lin_rtol:
                kw["lin_rtol"] = args.final_lin_rtol
            if sc == args.sequence[-1] and args.final_cfl_main:
                kw["cfl_main"] = tuple(args.final_cfl_main)
            if sc == args.sequence[-1] and args.final_amg_sweeps:
                kw["amg_sweeps"], kw["amg_coarse"] = args.final_amg_sweeps
            if sc == args.sequence[-1] and args.final_lin_maxit:
                kw["lin_maxit"] = kw["restart"] = args.final_lin_maxit
            if prev is not None:
                m, _ = c4_mesh(fa, sc, 2, wall=args.wall, topology="cgrid" if args.quads else "hybrid")
                u0 = carry_over(prev["_rc"], prev["_state"], np.asarray(m.rc[:m.nelem]))
                del m
            r = run(sc, u0=u0, want_state=True, **kw)
            prev = r
            out = {k: v for k, v in r.items() if not k.startswith("_")}
            out["tag"], out["sequence_scale"] = args.tag, sc
            print(json.dumps(out), flush=True)
            if not r.get("main", {}).get("converged"):
                break
        if args.save_state and prev is not None and "_state" in prev:
            np.savez_compressed(args.save_state, u=prev["_state"])
            print(json.dumps({"saved": args.save_state, "bytes": os.path.getsize(args.save_state)}), flush=True)
        return
    r = run(args.scale, not args.assembled, args.main_steps, init_steps=args.init_steps, lin_maxit=args.lin_maxit, restart=args.restart,
            sweeps=args.sweeps, heartbeat=lambda s: print(s, flush=True), cfl_init=args.cfl_init,
            cfl_main=args.cfl_main, min_relax=args.min_relax, lin_rtol=args.lin_rtol, wall=args.wall, mf_eps=args.mf_eps, quads=args.quads,
            amg=args.amg, amg_sweeps=args.amg_sweeps, amg_coarse=args.amg_coarse, amg_thr=args.amg_thr,
            lines=not args.no_lines, amg_fine=args.amg_fine, single=args.single, chunk=args.chunk,
            symmetrize=args.symmetrize, deadline=None if args.deadline is None else T0 + args.deadline)
    r["tag"] = args.tag
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
