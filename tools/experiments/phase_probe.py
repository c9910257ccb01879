#!/usr/bin/env python3
"""Where a fused-residual block's lifetime goes (diagnostic; needs the -DFVHIP_PROBE_PHASES build):
    make -C fvens_amd OBJDIR=build_probe LIB=build_probe/libfvhip_probe.so EXTRA=-DFVHIP_PROBE_PHASES
    FVHIP_LIB=fvens_amd/build_probe/libfvhip_probe.so python tools/phase_probe.py [--scale S] [--rec VANALBADA]
Thread 0 of every block stamps the 100 MHz real-time counter at the kernel's phase boundaries
(start, staging barrier, gradient barrier, end of the face work, flux-staging barrier, end) and the
shader clock at start and end; the last launch's stamps are written at handle destruction and
summarised here: mean phase durations, block lifetime, blocks resident over time, clock."""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--rec", default="VANALBADA")
    ap.add_argument("--visc", action="store_true")
    ap.add_argument("--steps", type=int, default=1500)
    args = ap.parse_args()
    import torch
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    out = os.path.join(tempfile.gettempdir(), "fz_probe.bin")
    os.environ["FVHIP_PROBE_OUT"] = out
    mesh, dims = c4_mesh(fa, args.scale)
    p = cases.physics("visc" if args.visc else "naca")
    n = cases.numerics("ROE", "LEASTSQUARES", args.rec)
    u = cases.state(mesh, p, seed=42)
    sp = fa.FlowFV(mesh, p, n, device=0)
    du = torch.tensor(u[sp.permutation()], device="cuda")
    dr = torch.empty((mesh.nelem, 4), dtype=torch.float64, device="cuda")
    dt = torch.empty(mesh.nelem, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    for _ in range(args.steps):
        sp.compute_residual_device(du.data_ptr(), dr.data_ptr(), dt.data_ptr(), True, True)
    sp.synchronize()
    st = sp.layout_stats()
    sp.close()
    a = np.fromfile(out, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
    a = a[a[:, 0] > 0]
    rt = a[:, :6] - a[:, 0:1]
    ph = np.diff(a[:, :6], axis=1) * 10.0 / 1000.0             # us (100 MHz ticks)
    life = rt[:, 5] * 10.0 / 1000.0
    span = (a[:, 5].max() - a[:, 0].min()) * 10.0 / 1000.0
    clk = (a[:, 7] - a[:, 6]) / np.maximum(a[:, 5] - a[:, 0], 1) * 100e6
    # blocks resident over the launch, sampled every 0.1 us
    t0 = a[:, 0].min()
    s = (a[:, 0] - t0).astype(np.int64)
    e = (a[:, 5] - t0).astype(np.int64)
    ev = np.zeros(int(e.max()) + 2, np.int64)
    np.add.at(ev, s, 1)
    np.add.at(ev, e, -1)
    res = np.cumsum(ev)[:-1]
    names = ["staging", "gradients", "faces", "flux_stage", "scatter"]
    d = {"blocks": int(len(a)), "cells": st["cells"], "launch_span_us": round(span, 2),
         "block_life_us": {"mean": round(float(life.mean()), 3), "p10": round(float(np.percentile(life, 10)), 3),
                           "p90": round(float(np.percentile(life, 90)), 3)},
         "phase_us_mean": {k: round(float(ph[:, i].mean()), 3) for i, k in enumerate(names)},
         "phase_frac": {k: round(float(ph[:, i].mean() / life.mean()), 3) for i, k in enumerate(names)},
         "resident_blocks_mean": round(float(res.mean()), 1), "resident_blocks_max": int(res.max()),
         "clock_GHz_median": round(float(np.median(clk)) / 1e9, 3),
         "first_start_to_last_start_us": round(float((a[:, 0].max() - t0) * 10.0 / 1000.0), 2),
         "tail_us": round(float((a[:, 5].max() - a[:, 0].max()) * 10.0 / 1000.0), 2)}
    print(json.dumps(d))


if __name__ == "__main__":
    main()
