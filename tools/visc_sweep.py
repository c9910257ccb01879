#!/usr/bin/env python3
"""Schedules of the C5-family convergence run (tools/visc_converge.run) tried one after the other in one
process: one JSON line per variant with both stages' step counts, linear-solve outcomes, residual
histories (every 10th) and, for a finished main solve, CL / CDp / CDsf.
usage: python tools/visc_sweep.py SCALE '<json list of run() keyword dicts>'"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    scale = int(sys.argv[1])
    variants = json.loads(sys.argv[2])
    import torch
    torch.cuda.set_device(0)
    from visc_converge import run
    for kw in variants:
        t0 = time.time()
        r = run(scale=scale, heartbeat=lambda s: print(s, flush=True), **kw)
        out = {"variant": kw, "cells": r["cells"], "seconds": round(time.time() - t0, 1)}
        for st in ("init", "main"):
            if st in r:
                s = r[st]
                h = s.get("history", [])
                out[st] = {k: s.get(k) for k in ("steps", "converged", "resratio", "lin_iters", "lin_unconverged",
                                                 "lin_worst", "cfl", "error", "ms_per_step")}
                out[st]["hist"] = [float("%.3e" % x) for x in h[::10]] + ([float("%.3e" % h[-1])] if h else [])
        for k in ("CL", "CDp", "CDsf"):
            if k in r:
                out[k] = r[k]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
