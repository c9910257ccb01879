#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of bench.py over the TIMED window only.

bench.py's primary path dispatches its fused residual: warm-up steps, the pre-heat burst, the `steps`
timed steps, then `steps` more under HIP-event profiling. So the timed region is the kernel's
dispatches [-2*steps, -steps) of its last run. Reads <dir>/run_kernel_trace.csv (rocprofv3
--kernel-trace --output-format csv), prints one JSON object: per-window mean / median / min / max / p90
of the duration, the whole-run average (what --stats reports), and the dispatch gaps.
usage: python tools/trace_window.py <trace dir> <steps> [kernel substring] [> out.json]
"""
import csv
import glob
import json
import os
import sys

import numpy as np


def main():
    d, steps = sys.argv[1], int(sys.argv[2])
    sub = sys.argv[3] if len(sys.argv) > 3 else "exact::k_residual_wls<4, 1, true, 0, 0>"
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit("no kernel_trace.csv under " + d)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if sub in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    st = np.array([a for a, _ in rows], dtype=np.int64)
    du = np.array([b - a for a, b in rows], dtype=np.float64) / 1e3      # us
    n = len(du)
    win = du[n - 2 * steps:n - steps]
    wst = st[n - 2 * steps:n - steps]
    wen = wst + (win * 1e3).astype(np.int64)
    gaps = (wst[1:] - wen[:-1]) / 1e3

    def s(x):
        return {"n": int(len(x)), "mean_us": round(float(x.mean()), 3), "median_us": round(float(np.median(x)), 3),
                "min_us": round(float(x.min()), 3), "max_us": round(float(x.max()), 3),
                "p90_us": round(float(np.percentile(x, 90)), 3)}
    out = {"kernel": sub, "source": os.path.relpath(files[0]), "dispatches": n, "steps": steps,
           "timed_window": s(win), "event_pass_window": s(du[n - steps:]), "all_dispatches": s(du),
           "timed_window_gap_us": {"median": round(float(np.median(gaps)), 3), "max": round(float(gaps.max()), 3)},
           "timed_window_span_ms": round(float((wen[-1] - wst[0]) / 1e6), 4),
           "note": "timed window = dispatches [-2*steps, -steps) of the kernel (bench.py: timed steps, then the "
                   "same number under HIP-event profiling)"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
