#!/usr/bin/env python3
"""Summarise the rocprofv3 passes written by tools/gpu_prof.sh into profiles/<round>/.

Reads <prof>/trace/run_kernel_stats.csv and the separate PMC passes <prof>/{fetch,write,sq}/
run_counter_collection.csv, and writes
  profiles/<round>/kernel_stats.csv   (the trace's --stats summary, copied)
  profiles/<round>/pmc_traffic.json   (per-kernel mean per dispatch of each counter; HBM bytes =
                                       2 x FETCH_SIZE + WRITE_SIZE, KB -> bytes)
The FETCH_SIZE x2 calibration (gfx950 reports half of 16-byte-per-lane reads) is checked on the
streaming kernel k_prep_cells when present (it must read exactly 32 B per cell), and recorded.
usage: python tools/pmc_summary.py gpurun_out/prof profiles/r01 "<workload text with cell count>" [cells] [name]
(name: output basename instead of pmc_traffic)
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def short(name):
    # "void fvhip::exact::k_sweep<4, 1, 0, true, false>(fvhip::DevMesh, ...)" -> "fvhip::exact::k_sweep<4, 1, 0, true, false>"
    n = name[5:] if name.startswith("void ") else name
    depth = 0
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return n[:i]
    return n


def counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def main():
    prof, out, workload = sys.argv[1], sys.argv[2], sys.argv[3]
    cells = int(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4] else None
    name = sys.argv[5] if len(sys.argv) > 5 else "pmc_traffic"
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(prof, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(out, "kernel_stats.csv" if name == "pmc_traffic" else name + "_kernel_stats.csv"))
    merged = defaultdict(dict)
    for sub in sorted(os.listdir(prof)):          # every PMC pass (one subdirectory each)
        p = os.path.join(prof, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for k, cs in counters(p).items():
            for c, vals in cs.items():
                merged[k][c] = sum(vals) / len(vals)
    kernels = {}
    for k, cs in merged.items():
        d = dict(cs)
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            d["fetch_kb_raw"] = cs["FETCH_SIZE"]
            d["write_kb"] = cs["WRITE_SIZE"]
            d["hbm_bytes_corrected"] = 1024.0 * (2.0 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"])
        kernels[k] = d
    cal = "FETCH_SIZE x2 (gfx950 reports half of 16B/lane reads)"
    for k, d in kernels.items():
        if k.endswith("k_prep_cells") and cells and "FETCH_SIZE" in d:
            cal += f"; check on k_prep_cells: FETCH {d['FETCH_SIZE']:.0f} KB vs {32 * cells / 1024:.0f} KB read"
    doc = {"workload": workload,
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE / --pmc SQ_* in separate passes over "
                     "bench.py; mean per dispatch",
           "calibration": cal, "kernels": kernels}
    with open(os.path.join(out, name + ".json"), "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps({k: round(v.get("hbm_bytes_corrected", 0) / 1e6, 1) for k, v in kernels.items()}))


if __name__ == "__main__":
    main()
