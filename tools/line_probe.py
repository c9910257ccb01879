#!/usr/bin/env python3
"""Probe: the line-implicit preconditioner's line set on a mesh (ctx.hpp ensureLines): number of lines,
length distribution, how they fill the lane groups of k_line_factor / k_line_solve (lines of >= 16 cells
solved from both ends, 32 per group; others 64 per group, a group's rows = its longest lane), and the
rows x 64 lane slots the kernels walk against the cells they hold. One GPU (the line set is built by the
handle). usage: python tools/line_probe.py [--scale S] [--line-max 256]"""
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
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--line-max", type=int, default=256, help="the library's FVHIP_LINE_MAX (for the group model)")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    mesh, dims = c4_mesh(fa, args.scale)
    sp = fa.FlowFV(mesh, cases.physics("naca"), cases.numerics("ROE", "LEASTSQUARES", "VANALBADA"), device=0)
    lines = sp.lines()
    lens = np.array(sorted((len(c) for c, _ in lines), reverse=True))
    tw = lens[lens >= 16]
    rest = lens[lens < 16]
    g_tw = [tw[i:i + 32] for i in range(0, len(tw), 32)]
    g_rest = [rest[i:i + 64] for i in range(0, len(rest), 64)]
    rows_tw = sum(int((g[0] - 1) // 2 + 1 + 0) for g in g_tw)          # top half + twist cell of the longest
    rows_rest = sum(int(g[0]) for g in g_rest)
    hist = {str(k): int(v) for k, v in zip(*np.unique(np.minimum(lens, 300), return_counts=True))}
    print(json.dumps({"cells": mesh.nelem, "lines": int(len(lens)), "cells_in_lines_ge2": int(lens[lens >= 2].sum()),
                      "single_cells": int((lens == 1).sum()), "max_len": int(lens.max()),
                      "twisted_lines": int(len(tw)), "twisted_groups": len(g_tw), "other_groups": len(g_rest),
                      "rows_twisted": rows_tw, "rows_other": rows_rest,
                      "lane_slots": 64 * (rows_tw + rows_rest),
                      "length_percentiles": {p: float(np.percentile(lens, p)) for p in (50, 90, 99, 99.9)},
                      "length_hist_capped300": hist}), flush=True)
    sp.close()


if __name__ == "__main__":
    main()
