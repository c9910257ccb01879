#!/usr/bin/env python3
"""Static instruction mix of one kernel in a gfx950 assembly listing (hipcc --cuda-device-only -S):
counts of FP64 VALU (add/mul/fma/min/max), FP64 transcendentals (rcp/rsq/sqrt), FP64 compares, other
VALU, LDS, global/buffer memory and scalar instructions, and the VGPR / occupancy metadata.
Static counts of an unrolled straight-line body track the dynamic cost of A/B variants closely.
usage: python tools/isa_count.py listing.s <mangled-name substring> [...]"""
import re
import sys
from collections import Counter


def kernel_body(lines, key):
    start = None
    for i, l in enumerate(lines):
        if start is None and l.startswith("_Z") and key in l.split(":")[0] and l.rstrip().endswith(
                l.split(":")[0] + ":" + l.split(":", 1)[1]) and ":" in l:
            start = i
            name = l.split(":")[0]
            continue
        if start is not None and l.startswith(".Lfunc_end") :
            return name, lines[start:i], lines[i:i + 400]
    return None, [], []


def classify(op):
    if op.startswith("v_"):
        if re.match(r"v_(rcp|rsq|sqrt)_f64", op):
            return "f64_trans"
        if re.match(r"v_cmp\w*_f64", op):
            return "f64_cmp"
        if re.match(r"v_(add|mul|fma|min|max|ldexp|div_\w+|fract|frexp\w*|trig_preop)_f64", op) or "_f64" in op:
            return "f64_alu"
        if op.startswith("v_cndmask"):
            return "cndmask"
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    lines = open(sys.argv[1]).read().splitlines()
    for key in sys.argv[2:]:
        name, body, tail = kernel_body(lines, key)
        if not body:
            print(key, "not found")
            continue
        c = Counter()
        for l in body:
            t = l.strip()
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue
            k = classify(t.split()[0])
            if k:
                c[k] += 1
        meta = {}
        for l in tail:
            m = re.match(r"\s*\.(vgpr_count|sgpr_count|agpr_count|group_segment_fixed_size|private_segment_fixed_size):\s*(\d+)", l)
            if m and m.group(1) not in meta:
                meta[m.group(1)] = int(m.group(2))
        for l in body[-60:] + tail[:60]:
            m = re.search(r"; (NumVgprs|Occupancy|ScratchSize): (\d+)", l)
            if m:
                meta[m.group(1)] = int(m.group(2))
        c["f64_weighted"] = c["f64_alu"] + c["f64_cmp"] + 4 * c["f64_trans"]
        print(name[:90], dict(sorted(c.items())), meta)


if __name__ == "__main__":
    main()
