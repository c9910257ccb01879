#!/usr/bin/env python3
"""Layout statistics of the bench mesh (patches, slots, ring-1 staging of the fused residual)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401  (HIP runtime first)
import fvens_amd as fa
import cases
from bench import c4_mesh
m, _ = c4_mesh(fa, int(sys.argv[1]) if len(sys.argv) > 1 else 1)
sp = fa.FlowFV(m, cases.physics("naca"), cases.numerics("ROE", "LEASTSQUARES", "VANALBADA"))
st = sp.layout_stats()
st["ring1_over_cells"] = round(st["ring1_cells"] / st["cells"], 4)
st["slots_over_faces"] = round(st["slots"] / st["faces"], 4)
print(json.dumps(st))
