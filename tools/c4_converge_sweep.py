"""probe: tools/c4_converge.converge over reconstructions / wall spacings / CFL schedules at a reduced
scale (one JSON summary line per run)"""
import json
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tools"); sys.path.insert(0, "tests")
import torch
from c4_converge import converge

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 8
torch.cuda.set_device(0)
for wall, iflux in ((1e-3, "ROE"), (1e-5, "LLF")):
    for rec in ("VENKATAKRISHNAN", "NONE", "VANALBADA"):
        for mcfl in ((5.0, 200.0), (20.0, 2000.0)):
            try:
                r = converge(scale, wall, iflux, 1500, (5.0, 200.0), mcfl, 1e-6, 3000, rec, verbose=False)
                s0, s1 = r["stages"]
                print(json.dumps({"wall": wall, "rec": rec, "main_cfl": mcfl,
                                  "init": [s0["steps"], "%.1e" % s0["drop_from_peak"], s0["seconds"]],
                                  "main": [s1["steps"], s1["converged"], "%.1e" % s1["resratio"], s1["cfl_end"], s1["seconds"]],
                                  "CL": r["CL"], "CDp": r["CDp"]}), flush=True)
            except RuntimeError as e:
                print(json.dumps({"wall": wall, "rec": rec, "main_cfl": mcfl, "error": str(e)}), flush=True)
