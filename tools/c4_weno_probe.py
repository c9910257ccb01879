"""probe: the reference's own transonic-implicit.ctrl numerics (Roe + least squares + WENO, limiter
parameter 20) as the second-order stage on the C4 family, after a point-block-Jacobi first-order start"""
import json
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tools"); sys.path.insert(0, "tests")
import torch
from c4_converge import converge

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 8
walls = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1e-5, 1e-3]
torch.cuda.set_device(0)
for wall in walls:
    iflux = "LLF" if wall < 1e-4 else "ROE"
    for mcfl, sweeps in (((50.0, 500.0), 1), ((5.0, 200.0), 1), ((50.0, 500.0), 4)):
        try:
            r = converge(scale, wall, iflux, 1500, (5.0, 200.0), mcfl, 1e-7, 2000, "WENO", sweeps=sweeps, verbose=False)
            s0, s1 = r["stages"]
            print(json.dumps({"wall": wall, "main_cfl": mcfl, "sweeps": sweeps,
                              "init": [s0["steps"], "%.1e" % s0["drop_from_peak"], s0["seconds"]],
                              "main": [s1["steps"], s1["converged"], "%.1e" % s1["resratio"], round(s1["cfl_end"]), s1["seconds"],
                                       s1["lin_iters_per_step"]],
                              "CL": r["CL"], "CDp": r["CDp"]}), flush=True)
        except RuntimeError as e:
            print(json.dumps({"wall": wall, "main_cfl": mcfl, "sweeps": sweeps, "error": str(e)}), flush=True)
