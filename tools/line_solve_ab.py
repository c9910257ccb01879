#!/usr/bin/env python3
"""A/B of line-solve builds (FVHIP_LIB selects the library): the line-implicit preconditioner
(fvhip_line_precondition_device: factor + solve) on the C4 or C5 mesh with the first-order Jacobian plus a
pseudo-time term, and a 3-step matrix-free implicit solve whose finite-difference step comes from the line
solve's own |z| (one sweep). Prints one JSON line with the SHA-256 of z and the residual history's hex, so
two builds can be compared bit for bit; run under rocprofv3 --kernel-trace --stats for the kernel times.
usage: python tools/line_solve_ab.py [--case c4|c5] [--scale 1] [--reps 20]"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="c4")
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--implicit-scale", type=int, default=4, help="the matrix-free solve's mesh: C5 / this")
    ap.add_argument("--jac-reps", type=int, default=1, help="Jacobian assemblies (the last one is used)")
    ap.add_argument("--no-implicit", action="store_true")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    out = {"library": fa._ffi.build_info()["library"], "case": args.case, "scale": args.scale}
    mesh, dims = c4_mesh(fa, args.scale, 1 if args.case == "c4" else 2)
    if args.case == "c4":
        p, n = cases.physics("naca"), cases.numerics("ROE", "NONE", "NONE", order2=False)
    else:
        p, n = cases.physics("visc"), cases.numerics("ROE", "NONE", "NONE", order2=False)
    h = fa.FlowFV(mesh, p, n)
    N, Fi = mesh.nelem, mesh.naface - mesh.nbface
    rng = np.random.default_rng(7)
    u = torch.tensor(cases.state(mesh, p, 3)[h.permutation()], device="cuda")
    diag = torch.zeros((N, 16), dtype=torch.float64, device="cuda")
    lower = torch.zeros((Fi, 16), dtype=torch.float64, device="cuda")
    upper = torch.zeros((Fi, 16), dtype=torch.float64, device="cuda")
    r = torch.zeros((N, 4), dtype=torch.float64, device="cuda")
    dtm = torch.zeros(N, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    h.compute_residual_device(u.data_ptr(), r.data_ptr(), dtm.data_ptr(), True, True)
    for _ in range(args.jac_reps):                  # the face-Jacobian kernel's timing (A/B of its builds)
        h.assemble_jacobian_device(u.data_ptr(), diag.data_ptr(), lower.data_ptr(), upper.data_ptr())
    h.synchronize()
    out["jacobian_sha256"] = hashlib.sha256(lower.cpu().numpy().tobytes() + upper.cpu().numpy().tobytes()
                                            + diag.cpu().numpy().tobytes()).hexdigest()[:16]
    h.add_pseudo_time_term_device(100.0, dtm.data_ptr(), diag.data_ptr())
    v = torch.tensor(rng.standard_normal((N, 4)), device="cuda")
    z = torch.zeros_like(v)
    h.synchronize()
    for _ in range(args.reps):
        h.line_precondition_device(diag.data_ptr(), lower.data_ptr(), upper.data_ptr(), v.data_ptr(), z.data_ptr())
    h.synchronize()
    zc = z.cpu().numpy()
    out.update(cells=N, z_sha256=hashlib.sha256(zc.tobytes()).hexdigest()[:16], z_finite=bool(np.isfinite(zc).all()),
               z_absmax=float(np.abs(zc).max()))
    h.close()
    if args.no_implicit:
        print(json.dumps(out), flush=True)
        return
    # matrix-free implicit steps with the line solve's |z| (single domain, one sweep)
    m5, _ = c4_mesh(fa, args.implicit_scale, 2)
    p5 = cases.physics("visc")
    h5 = fa.FlowFV(m5, p5, cases.numerics("ROE", "LEASTSQUARES", "NONE"))
    u5 = torch.tensor(np.tile(cases.freestream(p5), (m5.nelem, 1))[h5.permutation()], device="cuda")
    torch.cuda.synchronize()
    st, hist = h5.steady_backward_euler_device(u5.data_ptr(), fa.ImplicitConfig(
        cflinit=25.0, cflfin=25.0, tol=0.0, maxiter=3, lin_rtol=1e-2, lin_maxit=30, restart=30, prec_lines=True,
        prec_sweeps=1, matrix_free=True, min_relax=1.0))
    torch.cuda.synchronize()
    out.update(implicit_cells=m5.nelem, lin_iters=st["lin_iters"], history_hex=[float(x).hex() for x in hist],
               state_sha256=hashlib.sha256(u5.cpu().numpy().tobytes()).hexdigest()[:16])
    h5.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
