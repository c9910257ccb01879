#!/usr/bin/env python3
"""Why does GMRES stall on the C5 family's main solve? Runs the visc-naca0012 deck (first-order start,
then `--main-steps` second-order matrix-free steps) on C5/scale, then at that state compares the operators
the linear solve sees: the matrix-free second-order operator A2 (alinalg.cpp:142-233), the assembled
first-order operator J1 + mdt that preconditions it, and the line-implicit z = M^-1 r. Prints one JSON line:
cosines of A2 z and J1 z with r, the relative difference of A2 z and J1 z, A2's linearity and its
sensitivity to the difference step, and the cells that dominate |r| and |A2 z - J1 z|.
usage: python tools/mf_diagnose.py [--scale 8] [--main-steps 30]"""
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
    ap.add_argument("--scale", type=int, default=8)
    ap.add_argument("--main-steps", type=int, default=30)
    ap.add_argument("--farmap", type=int, default=None, help="an O-grid with this generateNacaOgrid farmap (default: the C5 C-grid)")
    ap.add_argument("--cfl", type=float, default=None, help="CFL of the diagnosed system (default: the main's last)")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    mesh, dims = c4_mesh(fa, args.scale, 2, farmap=args.farmap)
    p = cases.physics("visc")
    h1 = fa.FlowFV(mesh, p, cases.numerics("ROE", "NONE", "NONE", order2=False))
    h2 = fa.FlowFV(mesh, p, cases.numerics("ROE", "LEASTSQUARES", "NONE"))
    perm = h2.permutation()
    assert np.array_equal(perm, h1.permutation())
    N, Fi = mesh.nelem, mesh.naface - mesh.nbface
    dev = dict(dtype=torch.float64, device="cuda")
    u = torch.tensor(np.tile(cases.freestream(p), (N, 1))[perm], device="cuda")
    torch.cuda.synchronize()
    lin = dict(lin_rtol=1e-1, lin_maxit=60, restart=60, prec_lines=True, prec_sweeps=3, min_relax=1.0)
    st0, _ = h1.steady_backward_euler_device(u.data_ptr(), fa.ImplicitConfig(cflinit=200.0, cflfin=1000.0, tol=1e-1,
                                                                            maxiter=50, **lin))
    st, hist = h2.steady_backward_euler_device(u.data_ptr(), fa.ImplicitConfig(
        cflinit=500.0, cflfin=5000.0, tol=1e-6, maxiter=args.main_steps, matrix_free=True, **lin))
    torch.cuda.synchronize()
    cfl = args.cfl or st["cfl"]
    out = {"cells": N, "dims": dims, "init": {k: st0[k] for k in ("steps", "resratio", "lin_worst")},
           "main": {k: st[k] for k in ("steps", "resratio", "lin_worst", "cfl")}, "history_tail": [float(x) for x in hist[-3:]],
           "cfl": cfl}
    r = torch.zeros((N, 4), **dev)
    dtm = torch.zeros(N, **dev)
    h2.compute_residual_device(u.data_ptr(), r.data_ptr(), dtm.data_ptr(), True, True)
    diag = torch.zeros((N, 16), **dev)
    lower = torch.zeros((Fi, 16), **dev)
    upper = torch.zeros((Fi, 16), **dev)
    h1.assemble_jacobian_device(u.data_ptr(), diag.data_ptr(), lower.data_ptr(), upper.data_ptr())
    h1.add_pseudo_time_term_device(cfl, dtm.data_ptr(), diag.data_ptr())        # dtm <- area / (CFL dt)
    h2.matfree_set_state_device(u.data_ptr(), r.data_ptr(), dtm.data_ptr())

    def A2(x, eps=None):
        if eps is not None:
            h2.matfree_set_eps(eps)
        y = torch.zeros_like(x)
        h2.matfree_apply_device(x.data_ptr(), y.data_ptr())
        h2.synchronize()
        if eps is not None:
            h2.matfree_set_eps(1e-7)
        return y

    def J1(x):
        y = torch.zeros_like(x)
        h1.block_apply_device(diag.data_ptr(), lower.data_ptr(), upper.data_ptr(), x.data_ptr(), y.data_ptr())
        h1.synchronize()
        return y

    def Minv(x):
        y = torch.zeros_like(x)
        h1.line_precondition_device(diag.data_ptr(), lower.data_ptr(), upper.data_ptr(), x.data_ptr(), y.data_ptr())
        h1.synchronize()
        return y

    def cos(a, b):
        return float((a * b).sum() / (a.norm() * b.norm()))

    def rel(a, b):
        return float((a - b).norm() / b.norm())
    z = Minv(r)
    a2z, j1z = A2(z), J1(z)
    rng = np.random.default_rng(3)
    x = torch.tensor(rng.standard_normal((N, 4)), **dev)
    a2x, j1x = A2(x), J1(x)
    out.update({
        "cos_A2z_r": cos(a2z, r), "cos_J1z_r": cos(j1z, r), "rel_A2z_J1z": rel(a2z, j1z), "rel_J1z_r": rel(j1z, r),
        "rel_A2x_J1x_random": rel(a2x, j1x),
        "A2_linearity_2z": rel(A2(2.0 * z), 2.0 * a2z), "A2_linearity_sum": rel(A2(z + x), a2z + a2x),
        "A2z_eps1e-5": rel(A2(z, 1e-5), a2z), "A2z_eps1e-9": rel(A2(z, 1e-9), a2z),
        "norms": {"r": float(r.norm()), "z": float(z.norm()), "A2z": float(a2z.norm()), "J1z": float(j1z.norm()),
                  "mdt_z": float((dtm[:, None] * z).norm())},
    })
    rc = mesh.rc[perm] if hasattr(mesh, "rc") else None

    def top(v, k=8):
        q = v.norm(dim=1).cpu().numpy()
        idx = np.argsort(-q)[:k]
        share = float((np.sort(q ** 2)[::-1][:100]).sum() / (q ** 2).sum())
        return {"share_top100": share, "cells": [[int(c), float("%.3e" % q[c]), [round(float(t), 6) for t in rc[c]]]
                                                 for c in idx]}
    out["top_r"] = top(r)
    out["top_z"] = top(z)
    out["top_A2z_minus_J1z"] = top(a2z - j1z)
    h1.close()
    h2.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
