#!/usr/bin/env python3
"""Probe: run a few implicit steps (residual, Jacobian assembly with its pseudo-time diagonal, GMRES with the
line-implicit or point-block Jacobi preconditioner, update) on a C4-family mesh from the free stream and save
the final state, the residual history and the GMRES iterations -- run it with two builds of the library
(FVHIP_LIB) and compare the files bitwise. usage: python tools/implicit_state_dump.py OUT.npz [--scale S]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--scale", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import fvens_amd as fa
    import cases
    from bench import c4_mesh
    mesh, _ = c4_mesh(fa, args.scale)
    p = cases.physics("naca")
    res = {}
    for key, extra in (("lines", dict(prec_lines=True)), ("pbj", dict()), ("pbj2", dict(prec_sweeps=2)),
                       ("gs", dict(prec_gs=True, prec_sweeps=2))):
        sp = fa.FlowFV(mesh, p, cases.numerics("ROE", "LEASTSQUARES", "VANALBADA"), device=0)
        u0 = np.tile(cases.freestream(p), (mesh.nelem, 1))[sp.permutation()]
        du = torch.tensor(u0, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        kw = dict(prec_sweeps=1, **extra) if "prec_sweeps" not in extra else dict(extra)
        cfg = fa.ImplicitConfig(cflinit=25.0, cflfin=25.0, tol=0.0, maxiter=args.steps, lin_rtol=1e-2, lin_maxit=30,
                                restart=30, **kw)
        st, hist = sp.steady_backward_euler_device(du.data_ptr(), cfg)
        sp.synchronize()
        res[key + "_u"] = du.cpu().numpy()
        res[key + "_hist"] = np.asarray(hist, dtype=np.float64)
        res[key + "_lin"] = np.asarray([st["lin_iters"]])
        sp.close()
    np.savez(args.out, **res)
    print({k: (v.shape, float(np.abs(v).sum())) for k, v in res.items()})


if __name__ == "__main__":
    main()
