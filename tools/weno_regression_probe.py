#!/usr/bin/env python3
"""Probe: the reference's SpatialFlow_Euler_NACA0012_WENO_LeastSquares_HLLC_
FunctionalRegression (testcases/naca0012/CMakeLists.txt:7-14: transonic-sanity-test-weno.ctrl +
opts.solverc on naca0012luo.msh, regr-WENO_LeastSquares_HLLC.txt = CL 0.151870649085658, CDp
0.013085625502343) with the device implicit driver, for several WENO central weights lambda: the
reference never parses `limiter_parameter` (controlparser.cpp:182, 230), so its lambda is whatever the
uninitialised FlowParserOptions member held. Starter and main solves as tests/test_gpu_implicit.py's
MUSCL regression (first-order HLLC CFL 50-1000 tol 1e-1 20 steps; main CFL 500-5000 tol 1e-7; robust
update 0.2; rtol 1e-1, 30 its); then the main solve continued to a 1e-11 drop. One JSON line per lambda.
usage: python tools/weno_regression_probe.py [--lambdas 20,0,1]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

CL_REF, CDP_REF = 0.151870649085658, 0.013085625502343


def run(lam, precs=("pbj",), maxiter=600):
    import torch
    import fvens_amd as fa
    import cases
    m = fa.UMesh.read_gmsh(cases.fixture_mesh("naca0012luo"))
    p = cases.physics("naca")
    n1 = cases.numerics("HLLC", "NONE", "NONE", order2=False)
    n2 = cases.numerics("HLLC", "LEASTSQUARES", "WENO", K=lam)
    start, main = fa.FlowFV(m, p, n1), fa.FlowFV(m, p, n2)
    perm = main.permutation()
    u0 = np.tile(cases.freestream(p), (m.nelem, 1))
    out = []
    for prec in precs:
        dU = torch.tensor(u0[perm], device="cuda")
        lin = dict(lin_rtol=1e-1, lin_maxit=30, restart=30, prec_sweeps=4 if prec == "pbj" else 1, min_relax=0.2,
                   prec_lines=prec == "lines")
        st0, _ = start.steady_backward_euler_device(dU.data_ptr(), fa.ImplicitConfig(
            cflinit=50.0, cflfin=1000.0, tol=1e-1, maxiter=20, **lin))
        rec = {"lambda": lam, "prec": prec, "starter": st0}
        try:
            st, hist = main.steady_backward_euler_device(dU.data_ptr(), fa.ImplicitConfig(
                cflinit=500.0, cflfin=5000.0, tol=1e-7, maxiter=maxiter, **lin))
            (cl, cdp, _), _ = main.surface_data_device(dU.data_ptr(), 2)
            rec.update(main=st, CL=cl, CDp=cdp, CL_rel=abs(cl - CL_REF) / CL_REF, CDp_rel=abs(cdp - CDP_REF) / CDP_REF)
            st2, _ = main.steady_backward_euler_device(dU.data_ptr(), fa.ImplicitConfig(
                cflinit=500.0, cflfin=5000.0, tol=1e-4, maxiter=maxiter, **lin))
            (cl2, cdp2, _), _ = main.surface_data_device(dU.data_ptr(), 2)
            rec.update(further=st2, CL_conv=cl2, CDp_conv=cdp2, CL_conv_rel=abs(cl2 - CL_REF) / CL_REF,
                       CDp_conv_rel=abs(cdp2 - CDP_REF) / CDP_REF)
        except RuntimeError as e:
            rec["error"] = str(e)
        out.append(rec)
    start.close()
    main.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lambdas", default="20,0,1")
    ap.add_argument("--precs", default="pbj")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    for lam in [float(x) for x in args.lambdas.split(",")]:
        for rec in run(lam, tuple(args.precs.split(","))):
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
