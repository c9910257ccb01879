"""The implicit legs at the BASELINE configurations' full sizes (SteadyBackwardEulerSolver::solve,
aodesolver.cpp:363-638, with the linear systems on the device; what bench.py's implicit figure times).
Size-independent properties, checked on the meshes the bench runs:
  * C4 (4,063,232 cells, config 4's mesh), assembled operator, line-implicit preconditioner: three steps
    from the free stream stay finite, every linear solve reaches lin_rtol, the residual falls;
  * C5 (the 8,054,616-cell hybrid mesh, config 5: the visc-naca0012 deck's numerics -- Roe, WLS, limiter none, Sutherland,
    alpha 0), matrix-free operator (alinalg.cpp:142-233) with the assembled first-order Jacobian as the
    line-implicit preconditioner: the same checks;
  * C4 split 8 ways by the bench's partitioner (all ranks in one process, device copies for RCCL; lines
    cut at rank boundaries = block-Jacobi across ranks): one step with a tight linear solve gives one
    GPU's update to 1e-8.
"""
import numpy as np
import pytest

import fvens_amd as fa
import cases

pytestmark = pytest.mark.gpu

LIN = dict(lin_rtol=1e-2, lin_maxit=60, restart=30, prec_sweeps=1, prec_lines=True)


def _c4():
    from bench import c4_mesh
    return c4_mesh(fa, 1)[0]


def _three_steps(mesh, p, n, matrix_free):
    import torch
    h = fa.FlowFV(mesh, p, n)
    perm = h.permutation()
    du = torch.tensor(np.tile(cases.freestream(p), (mesh.nelem, 1))[perm], device="cuda")
    torch.cuda.synchronize()
    st, hist = h.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(
        cflinit=25.0, cflfin=25.0, tol=0.0, maxiter=3, matrix_free=matrix_free, **LIN))
    finite = bool(torch.isfinite(du).all().item())
    h.close()
    print(st, [float(x) for x in hist])
    assert st["steps"] == 3 and finite
    assert st["lin_unconverged"] == 0 and st["lin_worst"] <= LIN["lin_rtol"], st
    assert st["lin_iters"] <= 3 * LIN["lin_maxit"]
    assert st["resratio"] < 1.0, (st, hist)


def test_c4_assembled_line_implicit_steps():
    m = _c4()
    assert m.nelem == 4063232
    _three_steps(m, cases.physics("naca"), cases.numerics("ROE", "LEASTSQUARES", "VANALBADA"), False)


def test_c5_matrix_free_steps():
    from bench import c4_mesh
    m = c4_mesh(fa, 1, 2)[0]
    assert m.nelem == 8054616
    _three_steps(m, cases.physics("visc"), cases.numerics("ROE", "LEASTSQUARES", "NONE"), True)


def test_c4_eight_ranks_line_implicit_matches_one_gpu():
    import torch
    m = _c4()
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    u0 = cases.state(m, p, 8)
    cfg = fa.ImplicitConfig(cgs_refine=1, cflinit=25.0, cflfin=25.0, tol=0.0, maxiter=1, lin_rtol=1e-11, lin_maxit=2000,
                            restart=60, prec_sweeps=1, min_relax=1.0, prec_lines=True)
    one = fa.FlowFV(m, p, n)
    perm = one.permutation()
    d1 = torch.tensor(u0[perm], device="cuda")
    torch.cuda.synchronize()
    st1, _ = one.steady_backward_euler_device(d1.data_ptr(), cfg)
    u1 = np.empty_like(u0)
    u1[perm] = d1.cpu().numpy()
    one.close()
    del d1
    part = fa.partition_graph(m, 8, weights="cost")
    sps = [fa.FlowFV(m, p, n, partition=part, rank=k) for k in range(8)]
    dus, gs = [], []
    for k, s_ in enumerate(sps):
        g = np.nonzero(part == k)[0][s_.permutation()]
        d = torch.full((s_.nown + s_.nghost, 4), float("nan"), dtype=torch.float64, device="cuda")
        d[:s_.nown] = torch.tensor(u0[g], device="cuda")
        dus.append(d)
        gs.append(g)
    torch.cuda.synchronize()
    grp = fa.FlowFVGroup(sps)
    st, _ = grp.steady_backward_euler_device([d.data_ptr() for d in dus], cfg)
    u = np.empty_like(u0)
    for k, s_ in enumerate(sps):
        u[gs[k]] = dus[k][:s_.nown].cpu().numpy()
    grp.close()
    for s_ in sps:
        s_.close()
    print("one GPU", st1, "8 ranks", st)
    assert st1["lin_unconverged"] == 0 and st["lin_unconverged"] == 0, (st1, st)
    scale = np.abs(u1 - u0).max(axis=0)
    err = np.abs(u - u1).max(axis=0)
    print("max |u8 - u1| / max |du| per variable", err / scale)
    assert np.all(err <= 1e-8 * scale), err / scale
