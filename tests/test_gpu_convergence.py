"""Order of accuracy, the reference's own entropy-convergence tests (tests/inv-2dcyl/CMakeLists.txt:14-53,
driver tests/flow_conv.cpp): inviscid flow past a cylinder (inv-cyl-base.ctrl: M 0.38, slip wall 2,
far field 4) on the reference's nested triangle meshes testcases/2dcylinder/grids/2dcylinder{0..3}.msh,
solved to steady state by the device pseudo-time drivers (first-order starter, then the second-order
main solve, casesolvers.cpp:225-314), entropy error by the device FlowOutput::compute_entropy_cell
(aoutput.cpp:28-62) against the mesh size 1/sqrt(nelem). Pass bar (flow_conv.cpp:77-89): the finest
pair's slope of log(error) vs log(h) lies in [1.65, 2.1].

Linear solver: the reference's inv_cyl.solverc uses FGMRES (rtol 1e-1, 30 its) with block-Jacobi/ILU(0);
here device GMRES (same iteration cap) with the preconditioner that converges each case: two multicolour
block Gauss-Seidel sweeps and rtol 1e-2 (LS+HLLC), point-block Jacobi and rtol 1e-1 (GG+HLLC).

Deviation, measured on MI355X (tools/experiments/conv_probe.py and conv_probe2.py, in git history up to f4c3eb0): the implicit main solves run
towards a 1e-7 residual drop (1500 steps at most) instead of the decks' 1e-5 and must reach the decks'
1e-5. Stopped at 1e-5 the device path leaves more algebraic error on the finest mesh (LS+HLLC finest
slope 1.50); converged, the slopes are the discretisation's own: LS+HLLC 1.864/1.790/1.675, GG+HLLC
1.773/1.973/1.772. These inviscid solves are path-sensitive, and so is where they land: with rtol 1e-1
two Gauss-Seidel sweeps stagnate LS+HLLC on 2dcylinder3 near 4e-4 in one internal cell order (256-face
patches) and converge in another (512), point-block Jacobi stagnates on 2dcylinder2 at 3e-3, four
block-Jacobi sweeps on 2dcylinder3 at 8e-4; with rtol 1e-2 every preconditioner tried converges all
four meshes, to finest slopes 1.662-1.675 (two solutions of the LS+HLLC discretisation on 2dcylinder3,
log10 entropy error -2.9245 and -2.9286, both at a 1e-7 residual drop). Hence the per-case choice. The reference's driver does not check convergence at all (flow_conv.cpp only catches
Numerical_error) and stops at max_timesteps."""
import numpy as np
import pytest

import fvens_amd as fa
import _oracle as orc
import cases

pytestmark = pytest.mark.gpu

# (gradient, flux, implicit?, (starter cfl_min, cfl_max, tol, maxit), (main cfl_min, cfl_max, tol, maxit),
#  meshes, residual drop required of the main solve, preconditioner)
CASES = {
    # SpatialFlow_Euler_Cylinder_LeastSquares_HLLC_Tri_EntropyConvergence (inv-cyl-ls-hllc.ctrl)
    "ls_hllc_implicit": ("LEASTSQUARES", "HLLC", True, (25.0, 500.0, 1e-1, 150), (250.0, 5000.0, 1e-7, 1500), 4, 1e-5, dict(prec_sweeps=2, prec_gs=True, lin_rtol=1e-2)),
    # SpatialFlow_Euler_Cylinder_GreenGauss_HLLC_Tri_EntropyConvergence (inv-cyl-gg-hllc_tri.ctrl)
    "gg_hllc_implicit": ("GREENGAUSS", "HLLC", True, (25.0, 250.0, 1e-1, 250), (250.0, 1000.0, 1e-7, 1500), 4, 1e-5, dict(prec_sweeps=1)),
    # Flow_Explicit_Euler_Cylinder_GreenGauss_Roe_Tri_EntropyConvergence (expl-inv-cyl-gg-roe_tri.ctrl)
    "gg_roe_explicit": ("GREENGAUSS", "ROE", False, (0.5, 0.7, 1e-1, 15000), (0.25, 0.30, 1e-4, 60000), 3, 1e-4, None),
}


def solve_entropy(meshname, grad, flux, implicit, init, main, drop, prec=None):
    import torch
    m = fa.UMesh.read_gmsh(cases.fixture_mesh(meshname))
    p = cases.physics("cyl")
    n1 = cases.numerics(flux, "NONE", "NONE", order2=False)     # firstorder_spatial_numerics_config
    n2 = cases.numerics(flux, grad, "NONE")
    start, sp = fa.FlowFV(m, p, n1), fa.FlowFV(m, p, n2)
    perm = sp.permutation()
    u0 = np.tile(cases.freestream(p), (m.nelem, 1))
    du = torch.tensor(u0[perm], device="cuda")
    if implicit:
        lin = dict(lin_rtol=1e-1, lin_maxit=30, restart=30, min_relax=0.2)
        lin.update(prec or {})
        st0, _ = start.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(
            cflinit=init[0], cflfin=init[1], tol=init[2], maxiter=init[3], **lin))
        st, _ = sp.steady_backward_euler_device(du.data_ptr(), fa.ImplicitConfig(
            cflinit=main[0], cflfin=main[1], tol=main[2], maxiter=main[3], **lin))
        converged = st["resratio"] <= drop
    else:
        # the explicit solver steps with cfl_min (aodesolver.cpp:194-209)
        start.steady_forward_euler_device(du.data_ptr(), init[0], init[2], init[3])
        steps, ratio, _ = sp.steady_forward_euler_device(du.data_ptr(), main[0], main[2], main[3])
        st, converged = dict(steps=steps, resratio=ratio), ratio <= drop
    err = sp.entropy_error_device(du.data_ptr())
    u = np.empty_like(u0)
    u[perm] = du.cpu().numpy()
    om = orc.OracleMesh.read(cases.fixture_mesh(meshname))
    err_o = orc.OracleSpatial(om, p, n2).entropy(u)
    start.close()
    sp.close()
    return m.nelem, err, err_o, st, converged


@pytest.mark.parametrize("case", list(CASES))
def test_entropy_convergence(case):
    grad, flux, implicit, init, main, nmesh, drop, prec = CASES[case]
    lh, le = [], []
    for i in range(nmesh):
        nelem, err, err_o, st, conv = solve_entropy("2dcylinder%d" % i, grad, flux, implicit, init, main, drop, prec)
        # the device entropy error is the reference's to rounding (a parallel sum; device pow)
        assert abs(err - err_o) <= 1e-12 * err_o, (err, err_o)
        assert conv, st
        lh.append(np.log10(1.0 / np.sqrt(nelem)))
        le.append(np.log10(err))
        print(f"{case} mesh {i}: nelem {nelem} log h {lh[-1]:.4f} log err {le[-1]:.6f} {st}")
    slopes = [(le[i] - le[i - 1]) / (lh[i] - lh[i - 1]) for i in range(1, nmesh)]
    print(f"{case}: slopes {slopes}")
    assert 1.65 <= slopes[-1] <= 2.1, slopes
