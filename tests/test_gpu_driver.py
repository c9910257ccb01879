"""End-to-end through the C++ host wrapper (fvens_amd/host/flowfv_hip.hpp): the reference's explicit
pseudo-time loop (aodesolver.cpp:170-240) driven by a compiled C++ program against libfvhip.so,
compared with the oracle's forward Euler on the same mesh. Parity mode: the state after 40 steps
is BITWISE equal (every residual and time step is); fast-math mode: within 1e-10 relative."""
import os
import subprocess

import numpy as np
import pytest

import fvens_amd as fa
import _oracle as orc
import cases

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
EXE = os.path.join(HERE, "_build", "explicit_driver")


def build_driver():
    src = os.path.join(HERE, "native", "explicit_driver.cpp")
    hdr = os.path.join(ROOT, "fvens_amd", "host", "flowfv_hip.hpp")
    lib = os.path.join(ROOT, "fvens_amd", "libfvhip.so")
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    if (not os.path.exists(EXE) or os.path.getmtime(EXE) < max(os.path.getmtime(src), os.path.getmtime(hdr),
                                                             os.path.getmtime(lib))):
        subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", src, "-o", EXE, "-L" + os.path.dirname(lib),
                        "-lfvhip", "-Wl,-rpath," + os.path.dirname(lib)], check=True, capture_output=True)
    return EXE


def build_implicit_driver():
    src = os.path.join(HERE, "native", "implicit_driver.cpp")
    hdr = os.path.join(ROOT, "fvens_amd", "host", "flowfv_hip.hpp")
    lib = os.path.join(ROOT, "fvens_amd", "libfvhip.so")
    exe = os.path.join(HERE, "_build", "implicit_driver")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    if (not os.path.exists(exe) or os.path.getmtime(exe) < max(os.path.getmtime(src), os.path.getmtime(hdr),
                                                             os.path.getmtime(lib))):
        subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", src, "-o", exe, "-L" + os.path.dirname(lib),
                        "-lfvhip", "-Wl,-rpath," + os.path.dirname(lib)], check=True, capture_output=True)
    return exe


def test_driver_builds_against_wrapper():
    assert os.path.exists(build_driver())
    assert os.path.exists(build_implicit_driver())


@pytest.mark.gpu
def test_implicit_driver_matfree_vs_matrix():
    """SteadyBackwardEulerSolver_HIP (C++ wrapper) on the reference's MatFreeVsMat settings: both
    operators converge, in the same number of pseudo-steps (testmatrixfree.cpp:65)"""
    r = subprocess.run([build_implicit_driver(), os.path.join(HERE, "fixtures", "meshes", "2dcylinder2.msh")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("steps ")][0]
    a, b = [int(x) for x in line.split()[1:]]
    assert a == b and 0 < a < 100, r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("fast", [False, True])
def test_explicit_pseudo_time_matches_oracle(tmp_path, fast):
    nt, nq, ntri, nsteps, cfl = 96, 6, 18, 40, 0.5
    out = tmp_path / "u.bin"
    r = subprocess.run([build_driver(), str(out), str(nt), str(nq), str(ntri), str(nsteps), str(cfl),
                        "1" if fast else "0"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = np.fromfile(out, dtype=np.uint8)
    N = int(raw[:4].view(np.int32)[0])
    u_dev = raw[4:4 + 32 * N].view(np.float64).reshape(N, 4)
    hist = raw[4 + 32 * N:].view(np.float64)
    assert hist.shape == (nsteps,)

    m = fa.UMesh.naca_ogrid(nt, nq, ntri, 20.0, 1e-4)
    om = orc.OracleMesh.from_raw(m.raw())
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    u = np.tile(cases.freestream(p), (N, 1))
    steps, ratio = orc.OracleSpatial(om, p, n).forward_euler(u, cfl, 0.0, nsteps)
    assert steps == nsteps
    if fast:
        np.testing.assert_allclose(u_dev, u, rtol=1e-10, atol=1e-12)
    else:
        np.testing.assert_array_equal(u_dev, u)
        assert hist[-1] / hist[0] == ratio


@pytest.mark.gpu
@pytest.mark.parametrize("meshkey,kind,flux,grad,rec,order2", [
    ("2dcylinderhybrid.msh", "cyl", "LLF", "NONE", "NONE", False),        # BASELINE config 1 (C1-like)
    ("c1", "cyl", "LLF", "NONE", "NONE", False),                         # BASELINE config 1 at its size: 5,120 cells
    ("naca_small", "naca", "ROE", "LEASTSQUARES", "VANALBADA", True)])
def test_device_forward_euler_matches_oracle(meshkey, kind, flux, grad, rec, order2):
    """Device-resident explicit pseudo-time loop: state after 30 steps bitwise equal to the oracle's
    forward Euler (the norm reduction order differs, so only the state is compared bitwise). BASELINE
    config 1 (inviscid cylinder, LLF, first order, explicit; tests/inv-2dcyl/inv-cyl-base.ctrl) runs on
    SURVEY's 5,120-cell C1 O-grid as well as on the reference's 2dcylinderhybrid fixture."""
    import torch
    from test_gpu_residual import get_mesh
    m, om = get_mesh(meshkey)
    if meshkey == "c1":
        assert m.nelem == 5120 and m.naface == 7744
    p = cases.physics(kind)
    n = cases.numerics(flux, grad, rec, order2=order2)
    u0 = np.tile(cases.freestream(p), (m.nelem, 1))
    dev = fa.FlowFV(m, p, n)
    perm = dev.permutation()
    du = torch.tensor(u0[perm], device="cuda")
    steps, ratio, hist = dev.steady_forward_euler_device(du.data_ptr(), 0.5, 0.0, 30)
    u_dev = np.empty_like(u0)
    u_dev[perm] = du.cpu().numpy()
    u_ref = u0.copy()
    s2, r2 = orc.OracleSpatial(om, p, n).forward_euler(u_ref, 0.5, 0.0, 30)
    assert steps == s2 == 30
    np.testing.assert_array_equal(u_dev, u_ref)
    assert abs(ratio - r2) <= 1e-12 * abs(r2)
    dev.close()
