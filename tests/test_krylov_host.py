"""CPU check of the implicit solver's nonlinear update (fvens_amd/csrc/krylov.hpp relaxation_factor,
compiled for the host with the product's flags) against the restatement of FlowSimpleUpdate /
FullUpdate in tests/_oracle.py (nonlinearrelaxation.cpp:24-38, aphysics_defs.hpp:67-80): bitwise,
20,000 random cells per minimum factor, including updates large enough to be under-relaxed."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import _oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = "/opt/rocm/bin/hipcc"


def _lib():
    out = os.path.join(HERE, "_build")
    os.makedirs(out, exist_ok=True)
    lib = os.path.join(out, "librelax_host.so")
    src = os.path.join(HERE, "native", "relax_host_check.cpp")
    hdrs = [os.path.join(ROOT, "fvens_amd", "csrc", h) for h in ("krylov.hpp", "gasdyn.hpp")]
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(f) for f in [src] + hdrs):
        subprocess.run([HIPCC, "-std=c++17", "-O3", "-ffp-contract=off", "-x", "hip", "--offload-arch=gfx950",
                        "-shared", "-fPIC", src, "-o", lib], check=True, capture_output=True)
    L = ctypes.CDLL(lib)
    dp = ctypes.POINTER(ctypes.c_double)
    L.relaxed_update_host.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double, dp, dp, dp]
    L.relaxed_update_host.restype = None
    return L


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("minfactor", [0.2, 0.5, 1.0])
def test_relaxation_matches_restatement(minfactor):
    L = _lib()
    rng = np.random.default_rng(5)
    n, g = 20000, 1.4
    rho = 1.0 + 0.3 * rng.uniform(-1, 1, n)
    vx, vy = rng.uniform(-1, 1, n), rng.uniform(-1, 1, n)
    p = (1.0 + 0.3 * rng.uniform(-1, 1, n)) / (g * 0.64)
    u = np.stack([rho, rho * vx, rho * vy, p / (g - 1) + 0.5 * rho * (vx * vx + vy * vy)], 1)
    scale = 10.0 ** rng.uniform(-6, 0, n)                 # from tiny to O(1) relative changes
    du = u * scale[:, None] * rng.uniform(-1, 1, (n, 4))
    u = np.ascontiguousarray(u)
    du = np.ascontiguousarray(du)
    out = np.zeros_like(u)
    dptr = ctypes.POINTER(ctypes.c_double)
    L.relaxed_update_host(n, g, minfactor, du.ctypes.data_as(dptr), u.ctypes.data_as(dptr), out.ctypes.data_as(dptr))
    ref = orc.relaxed_update(u, du, g, minfactor)
    np.testing.assert_array_equal(out, ref)
    if minfactor < 1.0:
        assert np.any((out - u) != du), "no cell was under-relaxed: the test does not exercise the limiter"
