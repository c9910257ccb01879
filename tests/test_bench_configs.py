"""bench.py --numerics: every BASELINE configuration it measures names the fused-kernel instantiation
its numerics select (flux code of include/fvhip.h, SweepRec / SweepVisc of kernels.hpp) and the SURVEY
8(d) byte basis of its reconstruction; no GPU needed."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

# numerics -> (flux code, SweepRec, SweepVisc, limiter): ROE 4, HLLC 6; MUSCL 1, linear 2; Sutherland 1
EXPECT = {"headline": (4, 1, 0, 0), "config2": (4, 1, 0, 0), "config3": (6, 2, 1, 0),
          "config4": (4, 2, 0, 2), "config5": (4, 2, 1, 0)}


def test_kernel_symbols_match_numerics():
    for num, (fl, rec, visc, lim) in EXPECT.items():
        sym = bench.kernel_symbol("k_residual_wls<ROE>", num)
        assert sym == "k_residual_wls<%d, %d, true, %d, %d>" % (fl, rec, visc, lim), (num, sym)
        st = bench.kernel_symbol("k_sweep<ROE>", num)
        assert re.fullmatch(r"k_sweep<%d, %d, %d, true, (true|false)>" % (fl, rec, visc), st), (num, st)
        assert st.endswith("true>") == (lim != 0)


def test_byte_basis_follows_reconstruction():
    N, F, Fb = 1000, 2000, 40
    muscl = bench.sweep_algorithmic_bytes(N, F, Fb)
    linear = bench.config4_algorithmic_bytes(N, F, Fb)
    assert linear > muscl
    for num, (_, rec, _, _) in EXPECT.items():
        assert bench.kernel_bytes("k_residual_wls<ROE>", N, F, Fb, num) == (linear if rec == 2 else muscl), num
