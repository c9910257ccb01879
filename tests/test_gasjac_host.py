"""CPU check of the device Jacobian source (fvens_amd/csrc/gasjac.hpp), compiled for the host with
the product's flags, against the oracle's full-block flux and BC Jacobians: bitwise, 20,000 random
face states per flux (subsonic / supersonic / equal states / exact-zero velocity components).
The GPU build of the same source is checked through the C-ABI in test_gpu_jacobian.py."""
import os
import shutil
import subprocess

import pytest

import _oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_column_jacobians_match_oracle_on_host():
    orc.build()
    out = os.path.join(HERE, "_build")
    os.makedirs(out, exist_ok=True)
    exe = os.path.join(out, "gasjac_host_check")
    src = os.path.join(HERE, "native", "gasjac_host_check.cpp")
    odir = os.path.join(ROOT, "oracle")
    hdr = os.path.join(ROOT, "fvens_amd", "csrc", "gasjac.hpp")
    if not os.path.exists(exe) or os.path.getmtime(exe) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.run([HIPCC, "-std=c++17", "-O3", "-ffp-contract=off", "-x", "hip", "--offload-arch=gfx950",
                        src, "-o", exe, "-L" + odir, "-loracle", "-Wl,-rpath," + odir],
                       check=True, capture_output=True)
    r = subprocess.run([exe, "20000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout
