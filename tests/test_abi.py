"""The C-ABI library loads (no GPU needed) and exports every symbol include/fvhip.h declares."""
import ctypes
import os
import re

import fvens_amd._ffi as ffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "fvhip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b((?:fvhip|fvmesh)_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_functions():
    names = declared_functions()
    assert "fvhip_compute_residual" in names and "fvhip_create" in names
    assert len(names) >= 30


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(ffi.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_every_declared_symbol():
    assert set(declared_functions()) == set(ffi._SIGS)


def test_device_count_never_fails():
    assert ffi.lib().fvhip_device_count() >= 0


def test_errors_do_not_cross_the_abi():
    h = ctypes.c_void_p()
    rc = ffi.lib().fvmesh_read_gmsh(b"/nonexistent.msh", ctypes.byref(h))
    assert rc != 0
    assert b"cannot open" in ffi.lib().fvhip_last_error()
