"""Error behaviour of the boundary, no GPU needed: a configuration the reference's factories cannot
build (afactory.cpp:38-81, 178-211; abc.cpp:460-500) is refused before any device work, the C-ABI
returns a nonzero status with the reason in fvhip_last_error() (no exception crosses it), and the
Python mirror raises with the same reason. fvhip_create validates the configuration before it
touches the device, so these run on a host without a GPU."""
import ctypes
import math

import numpy as np
import pytest

import cases
import fvens_amd as fa
import fvens_amd._ffi as ffi


@pytest.fixture(scope="module")
def mesh():
    return fa.UMesh.naca_ogrid(32, 2, 4)


def create_error(mesh, p, n):
    """fvhip_create's status and message for (p, n) built by the Python mirror's own config struct"""
    cfg, keep = fa._config_struct(p, n)
    h = ctypes.c_void_p()
    rc = ffi.lib().fvhip_create(ctypes.byref(mesh.view), ctypes.byref(cfg), 0, ctypes.byref(h))
    return rc, ffi.lib().fvhip_last_error().decode()


def raw_config(p, n, **fields):
    cfg, keep = fa._config_struct(p, n)
    for k, v in fields.items():
        setattr(cfg, k, v)
    return cfg, keep


@pytest.mark.parametrize("field,value,msg", [
    ("conv_numflux", 7, "unknown flux"),
    ("conv_numflux", -1, "unknown flux"),
    ("conv_numflux_jac", 9, "unknown Jacobian flux"),
    ("reconstruction", 5, "Invalid reconstruction"),
    ("nbc", -1, "too many boundary conditions"),
    ("nbc", 1000, "too many boundary conditions"),
])
def test_create_refuses_unknown_schemes(mesh, field, value, msg):
    cfg, keep = raw_config(cases.physics("naca"), cases.numerics(), **{field: value})
    h = ctypes.c_void_p()
    rc = ffi.lib().fvhip_create(ctypes.byref(mesh.view), ctypes.byref(cfg), 0, ctypes.byref(h))
    assert rc != 0 and not h.value
    assert msg in ffi.lib().fvhip_last_error().decode()


def test_create_refuses_periodic_and_unknown_bc(mesh):
    """PERIODIC_BC throws 'BC type not implemented yet!' (abc.cpp:493-494)"""
    p = cases.physics("naca")
    types = np.array([fa.BCTYPES["periodic"]] * len(p.bcconf), np.int32)
    cfg, keep = raw_config(p, cases.numerics())
    cfg.bc_type = fa.iptr(types)
    h = ctypes.c_void_p()
    assert ffi.lib().fvhip_create(ctypes.byref(mesh.view), ctypes.byref(cfg), 0, ctypes.byref(h)) != 0
    assert "BC type not implemented yet!" in ffi.lib().fvhip_last_error().decode()
    types[:] = 8
    assert ffi.lib().fvhip_create(ctypes.byref(mesh.view), ctypes.byref(cfg), 0, ctypes.byref(h)) != 0
    p.bcconf[0].bc_type = "periodic"
    with pytest.raises(RuntimeError, match="BC type not implemented yet!"):
        fa.FlowFV(mesh, p, cases.numerics())


@pytest.mark.parametrize("rec,K", [
    ("VENKATAKRISHNAN", 0.0), ("VENKATAKRISHNAN", -5.0), ("VENKATAKRISHNAN", math.nan),
    ("VENKATAKRISHNAN", math.inf), ("WENO", -1.0), ("WENO", math.nan),
])
def test_create_refuses_unusable_limiter_parameter(mesh, rec, K):
    """Venkatakrishnan's eps^2 = (K clength)^3 (limitedlinearreconstruction.cpp:222) must be > 0: the
    reference never parses K (controlparser.cpp:227-232), so the boundary requires it explicitly"""
    rc, err = create_error(mesh, cases.physics("naca"), cases.numerics("ROE", "LEASTSQUARES", rec, K=K))
    assert rc != 0 and "limiter_param" in err


def test_null_arguments(mesh):
    cfg, keep = raw_config(cases.physics("naca"), cases.numerics())
    h = ctypes.c_void_p()
    assert ffi.lib().fvhip_create(None, ctypes.byref(cfg), 0, ctypes.byref(h)) != 0
    assert "null argument" in ffi.lib().fvhip_last_error().decode()
    assert ffi.lib().fvhip_create(ctypes.byref(mesh.view), None, 0, ctypes.byref(h)) != 0
    assert ffi.lib().fvhip_create(ctypes.byref(mesh.view), ctypes.byref(cfg), 0, None) != 0
    cfg.bc_type = None
    assert ffi.lib().fvhip_create(ctypes.byref(mesh.view), ctypes.byref(cfg), 0, ctypes.byref(h)) != 0
    assert "null argument" in ffi.lib().fvhip_last_error().decode()


def test_partitioned_create_checks_the_partition(mesh):
    cfg, keep = raw_config(cases.physics("naca"), cases.numerics())
    h = ctypes.c_void_p()
    part = np.zeros(mesh.nelem, np.int32)
    part[::2] = 1
    assert ffi.lib().fvhip_create_partitioned(ctypes.byref(mesh.view), ctypes.byref(cfg), fa.iptr(part), 2, 2, 0,
                                              ctypes.byref(h)) != 0
    assert "rank out of range" in ffi.lib().fvhip_last_error().decode()
    part[0] = 5
    assert ffi.lib().fvhip_create_partitioned(ctypes.byref(mesh.view), ctypes.byref(cfg), fa.iptr(part), 2, 0, 0,
                                              ctypes.byref(h)) != 0
    assert "partition entry out of range" in ffi.lib().fvhip_last_error().decode()


@pytest.mark.parametrize("field,name", [("conv_numflux", "SLAU"), ("conv_numflux_jac", "RUSANOV"),
                                        ("reconstruction", "MINMOD")])
def test_python_mirror_names_unknown_schemes(mesh, field, name):
    n = cases.numerics()
    setattr(n, field, name)
    with pytest.raises(ValueError, match=name):
        fa.FlowFV(mesh, cases.physics("naca"), n)


def test_unknown_gradient_scheme_is_zero_gradients():
    """afactory.cpp:123-127: any other gradient name is ZeroGradients, not an error"""
    cfg, keep = fa._config_struct(cases.physics("naca"), cases.numerics("ROE", "SOMETHING", "NONE"))
    assert cfg.gradientscheme == fa.GRADIENTS["ZERO"]


def test_null_handle_is_refused_before_any_access():
    lib = ffi.lib()
    null = ctypes.c_void_p()
    assert lib.fvhip_destroy(null) == 0 and lib.fvhip_group_destroy(null) == 0
    r = np.zeros((4, 4))
    calls = [lambda: lib.fvhip_compute_residual(null, fa.dptr(r), fa.dptr(r), 0, None),
             lambda: lib.fvhip_compute_residual_device(null, None, None, 0, None, 0),
             lambda: lib.fvhip_synchronize(null),
             lambda: lib.fvhip_matfree_set_eps(null, 1e-7),
             lambda: lib.fvhip_tvdrk_device(null, None, 3, 0.5, 1.0, 10, None, None),
             lambda: lib.fvhip_group_compute_residual_device(null, None, None, 0, None, 0)]
    for call in calls:
        assert call() != 0
        assert lib.fvhip_last_error().decode() in ("null handle", "null group")


def test_partition_entries_refuse_null_arrays(mesh):
    """the host partition entry points check their mesh and output arrays before touching them"""
    lib = ffi.lib()
    part = np.zeros(mesh.nelem, np.int32)
    w = np.ones(mesh.nelem, np.int32)
    counts = np.zeros(6, np.int32)
    mv = ctypes.byref(mesh.view)
    calls = [(lambda: lib.fvhip_partition_rcb(None, 2, fa.iptr(part)), "null mesh"),
             (lambda: lib.fvhip_partition_rcb(mv, 2, None), "null part"),
             (lambda: lib.fvhip_partition_graph(None, 2, fa.iptr(part)), "null mesh"),
             (lambda: lib.fvhip_partition_graph(mv, 2, None), "null part"),
             (lambda: lib.fvhip_partition_graph_weighted(None, 2, fa.iptr(w), fa.iptr(part)), "null mesh"),
             (lambda: lib.fvhip_partition_graph_weighted(mv, 2, fa.iptr(w), None), "null part"),
             (lambda: lib.fvhip_partition_info(mv, None, 0, fa.iptr(counts), None, None, None, None, None), "null part"),
             (lambda: lib.fvhip_partition_info(None, fa.iptr(part), 0, fa.iptr(counts), None, None, None, None, None),
              "null mesh"),
             (lambda: lib.fvhip_partition_info(mv, fa.iptr(part), 0, None, None, None, None, None, None), "null counts")]
    for call, msg in calls:
        assert call() != 0
        assert lib.fvhip_last_error().decode() == msg
    assert lib.fvhip_partition_edge_cut(mv, None) == -1
    assert lib.fvhip_last_error().decode() == "null part"
    # and the weighted partition still works with and without weights
    assert lib.fvhip_partition_graph_weighted(mv, 2, fa.iptr(w), fa.iptr(part)) == 0
    assert set(np.unique(part)) == {0, 1}
    assert lib.fvhip_partition_graph_weighted(mv, 2, None, fa.iptr(part)) == 0
