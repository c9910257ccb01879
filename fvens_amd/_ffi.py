"""ctypes binding of libfvhip.so (include/fvhip.h).

This is the Python face of the C-ABI; it mirrors what a reference-side binding would do
(INTEGRATION.md). The library must be present: there is no CPU fallback for the product path.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# FVHIP_LIB selects another build of the library (experiments only); default: the in-tree build
LIB_PATH = os.environ.get("FVHIP_LIB") or os.path.join(_HERE, "libfvhip.so")

c_int_p = ctypes.POINTER(ctypes.c_int)
c_dbl_p = ctypes.POINTER(ctypes.c_double)


class FvMeshView(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("nelem", "npoin", "nbface", "naface", "nconnface", "maxnnode", "maxnfael", "nbtag")] + [
        ("coords", c_dbl_p), ("inpoel", c_int_p), ("nnode", c_int_p), ("esuel", c_int_p),
        ("elemface", c_int_p), ("intfac", c_int_p), ("btags", c_int_p), ("facemetric", c_dbl_p),
        ("area", c_dbl_p), ("rc", c_dbl_p), ("rcbp", c_dbl_p), ("gr", c_dbl_p), ("connface", c_int_p)]


class FvFlowConfig(ctypes.Structure):
    _fields_ = [("gamma", ctypes.c_double), ("Minf", ctypes.c_double), ("Tinf", ctypes.c_double),
                ("Reinf", ctypes.c_double), ("Pr", ctypes.c_double), ("aoa", ctypes.c_double),
                ("viscous_sim", ctypes.c_int), ("const_visc", ctypes.c_int),
                ("conv_numflux", ctypes.c_int), ("conv_numflux_jac", ctypes.c_int),
                ("gradientscheme", ctypes.c_int), ("reconstruction", ctypes.c_int),
                ("limiter_param", ctypes.c_double), ("order2", ctypes.c_int), ("nbc", ctypes.c_int),
                ("bc_type", c_int_p), ("bc_tag", c_int_p), ("bc_vals", c_dbl_p), ("fast_math", ctypes.c_int)]


class FvImplicitConfig(ctypes.Structure):
    _fields_ = [("cflinit", ctypes.c_double), ("cflfin", ctypes.c_double), ("tol", ctypes.c_double),
                ("maxiter", ctypes.c_int), ("matrix_free", ctypes.c_int), ("mf_eps", ctypes.c_double),
                ("lin_rtol", ctypes.c_double), ("lin_maxit", ctypes.c_int), ("restart", ctypes.c_int),
                ("prec_sweeps", ctypes.c_int), ("min_relax", ctypes.c_double),
                ("prec_single", ctypes.c_int), ("prec_gs", ctypes.c_int), ("prec_lines", ctypes.c_int),
                ("line_threshold", ctypes.c_double), ("prec_ilu", ctypes.c_int), ("cgs_refine", ctypes.c_int),
                ("prec_amg", ctypes.c_int), ("amg_sweeps", ctypes.c_int), ("amg_coarse_sweeps", ctypes.c_int),
                ("amg_threshold", ctypes.c_double), ("amg_fine_sweeps", ctypes.c_int), ("resume_res0", ctypes.c_double), ("resume_res", ctypes.c_double),
                ("resume_res_prev", ctypes.c_double), ("resume_cfl", ctypes.c_double)]


class FvSolveStats(ctypes.Structure):
    _fields_ = [("steps", ctypes.c_int), ("converged", ctypes.c_int), ("lin_iters", ctypes.c_int),
                ("resratio", ctypes.c_double), ("cfl", ctypes.c_double), ("lin_unconverged", ctypes.c_int),
                ("lin_worst", ctypes.c_double)]


_vpp = ctypes.POINTER(ctypes.c_void_p)

# name -> (restype, argtypes); kept in sync with include/fvhip.h (tests check every symbol)
_SIGS = {
    "fvhip_last_error": (ctypes.c_char_p, []),
    "fvhip_version": (ctypes.c_char_p, []),
    "fvhip_device_count": (ctypes.c_int, []),
    "fvhip_create": (ctypes.c_int, [ctypes.POINTER(FvMeshView), ctypes.POINTER(FvFlowConfig), ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_void_p)]),
    "fvhip_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "fvhip_set_rank": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "fvhip_partition_rcb": (ctypes.c_int, [ctypes.POINTER(FvMeshView), ctypes.c_int, c_int_p]),
    "fvhip_partition_graph": (ctypes.c_int, [ctypes.POINTER(FvMeshView), ctypes.c_int, c_int_p]),
    "fvhip_partition_graph_weighted": (ctypes.c_int, [ctypes.POINTER(FvMeshView), ctypes.c_int, c_int_p, c_int_p]),
    "fvhip_partition_edge_cut": (ctypes.c_longlong, [ctypes.POINTER(FvMeshView), c_int_p]),
    "fvhip_partition_info": (ctypes.c_int, [ctypes.POINTER(FvMeshView), c_int_p, ctypes.c_int, c_int_p, c_int_p,
                                            c_int_p, c_int_p, c_int_p, c_int_p]),
    "fvhip_partition_halo_layers": (ctypes.c_int, [ctypes.POINTER(FvMeshView), c_int_p, ctypes.c_int, c_int_p,
                                                   c_int_p]),
    "fvhip_create_partitioned": (ctypes.c_int, [ctypes.POINTER(FvMeshView), ctypes.POINTER(FvFlowConfig), c_int_p,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_void_p)]),
    "fvhip_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "fvhip_comm_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "fvhip_group_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_void_p)]),
    "fvhip_group_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "fvhip_build_info": (ctypes.c_char_p, []),
    "fvhip_divsqrt_probe": (ctypes.c_int, [ctypes.c_int, c_dbl_p, c_dbl_p, c_dbl_p]),
    "fvhip_trace_exchange_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "fvhip_group_trace_exchange_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                                         ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]),
    "fvhip_group_compute_residual_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                                           ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                                           ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]),
    "fvhip_compute_residual": (ctypes.c_int, [ctypes.c_void_p, c_dbl_p, c_dbl_p, ctypes.c_int, c_dbl_p]),
    "fvhip_compute_residual_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_int]),
    "fvhip_get_gradients": (ctypes.c_int, [ctypes.c_void_p, c_dbl_p, c_dbl_p]),
    "fvhip_surface_data_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, c_dbl_p, c_dbl_p,
                                                 c_int_p]),
    "fvhip_entropy_error_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, c_dbl_p]),
    "fvhip_group_entropy_error_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), c_dbl_p]),
    "fvhip_assemble_jacobian": (ctypes.c_int, [ctypes.c_void_p, c_dbl_p, c_dbl_p, c_dbl_p, c_dbl_p]),
    "fvhip_assemble_jacobian_device": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 4),
    "fvhip_add_pseudo_time_term_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p,
                                                         ctypes.c_void_p]),
    "fvhip_block_apply_device": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 5),
    "fvhip_jacobian_pattern": (ctypes.c_int, [ctypes.c_void_p, c_int_p, c_int_p]),
    "fvhip_assemble_jacobian_bsr": (ctypes.c_int, [ctypes.c_void_p, c_dbl_p, c_int_p, c_int_p, c_dbl_p]),
    "fvhip_steady_forward_euler_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double,
                                                         ctypes.c_double, ctypes.c_int, c_int_p, c_dbl_p, c_dbl_p]),
    "fvhip_group_steady_forward_euler_device": (ctypes.c_int, [ctypes.c_void_p, _vpp, ctypes.c_double,
                                                               ctypes.c_double, ctypes.c_int, c_int_p, c_dbl_p,
                                                               c_dbl_p]),
    "fvhip_tvdrk_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_int, c_int_p, c_dbl_p]),
    "fvhip_group_tvdrk_device": (ctypes.c_int, [ctypes.c_void_p, _vpp, ctypes.c_int, ctypes.c_double,
                                                ctypes.c_double, ctypes.c_int, c_int_p, c_dbl_p]),
    "fvhip_steady_backward_euler_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p,
                                                          ctypes.POINTER(FvImplicitConfig),
                                                          ctypes.POINTER(FvSolveStats), c_dbl_p]),
    "fvhip_group_steady_backward_euler_device": (ctypes.c_int, [ctypes.c_void_p, _vpp,
                                                                ctypes.POINTER(FvImplicitConfig),
                                                                ctypes.POINTER(FvSolveStats), c_dbl_p]),
    "fvhip_gmres_blocks_device": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 5 +
                                  [ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_int_p, c_dbl_p]),
    "fvhip_line_precondition_device": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 3 +
                                       [ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "fvhip_lines": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_double, c_int_p, c_int_p, c_int_p, c_int_p]),
    "fvhip_find_lines": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_double, c_int_p, c_int_p, c_int_p, c_int_p]),
    "fvhip_ilu_precondition_device": (ctypes.c_int, [ctypes.c_void_p] * 6),
    "fvhip_amg_precondition_device": (ctypes.c_int, [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                                                         ctypes.c_int, ctypes.c_double, ctypes.c_void_p,
                                                                         ctypes.c_void_p, ctypes.c_void_p]),
    "fvhip_amg_level": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 6),
    "fvhip_colouring": (ctypes.c_int, [ctypes.c_void_p, c_int_p, c_int_p, ctypes.POINTER(ctypes.c_longlong)]),
    "fvhip_group_matfree_set_state_device": (ctypes.c_int, [ctypes.c_void_p, _vpp, _vpp, _vpp]),
    "fvhip_group_matfree_apply_device": (ctypes.c_int, [ctypes.c_void_p, _vpp, _vpp]),
    "fvhip_matfree_set_state": (ctypes.c_int, [ctypes.c_void_p, c_dbl_p, c_dbl_p, c_dbl_p]),
    "fvhip_matfree_apply": (ctypes.c_int, [ctypes.c_void_p, c_dbl_p, c_dbl_p]),
    "fvhip_matfree_set_state_device": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 3),
    "fvhip_matfree_apply_device": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 2),
    "fvhip_matfree_set_eps": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_double]),
    "fvhip_to_internal": (ctypes.c_int, [ctypes.c_void_p, c_dbl_p, ctypes.c_void_p, ctypes.c_int]),
    "fvhip_from_internal": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, c_dbl_p, ctypes.c_int]),
    "fvhip_get_permutation": (ctypes.c_int, [ctypes.c_void_p, c_int_p]),
    "fvhip_device_alloc": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_ulonglong, ctypes.POINTER(ctypes.c_void_p)]),
    "fvhip_device_free": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "fvhip_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "fvhip_stream": (ctypes.c_void_p, [ctypes.c_void_p]),
    "fvhip_profile": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "fvhip_kernel_times": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                          c_dbl_p, c_int_p]),
    "fvhip_layout_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong)]),
    "fvhip_layout_probe": (ctypes.c_int, [ctypes.POINTER(FvMeshView), ctypes.POINTER(FvFlowConfig),
                                          ctypes.POINTER(ctypes.c_longlong)]),
    "fvhip_local_flux": (ctypes.c_int, [ctypes.c_int, c_dbl_p, ctypes.c_int, c_dbl_p, c_dbl_p, c_dbl_p, c_dbl_p]),
    "fvhip_local_flux_jacobian": (ctypes.c_int, [ctypes.c_int, c_dbl_p, ctypes.c_int, c_dbl_p, c_dbl_p, c_dbl_p,
                                                 c_dbl_p, c_dbl_p]),
    "fvmesh_read_gmsh": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]),
    "fvmesh_generate": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double, ctypes.POINTER(ctypes.c_void_p)]),
    "fvmesh_generate_hybrid": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_double, ctypes.c_double, ctypes.POINTER(ctypes.c_void_p)]),
    "fvmesh_write_gmsh": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    "fvmesh_amg_aggregates": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]),
    "fvmesh_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "fvmesh_view": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(FvMeshView)]),
    "fvmesh_partition_trivial": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_int_p]),
    "fvmesh_restrict": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "fvmesh_global_elem_index": (ctypes.c_int, [ctypes.c_void_p, c_int_p]),
    "fvmesh_raw_info": (ctypes.c_int, [ctypes.c_void_p, c_int_p]),
    "fvmesh_raw_arrays": (ctypes.c_int, [ctypes.c_void_p, c_dbl_p, c_int_p, c_int_p, c_int_p]),
}

_lib = None


def lib():
    """Loads libfvhip.so (raises if it has not been built: the product has no fallback)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same soname as
        # /opt/rocm's). Loading torch first makes libfvhip bind to that copy, so a process that also
        # uses torch.cuda / torch.distributed never holds two HSA runtimes.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing; build it with __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if os.environ.get("FVHIP_LIB") and not hasattr(L, name):
                continue      # an older experiment build may lack newer entry points
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def source_hash():
    """sha256 (first 16 hex digits) over the library's sources, in the Makefile's order (SRCHASH):
    sorted csrc/*.hip, *.cpp, *.hpp, then include/fvhip.h"""
    import glob
    import hashlib
    here = os.path.dirname(os.path.abspath(__file__))
    names = sorted(os.path.relpath(p, here) for ext in ("hip", "cpp", "hpp")
                   for p in glob.glob(os.path.join(here, "csrc", "*." + ext)))
    h = hashlib.sha256()
    for n in names:
        with open(os.path.join(here, n), "rb") as f:
            h.update(f.read())
    with open(os.path.join(os.path.dirname(here), "include", "fvhip.h"), "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def build_info():
    """{"library": path, "lib_src_hash": hash the loaded library was built from, "tree_src_hash": hash
    of the sources in this tree, "fresh": whether they agree}"""
    info = lib().fvhip_build_info().decode()
    kv = dict(x.split("=", 1) for x in info.split() if "=" in x)
    tree = source_hash()
    return {"library": LIB_PATH, "lib_src_hash": kv.get("src_sha256_16"), "tree_src_hash": tree,
            "fresh": kv.get("src_sha256_16") == tree, "extra": kv.get("extra", "")}


def check(rc):
    if rc != 0:
        raise RuntimeError(lib().fvhip_last_error().decode())
    return rc


def dptr(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(c_dbl_p)


def iptr(a):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(c_int_p)
