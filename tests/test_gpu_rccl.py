"""RCCL inside the library on a one-GPU box: a one-rank communicator.

The multi-rank halo path needs one GPU per rank (RCCL refuses two ranks on one device), so the
exchange itself is covered by the in-process groups (test_gpu_partition.py, test_gpu_implicit.py)
and the gloo protocol test. What one GPU can check is that the library's own communicator comes up
next to PyTorch's RCCL, that every collective the solvers issue on it (the residual-norm
ncclAllReduce of the implicit and explicit solvers, the surface-functional sums) runs, and that a
one-rank partition with a communicator gives the unpartitioned results bit for bit.
"""
import numpy as np
import pytest

import fvens_amd as fa
import cases
from test_gpu_residual import get_mesh

pytestmark = pytest.mark.gpu


def _pair():
    m, _ = get_mesh("naca_small")
    p = cases.physics("naca")
    n = cases.numerics("ROE", "LEASTSQUARES", "VANALBADA")
    one = fa.FlowFV(m, p, n)
    part = fa.FlowFV(m, p, n, partition=np.zeros(m.nelem, np.int32), rank=0)
    part.comm_init(1, 0, fa.comm_unique_id())
    return m, p, one, part


def _dev(a, perm):
    import torch
    return torch.tensor(np.ascontiguousarray(a[perm]), device="cuda")


def _host(d, perm):
    a = d.cpu().numpy()
    out = np.empty_like(a)
    out[perm] = a
    return out


def test_one_rank_communicator_same_bits():
    import torch
    m, p, one, part = _pair()
    u0 = cases.state(m, p, 11)
    p1, p2 = one.permutation(), part.permutation()
    res = []
    for sp, pm in ((one, p1), (part, p2)):
        du = _dev(u0, pm)
        dr = torch.empty_like(du)
        ddt = torch.empty(m.nelem, dtype=torch.float64, device="cuda")
        sp.compute_residual_device(du.data_ptr(), dr.data_ptr(), ddt.data_ptr(), True, True)
        sp.synchronize()
        res.append((_host(dr, pm), _host(ddt, pm)))
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])

    # explicit and implicit solvers: residual norms through ncclAllReduce on the library's communicator
    outs = []
    for sp, pm in ((one, p1), (part, p2)):
        du = _dev(u0, pm)
        steps, ratio, hist = sp.steady_forward_euler_device(du.data_ptr(), 0.5, 0.0, 5)
        cfg = fa.ImplicitConfig(cflinit=5.0, cflfin=5.0, tol=0.0, maxiter=2, lin_rtol=1e-3, lin_maxit=40,
                                restart=20, prec_sweeps=2)
        st, ihist = sp.steady_backward_euler_device(du.data_ptr(), cfg)
        (cl, cdp, cdf), faces = sp.surface_data_device(du.data_ptr(), 2)
        outs.append((_host(du, pm), hist, ihist, st["lin_iters"], (cl, cdp, cdf)))
    a, b = outs
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]) and a[3] == b[3]
    assert np.array_equal(a[0], b[0])
    assert a[4] == b[4]
    one.close()
    part.close()
