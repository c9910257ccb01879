"""The aggregation multigrid's host setup (amg.cpp amgCoarsen, fvhip_implicit_config::prec_amg; the device
counterpart of testcases/visc-naca0012/mgopts.solverc's GAMG), on the CPU through fvmesh_amg_aggregates: the first
coarsening of a mesh's cell graph (couplings face length / centre distance, strong when at least the threshold
times both cells' strongest). The device's coarse operators themselves are checked against scipy's P^T A P in
tests/test_gpu_implicit.py::test_amg_galerkin_operators_and_cycle."""
import numpy as np
import pytest
import scipy.sparse as sp
from scipy.sparse.csgraph import connected_components

import fvens_amd as fa


def _graph(m):
    F = m.intfac[m.nbface:m.naface - m.nconnface]
    L, R = F[:, 0], F[:, 1]
    keep = R < m.nelem
    return L[keep], R[keep]


@pytest.mark.parametrize("mesh", ["hybrid", "plate", "cylinder"])
def test_aggregates_partition_the_cells(mesh):
    """every cell in exactly one aggregate, every aggregate non-empty and connected over interior faces, the
    level at least 1.25 times smaller (the device stops coarsening otherwise), the same aggregates on a second call"""
    m = {"hybrid": lambda: fa.UMesh.naca_hybrid(192, 24, 48, 128, 20.0, 1e-5),
         "plate": lambda: fa.UMesh.flat_plate(64, 48),
         "cylinder": lambda: fa.UMesh.cylinder_ogrid(48, 12)}[mesh]()
    n, agg = m.amg_aggregates(0.2)
    assert agg.min() == 0 and agg.max() == n - 1 and len(np.unique(agg)) == n
    assert n * 5 <= m.nelem * 4, (n, m.nelem)
    L, R = _graph(m)
    same = agg[L] == agg[R]
    G = sp.csr_matrix((np.ones(int(same.sum())), (L[same], R[same])), shape=(m.nelem, m.nelem))
    ncomp, lab = connected_components(G, directed=False)
    assert ncomp == n                                    # one component per aggregate
    assert len(np.unique(np.stack([lab, agg], 1), axis=0)) == n   # ... and each component is one aggregate
    n2, agg2 = m.amg_aggregates(0.2)
    assert n2 == n and np.array_equal(agg, agg2)


def test_boundary_layer_semi_coarsening():
    """on the flat plate's wall-clustered quadrangles (first height 1e-4 of a 0.5 high box, 64 columns) the strong
    couplings are wall-normal, so the aggregates of the boundary layer are pieces of cell columns: every aggregate
    of the lowest quarter of the rows lies in one column; with threshold 0 (every coupling strong) they do not"""
    nx, ny = 64, 48
    m = fa.UMesh.flat_plate(nx, ny)
    i, j = np.arange(m.nelem) % nx, np.arange(m.nelem) // nx
    for thr, columns in ((0.2, True), (0.0, False)):
        n, agg = m.amg_aggregates(thr)
        low = np.zeros(n, bool)
        np.logical_or.at(low, agg, j < ny // 4)
        one_col = np.ones(n, bool)
        first = np.full(n, -1)
        for c in np.argsort(agg, kind="stable"):
            a = agg[c]
            if first[a] < 0:
                first[a] = i[c]
            elif first[a] != i[c]:
                one_col[a] = False
        bl = low & np.array([np.all(j[agg == a] < ny // 4) for a in range(n)])
        assert bl.any()
        assert one_col[bl].all() == columns, (thr, one_col[bl].mean())
