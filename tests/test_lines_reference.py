"""The reference's line finder (mesh/meshordering.cpp:143-264, computeWeights + findLines; the lines
its line orderings and line-based preconditioning start from), restated in partition.cpp
(`fvhip_find_lines`), against the reference's own known answer MeshUtils_findLines_smallmesh
(tests/mesh/CMakeLists.txt:35-40, tests/mesh/testlineordering.cpp): testanisotropic.msh with threshold
10 must give exactly the lines of testanisotropic-lines.txt, whose entries are gmsh element numbers
(cell + nbface + 1, testlineordering.cpp:73). Both files are the reference's, copied as fixtures. No GPU."""
import os

import numpy as np

import cases
import fvens_amd as fa

HERE = os.path.dirname(os.path.abspath(__file__))


def golden_lines():
    with open(os.path.join(HERE, "fixtures", "testanisotropic-lines.txt")) as f:
        return [[int(x) for x in ln.split()] for ln in f if ln.strip()]


def test_find_lines_smallmesh():
    m = fa.UMesh.read_gmsh(cases.fixture_mesh("testanisotropic"))
    lines = fa.find_lines(m, 10.0)
    assert [list(map(int, ln + m.nbface + 1)) for ln in lines] == golden_lines()


def test_find_lines_properties():
    """on a wall-resolved O-grid: lines start at boundary cells, are face-connected and disjoint; a
    threshold above every ratio finds none"""
    m = fa.UMesh.naca_ogrid(64, 12, 8, 20.0, 1e-4)
    nb = m.nbface
    esuel = m.esuel
    lines = fa.find_lines(m, 4.0)
    assert len(lines) > 0
    seen = np.concatenate(lines)
    assert len(np.unique(seen)) == len(seen)                   # disjoint
    bcells = set(m.intfac[:nb, 0].tolist())
    for ln in lines:
        assert len(ln) >= 2 and int(ln[0]) in bcells
        for a, b in zip(ln[:-1], ln[1:]):
            assert b in esuel[a]                               # face neighbours
    assert fa.find_lines(m, 1e30) == []
