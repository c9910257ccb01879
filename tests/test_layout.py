"""Host-only checks of the device layout (fvhip_layout_probe, no GPU): the fused residual stages
every cell a patch reads -- patch cells, ring 1 (far side of the cut faces) and ring 2 (the other
neighbours of the owned ring-1 cells) -- within its LDS budget."""
import fvens_amd as fa
import cases


def _probe(mesh, kind="naca", rec="VANALBADA"):
    return fa.layout_probe(mesh, cases.physics(kind), cases.numerics("ROE", "LEASTSQUARES", rec))


def test_fused_layout_stages_ring_two():
    m = fa.UMesh.naca_ogrid(256, 16, 48, 20.0, 1e-5)
    st = _probe(m)
    assert st["cells"] == m.nelem and st["faces"] == m.naface
    assert st["ring1_cells"] > 0 and st["ring2_cells"] > 0
    # a patch never stages more rows than its LDS budget (slots * 11/8 rows of 112 B)
    assert st["max_staged_cells"] <= st["slots_per_patch"] * 11 // 8
    assert st["max_slots"] <= st["slots_per_patch"]
    # every face is in at least one patch; cut faces in two
    assert m.naface <= st["slots"] < 2 * m.naface


def test_staged_layout_has_no_fused_rows():
    m = fa.UMesh.naca_ogrid(128, 8, 24, 20.0, 1e-5)
    st = _probe(m, rec="WENO")      # staged path (WENO gradients): no fused staging lists
    assert st["ring1_cells"] == 0 and st["ring2_cells"] == 0 and st["max_staged_cells"] == 0


def test_fixture_mesh_layout():
    m = fa.UMesh.read_gmsh(cases.fixture_mesh("naca0012luo"))
    st = _probe(m)
    assert st["cells"] == m.nelem
    assert st["patches"] >= (m.naface + st["slots_per_patch"] - 1) // st["slots_per_patch"]
