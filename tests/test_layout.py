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


def test_fused_row_caps_fit_the_lds_budget():
    """the staged rows per patch fit the LDS each fused instantiation is launched with: inviscid
    unlimited 14-double rows x 284 (five blocks of 31.8 KB per CU), viscous 18-double rows x 284 (the
    per-row temperature terms: four blocks of 40.9 KB), limited 14-double rows x 352 (four of 39.4 KB)"""
    m = fa.UMesh.naca_ogrid(512, 32, 96, 20.0, 1e-5)
    for kind, rec, rows, width, blocks in (("naca", "VANALBADA", 284, 14, 5), ("visc", "VANALBADA", 284, 18, 4),
                                           ("naca", "VENKATAKRISHNAN", 352, 14, 4)):
        st = _probe(m, kind, rec)
        assert 0 < st["max_staged_cells"] <= rows, (kind, rec, st)
        assert blocks * rows * width * 8 <= 160 * 1024
