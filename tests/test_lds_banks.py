"""CPU check of the LDS layouts of csrc/sa_bwd.hip's sa_dy9 kernel: every access
pattern of their swizzled / padded images is free of bank conflicts under the lane groups of
MI355X_MICROARCH.md §LDS (tools/lds_banks_dy9.py enumerates them), and the swizzles are
bijections."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool():
    spec = importlib.util.spec_from_file_location("lds_banks_dy9",
                                                  os.path.join(ROOT, "tools", "lds_banks_dy9.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_sa_bwd_lds_images_conflict_free():
    res = _tool().main()
    assert len(res) >= 8
    assert all(v == 0 for v in res.values()), res


def test_swizzles_match_kernel_formulas():
    t = _tool()
    # csrc/sa_bwd.hip dsw / zsw, restated: the 8-row piece swizzle moves bits 1-3 of the line
    # index and folds bit 4 into bit 0; zsw swaps the two 2-bit fields of the row's low nibble
    assert [t.dsw(n) for n in range(8)] == [0, 1, 8, 9, 2, 3, 10, 11]
    assert t.dsw(16) == 1 and t.dsw(17) == 0
    assert [t.zsw(r) for r in range(6)] == [0, 4, 8, 12, 1, 5]


def test_sa_dy2_lds_images_conflict_free():
    """csrc/sa_bwd.hip sa_dy2_fused (round 6): the swizzled Ds / As images and the 66-dword Ys
    rows leave every access of the kernel conflict-free (the padded round-5 rows did not)"""
    t = _tool()
    res = t.dy2_census(True)
    assert len(res) == 4 and all(v == 0 for v in res.values()), res
    assert sum(t.dy2_census(False).values()) > 0
    assert [t.asw(r) for r in range(8)] == [0, 0, 4, 4, 0, 0, 4, 4]


def test_attention_tile_images_conflict_free():
    """csrc/attn.hip (round 6): the swizzled K / V / Q / dO images serve the row reads, the
    transposed v_operand reads and the tile stores without bank conflicts (the padded 72-element
    rows left the transposed reads 2-way)"""
    t = _tool()
    assert all(v == 0 for v in t.attn_census(True).values())
    assert t.attn_census(False)["transposed reads"] > 0
    assert [t.isw(r) for r in range(8)] == [0, 0, 4, 4, 1, 1, 5, 5]


def test_rows256_tile_image_conflict_free():
    """csrc/rows256.hip: the row & 15 chunk swizzle serves every 16-lane group of the fragment
    reads from distinct banks (plain 512-byte rows would put all 16 rows on the same banks)"""
    t = _tool()
    assert t.rows256_census(True) == 0
    assert t.rows256_census(False) > 0
