"""k_col2's stage-region placement (hbx_passes.hip col2_pos) against the LDS bank model
(tools/lds_swizzle_model.py, MI355X_MICROARCH.md LDS table).

The model reproduces the r03 counter exactly: 512 extra cycles per block per line set under
the 16-lane / 32-bank service of the ds_read2st64_b64 the compiler emits, x 2 sets x 4 line
iterations x 16,384 blocks = 67,108,864 = profiles/pmc_latest.json's SQ_LDS_BANK_CONFLICT for
k_col (r03l set).  The r04 placement must be conflict-free under both read models and for the
writers."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_r03_placement_reproduces_the_counter():
    import lds_swizzle_model as M
    rd16, rd32, wr = M.col2_stage_conflicts(32, M.col2_pos_r03)
    blocks = 128 * 8 * (512 // (8 * 4))           # jobs x planes x line blocks (ITER 4, 8 groups)
    predicted = rd16 * 2 * 4 * blocks
    assert (rd32, wr) == (0, 0)
    assert predicted == 67108864
    pmc = os.path.join(ROOT, "profiles", "r03_prof_r03l", "pmc_summary.json")
    if os.path.exists(pmc):
        assert json.load(open(pmc))["kernels"]["k_col"]["SQ_LDS_BANK_CONFLICT"] == predicted


def test_r04_placement_is_conflict_free():
    import lds_swizzle_model as M
    for R in (32, 16):
        assert M.col2_stage_conflicts(R, M.col2_pos) == (0, 0, 0), R


def test_r04_placement_is_a_bijection_inside_each_region():
    import lds_swizzle_model as M
    for R in (32, 16):
        N, TL = R * R, 256 // R
        RS = max(R * (R + 1), R * R + 32)
        for sp in range(TL // 2):
            pos = [M.col2_pos(R, sp, y) for y in range(N)]
            assert len(set(pos)) == N and min(pos) >= 0 and max(pos) < RS, (R, sp)


def test_rowfwd896_tile_keyed_on_kx_mod_28():
    """r04 k_rowfwd896: the tile swizzle keyed on kx mod 28 (one lane base for the lane-row
    writes kx = t + 28 k2) loses tile_pos<32, 8>'s write conflicts and keeps the 16-lane
    chunk reads conflict-free."""
    import lds_swizzle_model as M
    wr, rd64, rd16 = M.rowfwd896_tile_conflicts(M.tile896_pos)
    wr0, _, _ = M.rowfwd896_tile_conflicts(M.tile_pos_32_8)
    assert wr == 0 and rd16 == 0 and rd64 <= 16 and wr0 > 0
