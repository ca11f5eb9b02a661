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


def test_col896_model_matches_r04_counter_and_r05_is_conflict_free():
    """k_col896's 21.1 M SQ_LDS_BANK_CONFLICT cycles per 128-job launch (profiles/pmc_latest_896.json
    before r05): the model puts 94 extra cycles per wave and line on fft896_ns_s2's transposed reads
    (lanes 28..31 on column 0, lane 16's bank) and the H mirror (lane 0 on lane 12's bank), 92 with
    one of the 32 transposed reads issued as ds_read_b64 -- 92 x 4 waves x 7 lines x 8,192 blocks =
    21.1 M, the counter to 0.1 %.  The r05 placement is conflict-free."""
    import lds_swizzle_model as M
    assert M.col896_conflicts("r04") == 94
    per_launch = M.col896_conflicts("r04", b64_reads=1) * 4 * 7 * (128 * 8 * 8)
    assert abs(per_launch - 21088256) / 21088256 < 0.005
    assert M.col896_conflicts("r05") == 0 and M.col896_conflicts("r05", b64_reads=2) == 0


def test_rowfwd896_b128_chunk_reads_conflict_free():
    """r05 k_rowfwd896 reads each 16-B row pair of its plane tile with one ds_read_b128: the
    instruction's 16-lane groups (MI355X_MICROARCH.md LDS table) cover four whole 8-row lines,
    so any swizzle inside a line is conflict-free."""
    import lds_swizzle_model as M
    groups = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
    groups += [[l + 32 for l in g] for g in groups]
    for w in range(4):
        for i in range(7):
            banks_ok = True
            for g in groups:
                used = {}
                for lane in g:
                    c = w * 64 + lane + 256 * i
                    p0 = M.tile896_pos(c // 4, (c % 4) * 2) & ~1
                    for d in range(4):
                        a = 2 * p0 + d
                        used.setdefault(a % 64, set()).add(a)
                banks_ok &= max(len(v) for v in used.values()) == 1
            assert banks_ok, (w, i)


def test_rowfwd32_mirror_paired_order():
    """r05 k_rowfwd32: the second FFT stage reads column kMirrorK1[t] of the transposed tile, so
    the Hermitian split's mirror partner is lane t ^ 1 (DPP) instead of lane 32 - t (ds_bpermute).
    The order must pair k1 with 32 - k1 on lanes (2m, 2m + 1) and keep the plane-tile writes as
    conflict-free as the natural order; it must also match the table compiled into the kernels."""
    import re
    import lds_swizzle_model as M
    assert M.mirror_pair_order_ok()
    assert M.rowfwd32_tile_write_conflicts(lambda t: M.MIRROR_K1[t]) == 0
    assert M.rowfwd32_tile_write_conflicts(lambda t: t) == 0
    hdr = open(os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd", "csrc", "hbx_fft.hpp")).read()
    body = hdr[hdr.index("kMirrorK1[32] = {"):]
    table = [int(v) for v in re.findall(r"\d+", body[body.index("{") + 1:body.index("}")])]
    assert table == M.MIRROR_K1


def test_rowfwd16_b128_chunk_reads_conflict_free():
    """r05 k_rowfwd<16, 256> (N = 256): each 16-B row pair of the 16-row plane tile is read with
    one ds_read_b128 (the tile_pos<16, 16> swizzle XORs whole pairs) -- conflict-free, where the
    r04 reads were 2-way: 128 extra cycles per workgroup and row block in the model if all 16 were
    ds_read_b64 (the compiler emitted 12 of them plus two ds_read2st64_b64; the counter gave 0.79 M
    per 128-job launch, profiles/r05/prof_mono_r05t -- the model does not reproduce that figure)."""
    import lds_swizzle_model as M
    assert M.rowfwd16_chunk_read_conflicts("b64") > 0
    assert M.rowfwd16_chunk_read_conflicts("b128") == 0
    # every chunk pair is one aligned 16-B pair of the tile (the b128 read's precondition)
    for line in range(256):
        for r2 in range(0, 16, 2):
            p0, p1 = M.tile_pos_16(line, r2), M.tile_pos_16(line, r2 + 1)
            assert p0 // 2 == p1 // 2 and p0 != p1
