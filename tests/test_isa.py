"""ISA-level guard on the gfx950 code of every product kernel (CPU: hipcc cross-compiles).

r03: the bf16 / fp16 study variants of k_col2<32> were non-deterministic at N = 1024 because the
compiler placed a VALU write of a 128-bit store's data VGPR right behind the store
(`buffer_store_dwordx4 v[0:3] ... nt` -> `v_bfe_u32 v0, ...`; profiles/archive/r03/bf16_determinism_r03f.txt,
DESIGN.md 4g).  tools/hazard_scan.py finds such pairs; the product code must have none."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(not os.path.exists(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")) and not shutil.which("hipcc"),
                    reason="hipcc not available")
def test_no_store_data_overwrite_in_device_code(tmp_path):
    import hazard_scan
    files = hazard_scan.compile_all(str(tmp_path))
    hits = [h for f in files for h in hazard_scan.scan(f)]
    assert not hits, hits[:5]


def test_scanner_flags_the_r03_pattern(tmp_path):
    import hazard_scan
    s = tmp_path / "k.s"
    s.write_text("_Zk:                       ; @_Zk\n  buffer_store_dwordx4 v[0:3], v168, s[8:11], s1 offen nt\n"
                 "  v_bfe_u32 v0, v4, 16, 1\n"
                 "  buffer_store_dwordx4 v[4:7], v168, s[8:11], 0 offen nt\n  ds_read2st64_b64 v[4:7], v167\n"
                 "  global_store_dwordx4 v1, v[8:11], s[2:3]\n  v_mov_b32_e32 v12, v8\n")
    hits = hazard_scan.scan(str(s))
    rules = sorted(h[4] for h in hits)
    assert rules == ["data-overwrite", "register-soffset"], hits
    assert all(h[0] == "_Zk" for h in hits)
    assert any("v_bfe_u32 v0" in h[3] for h in hits)


def test_scanner_window_is_two_wait_states(tmp_path):
    """gfx940+ needs 2 wait states (the r03 scanner looked at one instruction):
    a VALU write one unrelated instruction behind the store is flagged, one behind `s_nop 1`
    or two unrelated instructions is not; 64-bit VALU destinations count both registers."""
    import hazard_scan
    cases = {
        "one_between": ("  v_mov_b32_e32 v9, 0\n  v_add_f32_e32 v2, v3, v4\n", 1),
        "nop1": ("  s_nop 1\n  v_add_f32_e32 v2, v3, v4\n", 0),
        "nop0": ("  s_nop 0\n  v_add_f32_e32 v2, v3, v4\n", 1),
        "two_between": ("  v_mov_b32_e32 v9, 0\n  s_add_i32 s1, s1, 1\n  v_add_f32_e32 v2, v3, v4\n", 0),
        "b64_dst": ("  v_lshlrev_b64 v[3:4], 1, v[5:6]\n", 1),
        "other_regs": ("  v_add_f32_e32 v20, v3, v4\n  v_add_f32_e32 v21, v3, v4\n", 0),
    }
    for name, (tail, want) in cases.items():
        s = tmp_path / f"{name}.s"
        s.write_text("_Zk:\n  buffer_store_dwordx4 v[0:3], v8, s[4:7], 0 offen\n" + tail)
        got = [h for h in hazard_scan.scan(str(s)) if h[4] == "data-overwrite"]
        assert len(got) == want, (name, got)


def test_scanner_flags_the_iter1_anomaly_pattern(tmp_path):
    """The r03 ITER = 1 k_col2<16> build (wrong B rows in workgroups >= 256): the stage store's
    data VGPR overwritten by the next VALU behind an SGPR-soffset store."""
    import hazard_scan
    s = tmp_path / "i1.s"
    s.write_text("_ZN3hbx6k_col2ILi16ELi0EEEv:\n  buffer_store_dwordx4 v[36:39], v0, s[4:7], s12 offen nt\n"
                 "  buffer_store_dwordx4 v[32:35], v0, s[4:7], s11 offen nt\n  v_add_f32_e32 v32, v3, v20\n")
    hits = hazard_scan.scan(str(s))
    assert sum(h[4] == "register-soffset" for h in hits) == 2
    assert [h[3] for h in hits if h[4] == "data-overwrite"] == ["v_add_f32_e32 v32, v3, v20"]
