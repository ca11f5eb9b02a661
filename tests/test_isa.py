"""ISA-level guard on the gfx950 code of every product kernel (CPU: hipcc cross-compiles).

r03: the bf16 / fp16 study variants of k_col2<32> were non-deterministic at N = 1024 because the
compiler placed a VALU write of a 128-bit store's data VGPR right behind the store
(`buffer_store_dwordx4 v[0:3] ... nt` -> `v_bfe_u32 v0, ...`; profiles/r03/bf16_determinism_r03f.txt,
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
    s.write_text("_Zk:\n  buffer_store_dwordx4 v[0:3], v168, s[8:11], s1 offen nt\n  v_bfe_u32 v0, v4, 16, 1\n"
                 "  buffer_store_dwordx4 v[4:7], v168, s[8:11], s1 offen nt\n  ds_read2st64_b64 v[4:7], v167\n"
                 "  global_store_dwordx4 v1, v[8:11], s[2:3]\n  v_mov_b32_e32 v12, v8\n")
    hits = hazard_scan.scan(str(s))
    assert len(hits) == 1 and "v_bfe_u32 v0" in hits[0][3]
