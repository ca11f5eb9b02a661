"""BASELINE configs[1] end to end: DBS_1024_24.py's greedy pixel-flip sweep over ALL
24 x 1024 x 1024 = 25,165,824 candidates of one image (synthetic seeded pre-model /
target, order = rng(3).permutation), on the device-resident walk: mode "psf" (the
incremental-field walk, hbx.dbs.greedy mode="psf", exact refresh every 4096 accepts) or "fft"
(the reference's algorithm -- every candidate an f32 re-propagation, on the plane cache with
device-decided batches, hbx_dbs_walk_planes).  Prints a progress line every ~20 s and one JSON
summary line at the end.
python tools/dbs_full_sweep.py [n_candidates] [psf|fft]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hbx  # noqa: E402
from hbx import dbs  # noqa: E402

total = 24 * 1024 * 1024
n = int(sys.argv[1]) if len(sys.argv) > 1 and int(sys.argv[1]) > 0 else total
mode = sys.argv[2] if len(sys.argv) > 2 else "psf"
assert mode in ("psf", "fft")
# optional 3rd argument "ktable=r06": the FFT walk's K policy from the r06 batch times with candidate
# retention (tools/dbs_walk_bench.py --k at q ~ 0.5, profiles/r06/walk_retain_r06af/) instead of r05's
KTABLE = sys.argv[3].split("=", 1)[1] if len(sys.argv) > 3 and sys.argv[3].startswith("ktable=") else "r05"
if KTABLE == "r06":
    _orig_k = dbs.walk_k_planes
    _r06 = {1: 45.0, 2: 56.4, 3: 72.3, 4: 78.4, 5: 91.8, 6: 98.3, 7: 104.4, 8: 110.4}
    dbs.walk_k_planes = lambda q, groups=3, k_min=1, k_max=64, table=None, slope=11.7: _orig_k(
        q, groups, k_min, k_max, table=_r06, slope=6.9)
cfg = hbx.rgb_config(1024)
g = torch.Generator(device="cuda").manual_seed(0)
pre = torch.rand((24, 1024, 1024), generator=g, device="cuda")
tgt = torch.rand((3, 1024, 1024), generator=g, device="cuda")
order = np.random.default_rng(3).permutation(total)[:n]
plan = hbx.Plan(cfg, max_jobs=64)
mask = hbx.pack_bits(pre >= 0.5)
dbs.greedy(plan, mask.clone(), tgt, order[:4096], mode=mode)   # warm-up
torch.cuda.synchronize()
last = [0.0]


def progress(pos, acc, psnr, sec):
    if sec - last[0] >= 20.0:
        last[0] = sec
        print(f"{sec:7.1f} s  pos {pos:>9d} / {n}  accepted {acc:>9d}  psnr {psnr:.6f}  "
              f"{pos / max(sec, 1e-9):.0f} candidates/s", flush=True)


t0 = time.perf_counter()
res = dbs.greedy(plan, mask, tgt, order, mode=mode, progress=progress)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
_, _, ps = plan.propagate(mask[None], tgt[None], want_intensity=False)
exact = float(ps[0])
print(json.dumps({
    "config": "BASELINE configs[1]: DBS_1024_24.py full pixel-flip sweep, 1024x1024x24, 1 MI355X",
    "candidates": res.steps, "accepted": len(res.accepted_positions), "seconds": round(dt, 2),
    "candidates_per_s": round(res.steps / dt, 1), "batches": res.launches,
    "initial_psnr": res.initial_psnr, "final_psnr": res.final_psnr, "final_psnr_exact_repropagation": exact,
    "final_psnr_drift_db": abs(exact - res.final_psnr),
    "mode": ("device-resident walk (hbx_dbs_walk_psf), exact refresh every 4096 accepts" if mode == "psf" else
             "FFT mode (f32 re-propagation per candidate, the reference's algorithm) on the plane cache, "
             "device-decided batches (hbx_dbs_walk_planes)"),
    "k_policy": KTABLE,
    "data": "synthetic seeded U[0,1) pre-model (threshold 0.5) and target"}))
