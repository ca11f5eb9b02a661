"""DBS_1024_24.py's loop over several images (`:208-211`) end to end: the full greedy
pixel-flip sweep (all 24 x 1024 x 1024 = 25,165,824 candidates) of IMAGES images,
run as side-by-side device walks (hbx.dbs.greedy_many: one plan and HIP stream per
image, exact refresh every 4096 accepts).  Synthetic seeded pre-model / target per
image, order = rng(3 + i).permutation.  A heartbeat line every 20 s, one JSON line
at the end.
python tools/dbs_full_sweep_many.py [images] [n_candidates]"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hbx  # noqa: E402
from hbx import dbs  # noqa: E402

images = int(sys.argv[1]) if len(sys.argv) > 1 else 4
total = 24 * 1024 * 1024
n = int(sys.argv[2]) if len(sys.argv) > 2 else total
cfg = hbx.rgb_config(1024)
plans, masks, tgts, orders = [], [], [], []
for i in range(images):
    g = torch.Generator(device="cuda").manual_seed(i)
    pre = torch.rand((24, 1024, 1024), generator=g, device="cuda")
    tgts.append(torch.rand((3, 1024, 1024), generator=g, device="cuda"))
    masks.append(hbx.pack_bits(pre >= 0.5))
    orders.append(np.random.default_rng(3 + i).permutation(total)[:n])
    plans.append(hbx.Plan(cfg, max_jobs=64))
dbs.greedy(plans[0], masks[0].clone(), tgts[0], orders[0][:4096], mode="psf")   # warm-up
torch.cuda.synchronize()

stop = threading.Event()
t0 = time.perf_counter()


def heartbeat():
    while not stop.wait(20.0):
        print(f"{time.perf_counter() - t0:7.1f} s  {images} walks running", flush=True)


threading.Thread(target=heartbeat, daemon=True).start()
res = dbs.greedy_many(plans, masks, tgts, orders, concurrency=images)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
stop.set()
per = []
for plan, mask, tgt, r in zip(plans, masks, tgts, res):
    _, _, ps = plan.propagate(mask[None], tgt[None], want_intensity=False)
    per.append({"candidates": r.steps, "accepted": len(r.accepted_positions), "initial_psnr": r.initial_psnr,
                "final_psnr": r.final_psnr, "final_psnr_drift_db": abs(float(ps[0]) - r.final_psnr)})
cand = sum(p["candidates"] for p in per)
print(json.dumps({
    "config": f"BASELINE configs[1] over {images} images (DBS_1024_24.py:208-211 image loop): full pixel-flip "
              "sweeps, 1024x1024x24, 1 MI355X, walks side by side",
    "images": images, "candidates": cand, "seconds": round(dt, 2), "candidates_per_s": round(cand / dt, 1),
    "seconds_per_image": round(dt / images, 2), "per_image": per,
    "mode": "hbx.dbs.greedy_many: device-resident walks (hbx_dbs_walk_psf) on their own streams, "
            "exact refresh every 4096 accepts",
    "data": "synthetic seeded U[0,1) pre-model (threshold 0.5) and target per image"}))
