"""Greedy-DBS FFT-mode candidates/s at 1024 x 24 (BASELINE configs[1], DBS_1024_24.py:313-422) for
the three FFT-mode variants: full re-propagation (planes=False), plane cache with host-decided
batches, plane cache with device-decided batches (the default).  Also the small-launch latency
chain: run under `rocprofv3 --kernel-trace --stats -- python tools/dbs_walk_bench.py --trace` for
per-kernel durations of the device walk.

    python tools/dbs_walk_bench.py [--flips 16384] [--trace]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from hbx import dbs  # noqa: E402
from hbx.plan import Plan, pack_bits, rgb_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flips", type=int, default=16384)
    ap.add_argument("--trace", action="store_true", help="device walk only (for a kernel trace)")
    ap.add_argument("--k", type=int, default=0, help="fixed K for the device walk (0: adaptive)")
    a = ap.parse_args()
    cfg = rgb_config(1024)
    g = torch.Generator(device="cuda").manual_seed(5)
    mask0 = pack_bits(torch.rand((cfg.channels, 1024, 1024), generator=g, device="cuda") >= 0.5)
    target = torch.rand((cfg.groups, 1024, 1024), generator=g, device="cuda")
    order = np.random.default_rng(3).permutation(cfg.channels * 1024 * 1024)[:a.flips]
    plan = Plan(cfg, max_jobs=256)
    variants = [("device_walk", dict())] if a.trace else [
        ("full_repropagation", dict(planes=False, device_walk=False)),
        ("planes_host", dict(planes=True, device_walk=False)),
        ("device_walk", dict())]
    kw = {} if not a.k else {"k_min": a.k, "k_max": a.k}   # a fixed speculation depth
    for name, opts in variants:
        m = mask0.clone()
        dbs.greedy(plan, m.clone(), target, order[:512], **opts)       # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = dbs.greedy(plan, m, target, order, **opts, **kw)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"{name}: {res.steps} candidates in {dt:.3f} s = {res.steps / dt:.1f}/s, "
              f"{len(res.accepted_positions)} accepts, {res.launches} batches "
              f"({dt / max(1, res.launches) * 1e6:.1f} us per batch)", flush=True)
    plan.close()


if __name__ == "__main__":
    main()
