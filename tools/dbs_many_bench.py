"""FFT-mode greedy DBS over several 1024x24 images side by side (dbs.greedy_many(mode="fft"):
one plan, plane cache and HIP stream per image): aggregate candidates/s for 1, 2, 4 and 8
images, 16,384 candidates each.  python tools/dbs_many_bench.py [candidates]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd"))


def main():
    import numpy as np
    import torch
    from hbx import dbs
    from hbx.plan import Plan, pack_bits, rgb_config
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    cfg = rgb_config(1024)
    for k in (1, 2, 4, 8):
        gens = [torch.Generator(device="cuda").manual_seed(100 + i) for i in range(k)]
        masks = [pack_bits(torch.rand((24, 1024, 1024), generator=g, device="cuda") >= 0.5) for g in gens]
        tgts = [torch.rand((3, 1024, 1024), generator=g, device="cuda") for g in gens]
        orders = [np.random.default_rng(3 + i).permutation(24 * 1024 * 1024)[:n] for i in range(k)]
        plans = [Plan(cfg, max_jobs=16) for _ in range(k)]
        dbs.greedy_many(plans, [m.clone() for m in masks], tgts, [o[:512] for o in orders], mode="fft")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = dbs.greedy_many(plans, masks, tgts, orders, mode="fft", concurrency=8)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"{k} image(s): {sum(r.steps for r in res)} candidates in {dt:.3f} s = "
              f"{sum(r.steps for r in res) / dt:.0f}/s aggregate, "
              f"{sum(len(r.accepted_positions) for r in res)} accepts", flush=True)
        for p in plans:
            p.close()
        del plans, masks, tgts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
