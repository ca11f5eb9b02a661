"""Where the host time of HologramVecEnv.step goes (256x256x8 mono, B = 128, SB3's numpy
actions, all five observations): cProfile over the steps, top functions by own time, plus the
step period without the profiler.

    python tools/step_prof.py [--steps 300] [--format torch|lazy|numpy]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--format", default="torch")
    ap.add_argument("--graph", action="store_true", help="HologramVecEnv(graph=True)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from hbx.env import OBS_KEYS, HologramVecEnv
    from hbx.plan import mono_config
    cfg, n, B = mono_config(256), 256, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    tg = [torch.rand((cfg.groups, n, n), generator=g, device="cuda") for _ in range(B)]
    pm = [torch.rand((cfg.channels, n, n), generator=g, device="cuda") for _ in range(B)]
    vec = HologramVecEnv(cfg, B, lambda i: tg[i], pre_model_source=lambda i: pm[i], obs_keys=OBS_KEYS,
                         obs_format=a.format, auto_reset=True, graph=a.graph)
    vec.reset()
    rng = np.random.default_rng(1)
    acts = rng.integers(0, cfg.channels * n * n, (a.steps + 50, B)).astype(np.int64)
    for k in range(30):
        vec.step(acts[k])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        vec.step(acts[k])
    torch.cuda.synchronize()
    period = (time.perf_counter() - t0) / a.steps * 1e3
    pr = cProfile.Profile()
    pr.enable()
    for k in range(a.steps):
        vec.step(acts[k])
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(f"format {a.format} graph {a.graph}: {period:.4f} ms per step without the profiler")
    print(s.getvalue())


if __name__ == "__main__":
    main()
