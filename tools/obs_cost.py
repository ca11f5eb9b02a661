"""Where the SB3-facing VecEnv.step spends its time over the bare device step.

    python tools/obs_cost.py [N]

(a) step_device, obs_keys=()     (b) step_device with every observation buffer kept
(c) VecEnv.step (host copy of rewards / dones each step, views as observations)
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "binary-hologram-reinforcement-learning_amd"))
import torch  # noqa: E402

from hbx.env import HologramVecEnv  # noqa: E402
from hbx.plan import mono_config, rgb_config  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
cfg = rgb_config(N) if N == 1024 else mono_config(N)
B = 128
dev = torch.device("cuda", 0)
tg = [torch.rand((cfg.groups, N, N), device=dev) for _ in range(B)]
pm = [torch.rand((cfg.channels, N, N), device=dev) for _ in range(B)]
steps = 40 if N == 1024 else 300
ALL = ("state_record", "state", "pre_model", "recon_image", "target_image")


def run(keys, full):
    vec = HologramVecEnv(cfg, B, lambda i: tg[i], pre_model_source=lambda i: pm[i], obs_keys=keys,
                         auto_reset=full, max_steps=10 ** 9, refresh_every=0, obs_format="torch")
    vec.reset()
    acts = torch.randint(0, cfg.channels * N * N, (3 * steps + 10, B), device=dev)
    k = 0
    best = 1e9
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            if full:
                vec.step(acts[k])
            else:
                vec.step_device(acts[k])
            k += 1
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / steps * 1e3)
    vec.close()
    return best


a = run((), False)
b = run(ALL, False)
c = run(ALL, True)
print(f"N={N}: bare {a:.4f}  obs-buffers {b:.4f} (+{(b - a) / a * 100:.1f}%)  "
      f"VecEnv.step {c:.4f} (+{(c - a) / a * 100:.1f}%) ms/step", flush=True)
