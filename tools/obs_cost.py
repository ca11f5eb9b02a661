"""Where the SB3-facing VecEnv.step spends its time over the bare device step.

    python tools/obs_cost.py [N]

(a) step_device, obs_keys=()                     the pure device step (launches back to back)
(b) step_device with every observation buffer kept (the recon / state-byte writes)
(c) VecEnv.step, obs_keys=()                     + the per-step host round trip only
(d) VecEnv.step, every observation               the SB3-facing step
(e) (d) without the settle launch                (the reconcile moves into the next k_rowinv)
(f) (d) with obs_format="lazy", nothing read     (snapshots of the step-mutable keys)
(g) (d) with numpy actions (SB3's form: the host-mapped action row)
(h) (g) replayed from the host-action HIP graph (graph=True)
"""
import os
import statistics
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


def run(keys, full, settle=True, fmt="torch", host=False, graph=False):
    vec = HologramVecEnv(cfg, B, lambda i: tg[i], pre_model_source=lambda i: pm[i], obs_keys=keys,
                         auto_reset=full, max_steps=10 ** 9, refresh_every=0, obs_format=fmt, graph=graph)
    vec.reset()
    if not settle:
        vec._settle = lambda: None
    acts = torch.randint(0, cfg.channels * N * N, (5 * steps + 10, B), device=dev)
    if host:
        acts = acts.cpu().numpy()
    k = 0
    ts = []
    for rep in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            if full:
                vec.step(acts[k])
            else:
                vec.step_device(acts[k])
            k += 1
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) / steps * 1e3)
    vec.close()
    return statistics.median(ts)


res = {"a pure device step": run((), False), "b + obs buffers": run(ALL, False),
       "c VecEnv.step, no obs": run((), True), "d VecEnv.step, all obs": run(ALL, True),
       "e d without settle": run(ALL, True, settle=False), "f d lazy, unread": run(ALL, True, fmt="lazy"),
       "g d, numpy actions": run(ALL, True, host=True), "h g, graph replay": run(ALL, True, host=True, graph=True)}
a = res["a pure device step"]
print(f"N={N}, B={B}, median of 5 x {steps} steps (ms/step, vs a):")
for k, v in res.items():
    print(f"  {k:28s} {v:.4f}  {(v - a) / a * 100:+.1f}%", flush=True)
