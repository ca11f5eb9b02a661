"""Per-step cost of a world-1 process group on the 256x256x8 mono env step.

    python tools/pg_overhead.py [none|nccl|gloo] [gather_every]

Times 400 VecEnv.step_device calls (B = 128) three times and prints ms/step.
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "binary-hologram-reinforcement-learning_amd"))
import torch  # noqa: E402

from hbx import dist as hd  # noqa: E402
from hbx.env import HologramVecEnv  # noqa: E402
from hbx.plan import mono_config  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "none"
every = int(sys.argv[2]) if len(sys.argv) > 2 else 0
tevery = int(sys.argv[3]) if len(sys.argv) > 3 else 0     # pass-timing sample stride (0: off)
SPR = int(sys.argv[4]) if len(sys.argv) > 4 else 300       # steps per rep
MJ = int(sys.argv[5]) if len(sys.argv) > 5 else 0          # jobs per launch chunk (0: all)
if mode != "none":
    hd.init(backend=mode, force=True)
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
cfg = mono_config(256)
B = 128
tg = [torch.rand((1, 256, 256), device=dev) for _ in range(B)]
pm = [torch.rand((8, 256, 256), device=dev) for _ in range(B)]
vec = HologramVecEnv(cfg, B, lambda i: tg[i], pre_model_source=lambda i: pm[i], obs_keys=(),
                     auto_reset=False, max_steps=10 ** 9, refresh_every=0, max_jobs=MJ or None)
vec.reset()
acts = torch.randint(0, 8 * 256 * 256, (4 * SPR + 100, B), device=dev)
mg = hd.StepMetricGather(B, every, dev) if every and hd.active() else None
k = 0
for rep in range(4):
    if tevery:
        vec.plan.set_timing(SPR, tevery)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(SPR):
        out = vec.step_device(acts[k])
        if mg is not None:
            mg.add(*out)
        k += 1
    if mg is not None:
        mg.flush()
    torch.cuda.synchronize()
    if tevery:
        tm = vec.plan.read_timing()
    if rep:
        print(f"{mode} every={every} timing={tevery} rep{rep}: {(time.perf_counter() - t0) / SPR * 1e3:.4f} ms/step", {k: round(v[0] / max(v[1], 1), 4) for k, v in tm.items()} if tevery else "", flush=True)
vec.close()
hd.shutdown()
