"""Exact field of 16 mono 256x256x8 envs after reset (incremental-mode state), saved as .npy --
for comparing libhbx builds (HBX_LIB=...):  MJ=<jobs per launch> python tools/dump_env_field.py out.npy"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "binary-hologram-reinforcement-learning_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hbx.env import HologramVecEnv  # noqa: E402
from hbx.plan import mono_config  # noqa: E402

cfg = mono_config(256)
g = torch.Generator(device="cuda").manual_seed(3)
B = 16
tg = [torch.rand((1, 256, 256), generator=g, device="cuda") for _ in range(B)]
pm = [torch.rand((8, 256, 256), generator=g, device="cuda") for _ in range(B)]
vec = HologramVecEnv(cfg, B, lambda i: tg[i], pre_model_source=lambda i: pm[i], obs_keys=(), auto_reset=False,
                     mode="psf", max_jobs=int(os.environ.get("MJ", "0")) or None)
vec.reset()
torch.cuda.synchronize()
np.save(sys.argv[1], vec.state.field.cpu().numpy())
