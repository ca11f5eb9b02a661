"""Plane-cached mode vs FFT mode, one step at a time (mono 256, few envs): after each step, the
stepped env's cached planes (through its slot table) against a fresh fill of the same masks.

    python tools/planes_debug.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd"))

import hbx                                   # noqa: E402
from hbx.env import HologramVecEnv           # noqa: E402


def main(N=256, B=4, steps=6):
    cfg = hbx.mono_config(256) if N == 256 else hbx.rgb_config(N)
    g = torch.Generator(device="cuda").manual_seed(3)
    pres = [torch.rand((cfg.channels, N, N), generator=g, device="cuda") for _ in range(B)]
    tgts = [torch.rand((cfg.groups, N, N), generator=g, device="cuda") for _ in range(B)]
    kw = dict(pre_model_source=lambda i: pres[i], auto_reset=False, obs_keys=())
    fft = HologramVecEnv(cfg, B, lambda i: tgts[i], mode="fft", **kw)
    pl = HologramVecEnv(cfg, B, lambda i: tgts[i], mode="planes", **kw)
    ref = HologramVecEnv(cfg, B, lambda i: tgts[i], mode="planes", **kw)
    fft.reset(); pl.reset(); ref.reset()
    CH = cfg.channels
    acts = torch.randint(0, CH * N * N, (steps, B), generator=g, device="cuda")
    for k in range(steps):
        r1 = fft.step_device(acts[k])
        r2 = pl.step_device(acts[k])
        torch.cuda.synchronize()
        acc = fft._acc.clone()
        same_r = torch.equal(fft._reward, pl._reward)
        # fresh fill of the planes env's current masks
        ref.state.mask.copy_(pl.state.mask)
        ref.refresh()
        torch.cuda.synchronize()
        print(f"step {k}: acc {acc.tolist()} reward equal {same_r} "
              f"dr {(fft._reward - pl._reward).abs().max().item():.3e} "
              f"stats equal {torch.equal(fft.state.chan_stats, pl.state.chan_stats)}")
        for b in range(B):
            s = pl.state.plane_slot[b].long()
            got = pl.state.plane_inten[b][s[:CH]]
            want = ref.state.plane_inten[b][:CH]
            bad = [q for q in range(CH) if not torch.equal(got[q], want[q])]
            a = int(acts[k, b]); ch = a // (N * N)
            if bad:
                d = (got - want).abs().amax(dim=(1, 2))
                print(f"   env {b}: action plane {ch}, slots {s.tolist()}, planes differing {bad}, "
                      f"max diff {[f'{float(d[q]):.2e}' for q in bad]}")
        # keep the fft env in lock-step even if they diverge: nothing to do (same actions)


if __name__ == "__main__":
    main(256, 4, 6)
    main(1024, 2, 6)
