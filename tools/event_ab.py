"""Same-process A/B of the envs' readback wait: a timing-free HIP event recorded on the raw
stream handle through ctypes (HipEvent below; r06w's variant) against torch.cuda.Event,
alternated, on the drop-in BinaryHologramEnv (B = 1, 1024x24 and 256x8) and the SB3 VecEnv step
(256x8, B = 128).  Prints one JSON line per case.

    python tools/event_ab.py [--reps 4]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd"))


class HipEvent:
    """hipEventCreateWithFlags(DisableTiming) / hipEventRecord(raw stream) / hipEventSynchronize
    through the HIP runtime this process already loaded (libamdhip64.so.7)."""

    def __init__(self):
        import ctypes as C
        self.rt = C.CDLL("libamdhip64.so.7", mode=C.RTLD_GLOBAL)
        self.rt.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
        self.rt.hipEventSynchronize.argtypes = [C.c_void_p]
        self.h = C.c_void_p()
        assert self.rt.hipEventCreateWithFlags(C.byref(self.h), 2) == 0

    def record(self, stream=None):
        import torch
        self.rt.hipEventRecord(self.h, torch._C._cuda_getCurrentRawStream(torch.cuda.current_device()))

    def synchronize(self):
        self.rt.hipEventSynchronize(self.h)


class TorchEvent:
    """torch.cuda.Event behind HipEvent's interface (the r05 readback)."""

    def __init__(self):
        import torch
        self.ev = torch.cuda.Event()

    def record(self, stream=None):
        self.ev.record()

    def synchronize(self):
        self.ev.synchronize()

    def query(self):
        return self.ev.query()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    import numpy as np
    import torch
    from hbx.env import OBS_KEYS, BinaryHologramEnv, HologramVecEnv
    from hbx.plan import mono_config, rgb_config

    def dropin(N, G, steps=300):
        cfg = mono_config(N) if G == 1 else rgb_config(N)
        pre = np.random.default_rng(0).random((cfg.channels, N, N), np.float32)
        tgt = np.random.default_rng(1).random((G, N, N), np.float32)
        env = BinaryHologramEnv(lambda t: torch.from_numpy(pre[None]).to(t.device),
                                [(torch.from_numpy(tgt[None]), ["synthetic.png"])], max_steps=10 ** 9,
                                T_PSNR=1e9, T_PSNR_DIFF=1e9, config=cfg, verbose=False)
        env.reset()
        acts = np.random.default_rng(2).integers(0, cfg.channels * N * N, steps + 20).tolist()
        return env, acts

    out = {}
    cases = {"dropin_1024x24": dropin(1024, 3), "dropin_256x8": dropin(256, 1)}
    cfg = mono_config(256)
    g = torch.Generator(device="cuda").manual_seed(0)
    tg = [torch.rand((1, 256, 256), generator=g, device="cuda") for _ in range(128)]
    pm = [torch.rand((8, 256, 256), generator=g, device="cuda") for _ in range(128)]
    vec = HologramVecEnv(cfg, 128, lambda i: tg[i], pre_model_source=lambda i: pm[i], obs_keys=OBS_KEYS,
                         obs_format="torch", auto_reset=True)
    vec.reset()
    vacts = np.random.default_rng(1).integers(0, cfg.channels * 256 * 256, (320, 128)).astype(np.int64)
    for name in list(cases) + ["vecenv_256x8"]:
        res = {"hip": [], "torch": []}
        for r in range(a.reps):
            for kind in ("hip", "torch"):
                ev = HipEvent() if kind == "hip" else TorchEvent()
                if name == "vecenv_256x8":
                    vec._readback = ev
                    for k in range(20):
                        vec.step(vacts[k])
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for k in range(20, 320):
                        vec.step(vacts[k])
                    res[kind].append((time.perf_counter() - t0) / 300 * 1e3)
                else:
                    env, acts = cases[name]
                    env._vec._readback = ev
                    for x in acts[:20]:
                        env.step(x)
                    t0 = time.perf_counter()
                    for x in acts[20:]:
                        env.step(x)
                    res[kind].append((time.perf_counter() - t0) / (len(acts) - 20) * 1e3)
        out[name] = {k: [round(v, 4) for v in vals] for k, vals in res.items()}
        print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
