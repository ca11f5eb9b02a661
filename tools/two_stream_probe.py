"""Do pass tails matter at 1024x24?  128 envs stepped as one batch on one stream against two
64-env VecEnvs (own plans) stepped on two HIP streams, each stream's launches overlapping the
other's pass boundaries.  python tools/two_stream_probe.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd"))


def main():
    import torch
    from hbx.env import HologramVecEnv
    from hbx.plan import rgb_config
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    cfg, N = rgb_config(1024), 1024
    g = torch.Generator(device="cuda").manual_seed(0)
    tg = [torch.rand((3, N, N), generator=g, device="cuda") for _ in range(128)]
    pm = [torch.rand((24, N, N), generator=g, device="cuda") for _ in range(128)]

    def make(lo, n):
        v = HologramVecEnv(cfg, n, lambda i: tg[lo + i], pre_model_source=lambda i: pm[lo + i], obs_keys=(),
                           auto_reset=False, max_steps=10 ** 9, refresh_every=0)
        v.reset()
        return v
    acts = torch.randint(0, 24 * N * N, (steps + 3, 128), generator=g, device="cuda")
    one = make(0, 128)
    for k in range(3):
        one.step_device(acts[k])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(3, steps + 3):
        one.step_device(acts[k])
    torch.cuda.synchronize()
    dt1 = time.perf_counter() - t0
    one.close()
    del one
    torch.cuda.empty_cache()
    a, b = make(0, 64), make(64, 64)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for k in range(3):
        with torch.cuda.stream(sa):
            a.step_device(acts[k, :64])
        with torch.cuda.stream(sb):
            b.step_device(acts[k, 64:])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(3, steps + 3):
        with torch.cuda.stream(sa):
            a.step_device(acts[k, :64])
        with torch.cuda.stream(sb):
            b.step_device(acts[k, 64:])
    torch.cuda.synchronize()
    dt2 = time.perf_counter() - t0
    print(f"one stream x 128 envs: {128 * steps / dt1:.0f} env-steps/s ({dt1 / steps * 1e3:.3f} ms/step); "
          f"two streams x 64 envs: {128 * steps / dt2:.0f} env-steps/s ({dt2 / steps * 1e3:.3f} ms/step)")


if __name__ == "__main__":
    main()
