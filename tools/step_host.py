"""Host-side phases of HologramVecEnv.step at 256x256x8 mono, B = 128, all five observations
(the SB3-facing step): per step the launch call, the work before the readback
wait, the wait itself (and how many event queries it took), the post-readback bookkeeping, and
the whole step period, against the bare device step's period.

    python tools/step_host.py [--steps 400]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    args = ap.parse_args()
    import numpy as np
    import torch
    from hbx.env import OBS_KEYS, HologramVecEnv
    from hbx.plan import mono_config
    cfg, n, B = mono_config(256), 256, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    tg = [torch.rand((cfg.groups, n, n), generator=g, device="cuda") for _ in range(B)]
    pm = [torch.rand((cfg.channels, n, n), generator=g, device="cuda") for _ in range(B)]
    vec = HologramVecEnv(cfg, B, lambda i: tg[i], pre_model_source=lambda i: pm[i], obs_keys=OBS_KEYS,
                         obs_format="torch", auto_reset=True, max_steps=10 ** 9, T_PSNR=1e9, T_PSNR_DIFF=1e9,
                         refresh_every=0)
    vec.reset()
    S = args.steps
    acts = torch.randint(0, cfg.channels * n * n, (2 * S + 40, B), generator=g, device="cuda")
    ns = time.perf_counter_ns
    med = lambda v: float(np.median(np.asarray(v))) / 1e3   # noqa: E731

    # 1. the step as VecEnv.step runs it, with stamps
    rec = {k: [] for k in ("launch", "pre_wait", "wait", "post", "period")}
    nq = []
    ev = vec._readback
    for k in range(S + 20):
        t0 = ns()
        vec._fast_step(acts[k])
        t1 = ns()
        obs = vec.observe(stepped=True)
        infos = [{} for _ in range(B)]
        ev.record()
        vec._settle()
        t2 = ns()
        q = 0
        while not ev.query():
            q += 1
        t3 = ns()
        r = vec._h_rew.copy()
        dones = np.logical_or(vec._h_term, vec._h_trunc)
        dones.any()
        t4 = ns()
        if k >= 20:
            rec["launch"].append(t1 - t0); rec["pre_wait"].append(t2 - t1); rec["wait"].append(t3 - t2)
            rec["post"].append(t4 - t3); nq.append(q)
            if k > 20:
                rec["period"].append(t0 - prev)
        prev = t0
    print("instrumented VecEnv.step (us, medians): " +
          "  ".join(f"{k} {med(v):.1f}" for k, v in rec.items()) + f"  queries {np.median(nq):.0f}")

    # 2. the real step() back to back, and with a blocking wait instead of the spin
    for label in ("step() event.synchronize", "step() spin on query"):
        if "spin" in label:
            def spin():
                while not ev.query():
                    pass
            vec._readback = type("E", (), {"record": ev.record, "query": ev.query,
                                           "synchronize": lambda self: spin()})()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(S):
            vec.step(acts[S + k])
        torch.cuda.synchronize()
        print(f"{label}: {(time.perf_counter() - t0) / S * 1e3:.4f} ms/step")
        vec._readback = ev
    # 3. the bare device step (no host wait)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(S):
        vec.step_device(acts[k])
    torch.cuda.synchronize()
    print(f"step_device (no wait, obs buffers kept): {(time.perf_counter() - t0) / S * 1e3:.4f} ms/step")
    # 4. the launch call alone when the GPU is busy (queue not empty)
    t = []
    for k in range(S):
        a = ns()
        vec._fast_step(acts[k])
        t.append(ns() - a)
    torch.cuda.synchronize()
    print(f"launch call with a busy queue: {med(t):.1f} us")
    vec.close()


if __name__ == "__main__":
    main()
