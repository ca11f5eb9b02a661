"""Per-flip PSNR change under bf16-rounded intermediates: eval_flips against a direct
propagation of each flipped mask, per size (bench.py precision_sweep's 1024x24 figure).

    python tools/bf16_diag.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd"))

from hbx import pack_bits, PRECISION_BF16_STORE, PRECISION_F32   # noqa: E402
from hbx.plan import Plan, rgb_config                              # noqa: E402


def run(n, k=16):
    cfg = rgb_config(n)
    rng = np.random.default_rng(0)
    pre = torch.from_numpy(rng.random((24, n, n), np.float32)).cuda()
    tgt = torch.from_numpy(rng.random((3, n, n), np.float32)).cuda()
    mask = pack_bits(pre >= 0.5)
    flips = torch.from_numpy(np.random.default_rng(4).integers(0, 24 * n * n, k)).cuda()
    res = {}
    for name, prec in (("f32", PRECISION_F32), ("bf16", PRECISION_BF16_STORE)):
        plan = Plan(cfg, max_jobs=256, precision=prec)
        _, st, p0 = plan.propagate(mask.unsqueeze(0), tgt.unsqueeze(0), want_intensity=False)
        ps, _ = plan.eval_flips(mask, tgt, st[0].contiguous(), flips)
        direct = []
        for f in flips.tolist():
            m = mask.clone().view(-1)
            w, b = divmod(f, 64)
            m[w] ^= (1 << b) if b < 63 else -(1 << 63)
            _, _, pd = plan.propagate(m.view_as(mask).unsqueeze(0), tgt.unsqueeze(0), want_intensity=False)
            direct.append(float(pd[0]))
        res[name] = (float(p0[0]), ps.cpu().numpy(), np.array(direct))
        plan.close()
    f0, fps, fdir = res["f32"]
    b0, bps, bdir = res["bf16"]
    print(f"N={n}: p0 f32 {f0:.9f} bf16 {b0:.9f} (dev {b0 - f0:.3e})")
    print(f"  f32: eval - direct max {np.max(np.abs(fps - fdir)):.3e}; change median {np.median(np.abs(fps - f0)):.3e}")
    print(f"  bf16: eval - direct max {np.max(np.abs(bps - bdir)):.3e}")
    e_eval = (bps - b0) - (fps - f0)
    e_dir = (bdir - b0) - (fdir - f0)
    print(f"  bf16 change err (eval) rms {np.sqrt(np.mean(e_eval ** 2)):.3e}, (direct) rms {np.sqrt(np.mean(e_dir ** 2)):.3e}")
    print(f"  bf16 eval changes {np.round(bps[:6] - b0, 12)}")
    print(f"  f32  eval changes {np.round(fps[:6] - f0, 12)}")


def determinism(n, prec):
    """Is a bf16 group propagation a function of its inputs alone?  The same mask twice in
    one launch, twice in separate launches, and the same flip at several job positions."""
    cfg = rgb_config(n)
    rng = np.random.default_rng(0)
    pre = torch.from_numpy(rng.random((24, n, n), np.float32)).cuda()
    tgt = torch.from_numpy(rng.random((3, n, n), np.float32)).cuda()
    mask = pack_bits(pre >= 0.5)
    plan = Plan(cfg, max_jobs=256, precision=prec)
    _, s1, _ = plan.propagate(mask.unsqueeze(0), tgt.unsqueeze(0), want_intensity=False)
    _, s2, _ = plan.propagate(mask.unsqueeze(0), tgt.unsqueeze(0), want_intensity=False)
    _, s3, _ = plan.propagate(torch.stack([mask, mask, mask]), torch.stack([tgt, tgt, tgt]), want_intensity=False)
    f = torch.tensor([5 * n * n + 77 * n + 300] * 5, device="cuda")
    _, g1 = plan.eval_flips(mask, tgt, s1[0].contiguous(), f)
    print(f"N={n} prec={prec}: launch-to-launch max |d stats| {float((s1 - s2).abs().max()):.3e}; "
          f"env0/env1/env2 of one launch {float((s3[0] - s3[1]).abs().max()):.3e} "
          f"{float((s3[0] - s3[2]).abs().max()):.3e}; one env vs three {float((s1[0] - s3[0]).abs().max()):.3e}")
    print(f"  same flip at 5 job positions: max spread {float((g1 - g1[0]).abs().max()):.3e}; stats {g1[:2].tolist()}")
    plan.close()


if __name__ == "__main__":
    if sys.argv[1:] == ["det"]:
        determinism(1024, PRECISION_BF16_STORE)
        sys.exit(0)
    for n in (256, 1024):
        for prec in (PRECISION_F32, PRECISION_BF16_STORE):
            determinism(n, prec)
    for n in (64, 256, 1024):
        run(n)
