"""Bitwise A/B of two libhbx builds on the FFT-mode propagation (the library under test is chosen
by HBX_LIB at import, so each build runs in its own process):
  HBX_LIB=.../libhbx.so         python tools/lib_bitcmp.py dump a.npz
  HBX_LIB=.../libhbx_exp_X.so   python tools/lib_bitcmp.py dump b.npz
  python tools/lib_bitcmp.py cmp a.npz b.npz
dump: seeded 1024x1024x24 RGB (4 envs), 256x256x8 mono (8 envs), 896 RGB, binary-phase fields and the
bf16 / fp16 intermediate-storage study -> group intensities, per-channel statistics and PSNR of
hbx_propagate."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "binary-hologram-reinforcement-learning_amd"))
import numpy as np  # noqa: E402


def dump(path):
    import torch
    from hbx import pack_bits
    from hbx.plan import Plan, mono_config, rgb_config
    out = {}
    from hbx import FIELD_PHASE, PRECISION_BF16_STORE, PRECISION_F16_STORE, PRECISION_F32
    cases = (("rgb1024", rgb_config(1024), 4, PRECISION_F32), ("mono256", mono_config(256), 8, PRECISION_F32),
             ("rgb896", rgb_config(896), 2, PRECISION_F32),
             ("rgb1024ph", rgb_config(1024, field_kind=FIELD_PHASE), 2, PRECISION_F32),
             ("mono256ph", mono_config(256, field_kind=FIELD_PHASE), 4, PRECISION_F32),
             ("mono256bf16", mono_config(256), 4, PRECISION_BF16_STORE),
             ("rgb1024f16", rgb_config(1024), 1, PRECISION_F16_STORE))
    for name, cfg, B, prec in cases:
        g = torch.Generator(device="cuda").manual_seed(11)
        ch = cfg.groups * cfg.planes
        n = cfg.height
        pre = torch.rand((B, ch, n, n), generator=g, device="cuda")
        tgt = torch.rand((B, cfg.groups, n, n), generator=g, device="cuda")
        mask = pack_bits(pre >= 0.5)
        plan = Plan(cfg, max_jobs=max(B * cfg.groups, 16), precision=prec)
        inten, st, ps = plan.propagate(mask, tgt, want_intensity=True)
        torch.cuda.synchronize()
        out[name + "_inten"] = inten.cpu().numpy()
        out[name + "_stats"] = st.cpu().numpy()
        out[name + "_psnr"] = ps.cpu().numpy()
        plan.close()
    np.savez(path, **out)
    print("dumped", path, {k: v.shape for k, v in out.items()})


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    ok = True
    for k in A.files:
        same = A[k].tobytes() == B[k].tobytes()
        ok &= same
        print(f"{k:16s} bitwise {'EQUAL' if same else 'DIFFERENT'}  max|d| {np.abs(A[k] - B[k]).max():.3e}")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
