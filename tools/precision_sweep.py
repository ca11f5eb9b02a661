"""Intermediate-precision study (SURVEY 8d cfg 5, DBS_ratio_0.5.py).

cfg 5 is the literal reference run: 256x256x8 mono greedy DBS that stops once
the PSNR has risen 0.5 dB (DBS_ratio_0.5.py:204,370-372).  It is run three
times, on libhbx.so (f32 intermediates, the product) and on the timing/precision
builds that round every stored pass intermediate to bf16 / fp16
(`make -C binary-hologram-reinforcement-learning_amd/csrc exp EXP=BF16_STORE`,
`EXP=F16_STORE`).  Reported per variant: flips visited to +0.5 dB, accepts,
the GPU's final PSNR against the float64 oracle's PSNR of the same final mask,
and the first candidate where the accept sequence leaves the f32 one.

A second table checks per-flip sensitivity at the benchmark size (1024x24 RGB):
the trial-flip PSNR change (hbx_eval_flips, one propagation per flip) of 2048
random flips against the all-flip map of the f32 build (correlations, ~1e-8 dB
from the oracle): max error and the fraction of flips whose improve / worsen
decision flips sign.

Each variant runs in its own child process (HBX_LIB selects the library);
the parent touches no GPU.  Output: one JSON document on stdout.
usage: python tools/precision_sweep.py [--out profiles/archive/r01_precision.json]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd")
VARIANTS = {"f32": "libhbx.so", "bf16": "libhbx_exp_BF16_STORE.so", "fp16": "libhbx_exp_F16_STORE.so"}


def worker(out_path: str, map_ref: bool):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG)
    import torch
    import hbx
    from hbx import dbs
    from oracle import hbx_oracle as O

    res = {}
    # cfg 5: 256 mono DBS to +0.5 dB
    ocfg = O.mono_config(256)
    pre, tgt = O.synthetic_inputs(ocfg, 0)
    cfg = hbx.mono_config(256)
    plan = hbx.Plan(cfg, max_jobs=256)
    mask = hbx.pack_bits(torch.from_numpy(pre).cuda() >= 0.5)
    t = torch.from_numpy(tgt).cuda()
    order = np.random.default_rng(3).permutation(ocfg.channels * 256 * 256)
    t0 = time.perf_counter()
    g = dbs.greedy(plan, mask, t, order, stop_diff=0.5, mode="fft")
    torch.cuda.synchronize()
    res["dbs_seconds"] = time.perf_counter() - t0
    acc = np.zeros(len(order), bool)
    acc[g.accepted_positions] = True
    res["dbs_steps"] = g.steps
    res["dbs_initial_psnr"] = g.initial_psnr
    res["dbs_final_psnr"] = g.final_psnr
    final_mask = hbx.unpack_bits(mask, 256).cpu().numpy().astype(np.uint8)
    plan.close()
    # 1024 RGB per-flip sensitivity
    ocfg = O.rgb_config(1024)
    pre, tgt = O.synthetic_inputs(ocfg, 11)
    plan = hbx.Plan(hbx.rgb_config(1024), max_jobs=256)
    bits = hbx.pack_bits(torch.from_numpy(pre).cuda() >= 0.5)
    t = torch.from_numpy(tgt).cuda()
    flips = torch.from_numpy(np.random.default_rng(12).integers(0, 24 * 1024 * 1024, 2048)).cuda()
    _, st, p0 = plan.propagate(bits[None], t[None])
    ps, _ = plan.eval_flips(bits, t, st[0].contiguous(), flips)
    res["flip_base_psnr"] = float(p0[0])
    res["flip_delta"] = (ps - p0[0]).cpu().numpy()
    if map_ref:
        dmap, base = plan.flip_map(bits, t)
        res["map_delta"] = dmap.reshape(-1)[flips].double().cpu().numpy()
        res["map_base"] = float(base.item())
    plan.close()
    np.savez(out_path, accepted=acc, final_mask=final_mask,
             **{k: np.asarray(v) for k, v in res.items()})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worker", nargs=2, metavar=("OUT", "MAPREF"))
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.worker:
        worker(a.worker[0], a.worker[1] == "1")
        return
    sys.path.insert(0, ROOT)
    from oracle import hbx_oracle as O
    tmp = tempfile.mkdtemp()
    runs = {}
    for name, lib in VARIANTS.items():
        path = os.path.join(PKG, "hbx", lib)
        if not os.path.exists(path):
            print(f"skip {name}: {path} not built", file=sys.stderr)
            continue
        out = os.path.join(tmp, f"{name}.npz")
        env = dict(os.environ, HBX_LIB=path)
        r = subprocess.run([sys.executable, __file__, "--worker", out, "1" if name == "f32" else "0"],
                           env=env, timeout=900)
        if r.returncode != 0:
            raise SystemExit(f"variant {name} failed with {r.returncode}")
        runs[name] = dict(np.load(out, allow_pickle=False))
    ocfg = O.mono_config(256)
    prop = O.Propagator(ocfg)
    _, tgt = O.synthetic_inputs(ocfg, 0)
    ref = runs["f32"]
    map_delta = ref["map_delta"]
    report = {"cfg5": {}, "flip_sensitivity_1024": {}}
    for name, r in runs.items():
        m = r["final_mask"]
        inten = prop.all_intensity(m)
        st = np.stack([O.chan_stats(inten[0], tgt[0])])
        oracle_final = prop.psnr(st)
        div = np.nonzero(r["accepted"] != ref["accepted"])[0]
        report["cfg5"][name] = {
            "flips_visited": int(r["dbs_steps"]), "accepted": int(r["accepted"].sum()),
            "seconds": round(float(r["dbs_seconds"]), 3),
            "initial_psnr": float(r["dbs_initial_psnr"]), "final_psnr_gpu": float(r["dbs_final_psnr"]),
            "final_psnr_oracle_f64": float(oracle_final),
            "final_psnr_dev_vs_oracle": float(r["dbs_final_psnr"]) - float(oracle_final),
            "first_divergence_from_f32": int(div[0]) if len(div) else None,
        }
        d = r["flip_delta"]
        err = d - map_delta
        clear = np.abs(map_delta) > 1e-8      # the map's own accuracy
        report["flip_sensitivity_1024"][name] = {
            "flips": int(len(d)), "base_psnr_dev_vs_f32_map": float(r["flip_base_psnr"]) - float(ref["map_base"]),
            "max_abs_err_db": float(np.max(np.abs(err))), "rms_err_db": float(np.sqrt(np.mean(err ** 2))),
            "median_abs_delta_db": float(np.median(np.abs(map_delta))),
            "sign_errors": int(np.sum(np.sign(d[clear]) != np.sign(map_delta[clear]))),
            "sign_error_frac": float(np.mean(np.sign(d[clear]) != np.sign(map_delta[clear]))),
        }
    report["note"] = ("bf16 / fp16 rows are precision builds (each stored pass intermediate rounded); "
                      "the layout stays f32, so only numerics are compared, not speed")
    js = json.dumps(report, indent=1)
    print(js)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js + "\n")


if __name__ == "__main__":
    main()
