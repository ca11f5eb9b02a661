"""bench.py -- env-steps/s of the batched 1024x1024x24 hologram VecEnv on MI355X.

Workload (BASELINE.json configs[2]; configs[3] at --gpus 8): 128 independent
environments per GPU, each a 1024x1024 mask of 24 binary planes (3 colour
groups x 8 time-multiplexed planes, 638/515/450 nm, 7.56 um pitch, z = 2 mm),
stepped with one action per env per VecEnv step.  One env-step = decode ->
flip -> re-propagate the touched colour group (8 planes, 2-D FFT ASM) ->
|.|^2 plane mean -> relative PSNR -> reward / accept-rollback / termination
(env.py:154-259; DBS_1024_24.py:313-422).  Synthetic data:
pre_model ~ U[0,1) -> mask = pre >= 0.5, target ~ U[0,1), actions ~ U{0..CH*N^2-1}.

The headline `value` is the FFT mode (the reference's algorithm: the whole
touched colour group is re-propagated every step).  The incremental-field
mode (SURVEY 8d "reported separately") is measured afterwards on the same
workload and reported under `incremental_psf_mode`.

N GPUs: one process per GPU (torchrun), 128 envs per rank (weak scaling), the
per-step rewards / psnr / done flags gathered to rank 0 over RCCL.

Prints ONE JSON line on rank 0 (driver contract), plus `roofline` for the
dominant kernel (live hipEvent timing) and `cpu_baseline` (the float64
numpy oracle timed on this host, rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--envs", type=int, default=128, help="envs per GPU")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--cpu-sample", type=int, default=20,
                    help="env-steps of the numpy oracle timed for cpu_baseline, after 2 warm-ups "
                         "(SURVEY 8d: >= 20; 0 = skip)")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the drop-in single-env lines (dropin_env_256 / dropin_env_1024x24)")
    ap.add_argument("--no-psnr-check", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--no-pg", action="store_true",
                    help="world 1: no process group (by default one is built and the RCCL metric gather runs)")
    ap.add_argument("--no-psf", action="store_true", help="skip the incremental-mode measurement")
    ap.add_argument("--psf-steps", type=int, default=200)
    ap.add_argument("--no-planes", action="store_true", help="skip the plane-cached FFT mode measurement")
    ap.add_argument("--chunk", type=int, default=0,
                    help="jobs per launch sequence (0 = all envs at once)")
    ap.add_argument("--dbs-flips", type=int, default=65536,
                    help="greedy-DBS prefix (flips of the shuffled order) timed on env 0's image, "
                         "SURVEY 8d cfg 2 (0 = skip)")
    ap.add_argument("--no-scipy", action="store_true", help="skip the multi-core scipy CPU baseline")
    ap.add_argument("--no-probe", action="store_true", help="skip the all-flip probe-sweep measurement")
    ap.add_argument("--no-ppo", action="store_true", help="skip the 256x256x8 mono (train-PPO) measurement")
    ap.add_argument("--no-crop", action="store_true",
                    help="skip the 896 x 896 centre-crop line (env_1024_24_128.py:144-149)")
    ap.add_argument("--no-obs", action="store_true",
                    help="skip the SB3-facing step with all five observations (vecenv_step_obs)")
    ap.add_argument("--no-precision", action="store_true",
                    help="skip the fp32-vs-bf16 intermediate-storage deviation (SURVEY 8d cfg 5)")
    ap.add_argument("--gather-every", type=int, default=8,
                    help="steps of per-env metrics per gather to rank 0 (hbx.dist.StepMetricGather; "
                         "the step kernel writes into the gather rows, one dist.gather per K steps)")
    ap.add_argument("--timing-every", type=int, default=4,
                    help="pass-timing hipEvent pairs on every K-th launch of each pass in the timed loop")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """`--gpus N` (N > 1) started without a launcher (no WORLD_SIZE in the environment): run
    `python -m torch.distributed.run --nproc-per-node N ... bench.py <argv>` as a CHILD process
    -- before this process touches torch or the GPU, and never by exec -- relay rank 0's one JSON
    line to stdout (everything else the child prints on stdout goes to stderr) and return the
    child's exit code.  Returns None when this process is already a rank (or N = 1): the bench
    then runs here.  One rank per GPU, 127.0.0.1 rendezvous (train-PPO.py:296-322's 8-GPU
    caller, BASELINE configs[3])."""
    import subprocess
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    print("bench.py: launching " + " ".join(cmd), file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    line = None
    for out in proc.stdout:
        try:
            obj = json.loads(out)
        except ValueError:
            obj = None
        if isinstance(obj, dict) and "metric" in obj:
            line = out.strip()
        else:
            sys.stderr.write(out)
            sys.stderr.flush()
    rc = proc.wait()
    if line is not None:
        print(line, flush=True)
    elif rc == 0:
        print("bench.py: the ranks exited 0 without a JSON line", file=sys.stderr)
        rc = 1
    return rc


def algorithmic_bytes(N: int, P: int):
    """HBM bytes each kernel must move per job (one colour group of one env):
    k_rowfwd: read P*N^2/8 mask bits, write P*N^2/2 complex64 (half spectrum)
    k_col:    read P*N^2/2 complex64, write P*N^2 complex64
    k_rowinv: read P*N^2 complex64 + N^2 f32 target
    k_psf_eval:   read the touched plane's field (8 N^2) + group intensity (4 N^2) + target (4 N^2)
    k_psf_commit: accepted envs only: read + write field and intensity (24 N^2)."""
    return {"k_rowfwd": P * N * N // 8 + P * N * N * 4,
            "k_col": P * N * N * 4 + P * N * N * 8,
            "k_rowinv": P * N * N * 8 + N * N * 4,
            "k_psf_eval": 16 * N * N,
            "k_psf_commit": 24 * N * N}


def plane_cached_bytes(N: int, P: int):
    """HBM bytes per job of the plane-cached FFT mode (ABI v9): the flipped plane's PAIR runs
    k_rowfwd / k_col (2 of the P planes), k_rowinv reads the pair's B planes, the P - 2 cached
    |U_q|^2 planes (f32) and the target channel and writes the pair's fresh |U|^2."""
    return {"k_rowfwd": 2 * N * N // 8 + 2 * N * N * 4,
            "k_col": 2 * N * N * 4 + 2 * N * N * 8,
            "k_rowinv": 2 * N * N * 8 + (P - 2) * N * N * 4 + N * N * 4 + 2 * N * N * 4}


def canonical_step_bytes(N: int, P: int) -> int:
    """SURVEY 8d's canonical bytes per FFT-mode env-step: two complex64 read+write
    round trips per plane + the touched target channel + the bit-packed mask."""
    return P * 4 * (8 * N * N) + 4 * N * N + P * N * N // 8


def cpu_model() -> str:
    """The host CPU's model string (/proc/cpuinfo "model name", what lscpu prints)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def host_cpus() -> int:
    """CPUs this process may run on (the box's share, not the whole machine)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline_scipy(n_steps: int, N: int, workers: int):
    """SURVEY 8d's second CPU figure: the same env-step with scipy.fft complex64
    over `workers` threads (numpy oracle for everything but the transforms)."""
    import numpy as np
    import scipy.fft as sf
    from oracle import hbx_oracle as O
    cfg = O.rgb_config(N)
    pre, tgt = O.synthetic_inputs(cfg, 0)
    h = [cfg.transfer(g).astype(np.complex64) for g in range(cfg.groups)]
    mask = (pre >= 0.5).astype(np.int8)
    rng = np.random.default_rng(2)
    acts = rng.integers(0, cfg.channels * N * N, n_steps + 2)

    def step(a):
        c, r, col = O.decode_action(int(a), N, N)
        mask[c, r, col] ^= 1
        g = c // cfg.planes
        u = mask[g * cfg.planes:(g + 1) * cfg.planes].astype(np.complex64)
        f = sf.ifft2(sf.fft2(u, axes=(-2, -1), workers=workers) * h[g], axes=(-2, -1), workers=workers)
        inten = np.mean(f.real * f.real + f.imag * f.imag, axis=0)
        return O.chan_stats(inten, tgt[g])

    step(acts[0]); step(acts[1])
    t0 = time.perf_counter()
    for a in acts[2:]:
        step(a)
    dt = time.perf_counter() - t0
    return {"value": n_steps / dt, "unit": "env-steps/s", "cores": workers, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus_visible": host_cpus(), "steps": n_steps, "warmup": 2,
            "sample": f"{n_steps} env-steps after 2 warm-ups, scipy.fft complex64 with workers={workers}, {dt:.1f} s"}


def dbs_prefix(cfg, mask, target, n_flips: int):
    """SURVEY 8d cfg 2: greedy DBS (strict accept, DBS_1024_24.py:313-422) over the
    first n_flips of rng(3).permutation(CH*N^2) on one image, speculative batches
    (hbx.dbs.greedy).  Returns flips/s and the extrapolated full-sweep time."""
    import numpy as np
    import torch
    from hbx import dbs
    from hbx.plan import Plan
    from hbx.plan import pack_bits as hbx_pack
    CH, N = cfg.channels, cfg.height
    order = np.random.default_rng(3).permutation(CH * N * N)[:n_flips]
    plan = Plan(cfg, max_jobs=256)
    m = mask.clone()
    dbs.greedy(plan, m.clone(), target, order[:256])          # warm-up (plan tables, kernels)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = dbs.greedy(plan, m, target, order)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rate = res.steps / dt
    out = {"flips": res.steps, "seconds": round(dt, 3), "flips_per_s": round(rate, 1),
           "accepted": len(res.accepted_positions), "launches": res.launches,
           "psnr_gain_db": round(res.final_psnr - res.initial_psnr, 6),
           "full_sweep_extrapolated_s": round(CH * N * N / rate, 1),
           "plane_cache": True,
           "walk": "device-decided (hbx_dbs_walk_planes): per batch the three passes over K candidates' "
                   "flipped pairs + one single-block decision kernel that commits up to G accepts "
                   "(candidates of colour groups no earlier accept of the batch touched); K from the "
                   "running acceptance rate (hbx.dbs.walk_k_planes)",
           "note": "FFT mode, speculative first-improving batches (serial accept sequence), "
                   "prefix of the shuffled order; acceptance is highest at the start of a sweep, "
                   "so the extrapolation is pessimistic.  Candidates propagate only the flipped "
                   "plane's pair against the base state's cached per-plane |U|^2 (hbx_eval_flips_planes, "
                   "the full re-propagation's PSNR bits; full_repropagation below)"}
    # the same greedy with every candidate re-propagating all 8 planes of its group (planes=False)
    nf = min(n_flips, 8192)
    mf = mask.clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rf = dbs.greedy(plan, mf, target, order[:nf], planes=False)
    torch.cuda.synchronize()
    dtf = time.perf_counter() - t0
    kpos = [p for p in res.accepted_positions if p < nf]
    # several images side by side in FFT mode (DBS_1024_24.py loops over a folder, :208-211)
    n_img, n_each = 4, min(n_flips, 16384)
    fplans = [Plan(cfg, max_jobs=16) for _ in range(n_img)]
    fgens = [torch.Generator(device=mask.device).manual_seed(200 + i) for i in range(n_img)]
    fmasks = [hbx_pack(torch.rand((CH, N, N), generator=gg, device=mask.device) >= 0.5) for gg in fgens]
    ftgts = [torch.rand((cfg.groups, N, N), generator=gg, device=mask.device) for gg in fgens]
    forders = [np.random.default_rng(30 + i).permutation(CH * N * N)[:n_each] for i in range(n_img)]
    dbs.greedy_many(fplans, [m.clone() for m in fmasks], ftgts, [o[:256] for o in forders], mode="fft")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fres = dbs.greedy_many(fplans, fmasks, ftgts, forders, mode="fft")
    torch.cuda.synchronize()
    dtf4 = time.perf_counter() - t0
    for pl in fplans:
        pl.close()
    out["several_images"] = {"images": n_img, "flips": sum(r.steps for r in fres), "seconds": round(dtf4, 3),
                             "flips_per_s_aggregate": round(sum(r.steps for r in fres) / dtf4, 1),
                             "accepted": sum(len(r.accepted_positions) for r in fres),
                             "note": "hbx.dbs.greedy_many(mode='fft'): one FFT-mode walk per image (own plan, "
                                     "plane cache and HIP stream), synthetic seeded images"}
    # EXTENSION (BASELINE configs[4]'s "50 % on-pixel constraint"; no reference counterpart):
    # the same prefix under the on-pixel ratio constraint (hbx_dbs_walk_planes_fill)
    mfill = mask.clone()
    dbs.greedy(plan, mfill.clone(), target, order[:256], fill_ratio=0.5, fill_tol=4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rfill = dbs.greedy(plan, mfill, target, order, fill_ratio=0.5, fill_tol=4)
    torch.cuda.synchronize()
    dtfill = time.perf_counter() - t0
    c0 = dbs.fill_counts(mask, cfg.groups, cfg.planes).tolist()
    out["fill_ratio_extension"] = {
        "flips": rfill.steps, "seconds": round(dtfill, 3), "flips_per_s": round(rfill.steps / dtfill, 1),
        "accepted": len(rfill.accepted_positions), "psnr_gain_db": round(rfill.final_psnr - rfill.initial_psnr, 6),
        "fill_ratio": 0.5, "fill_tol": 4, "group_counts_start": c0, "group_counts_end": rfill.fill_counts,
        "target_count": dbs.fill_target(0.5, cfg.planes, N, N),
        "note": "EXTENSION, no reference counterpart (SURVEY F7): greedy(fill_ratio=0.5) -- a candidate that "
                "would move its colour group's on-pixel count away from 50 % by more than fill_tol pixels is "
                "rejected without a propagation (hbx_dbs_walk_planes_fill); tests/test_gpu_fill.py"}
    out["full_repropagation"] = {
        "flips": rf.steps, "seconds": round(dtf, 3), "flips_per_s": round(rf.steps / dtf, 1),
        "same_accepts_and_psnr_bits_as_plane_cache": bool(
            rf.accepted_positions == kpos and rf.accepted_psnr == res.accepted_psnr[:len(kpos)]),
        "note": f"first {nf} candidates of the same prefix, hbx_eval_flips (all P planes per candidate)"}
    m2 = mask.clone()
    dbs.greedy(plan, m2.clone(), target, order[:256], mode="psf")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r2 = dbs.greedy(plan, m2, target, order, mode="psf")
    torch.cuda.synchronize()
    dt2 = time.perf_counter() - t0
    m3 = mask.clone()
    dbs.greedy(plan, m3.clone(), target, order[:256], mode="psf_host")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r3 = dbs.greedy(plan, m3, target, order, mode="psf_host")
    torch.cuda.synchronize()
    dt3 = time.perf_counter() - t0
    a1 = np.zeros(n_flips, bool)
    a2 = np.zeros(n_flips, bool)
    a1[res.accepted_positions] = True
    a2[r2.accepted_positions] = True
    diff = np.nonzero(a1 != a2)[0]
    first_change = None
    if len(diff):
        # both runs saw the same state up to the first differing candidate: replay it with the
        # incremental walk and evaluate that candidate's PSNR change in increment form
        # (resolved to ~1e-12 dB, tests/test_gpu_dbs_headline.py) -- a tie of the FFT mode's
        # f32 resolution (~1e-9 dB per candidate) or a real disagreement
        f = int(diff[0])
        m4 = mask.clone()
        if f > 0:
            dbs.greedy(plan, m4, target, order[:f], mode="psf")
        _, st4, p4 = plan.propagate(m4.unsqueeze(0), target.unsqueeze(0), want_intensity=False)
        fc4, it4 = plan.simulate(m4.unsqueeze(0), want_intensity=True)
        cand = torch.as_tensor(order[f:f + 1]).to(plan.device)
        ps4, _ = plan.eval_flips_psf(m4, target, st4[0].contiguous(), torch.view_as_real(fc4[0]).contiguous(),
                                     it4[0].contiguous(), cand)
        first_change = float((ps4 - p4).item())
    plan.close()
    # several images side by side (DBS_1024_24.py loops over a folder, :208-211): one walk per
    # image, each with its own plan and stream (hbx.dbs.greedy_many)
    n_img = 4
    plans = [Plan(cfg, max_jobs=cfg.groups) for _ in range(n_img)]
    gens = [torch.Generator(device=mask.device).manual_seed(100 + i) for i in range(n_img)]
    masks = [hbx_pack(torch.rand((CH, N, N), generator=gg, device=mask.device) >= 0.5) for gg in gens]
    tgts = [torch.rand((cfg.groups, N, N), generator=gg, device=mask.device) for gg in gens]
    orders = [np.random.default_rng(3 + i).permutation(CH * N * N)[:n_flips] for i in range(n_img)]
    dbs.greedy_many(plans, [m.clone() for m in masks], tgts, [o[:256] for o in orders])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rm = dbs.greedy_many(plans, masks, tgts, orders)
    torch.cuda.synchronize()
    dtm = time.perf_counter() - t0
    for pl in plans:
        pl.close()
    many = {"images": n_img, "flips": sum(r.steps for r in rm), "seconds": round(dtm, 3),
            "flips_per_s_aggregate": round(sum(r.steps for r in rm) / dtm, 1),
            "accepted": sum(len(r.accepted_positions) for r in rm),
            "note": "hbx.dbs.greedy_many: one device walk per image (own plan and HIP stream), same prefix "
                    "length per image, synthetic seeded images"}
    out["incremental_mode"] = {"flips": r2.steps, "seconds": round(dt2, 3),
                               "flips_per_s": round(r2.steps / dt2, 1), "accepted": len(r2.accepted_positions),
                               "same_accepts_as_fft_mode": bool(len(diff) == 0),
                               "first_decision_difference": int(diff[0]) if len(diff) else None,
                               "first_difference_change_db": first_change,
                               "decisions_differing": int(len(diff)),
                               "psnr_gain_db": round(r2.final_psnr - r2.initial_psnr, 6),
                               "full_sweep_extrapolated_s": round(CH * N * N / (r2.steps / dt2), 1),
                               "batches": r2.launches,
                               "several_images": many,
                               "walk": "device-resident (hbx_dbs_walk_psf): one launch per batch for K <= 4 (the previous "
                                       "batch's commits, K candidates with pair terms, last-arriving block decides up to two "
                                       "accepts), three launches for larger K; one host sync per 64 batches",
                               "host_decided_batches": {
                                   "flips_per_s": round(r3.steps / dt3, 1), "seconds": round(dt3, 3),
                                   "batches": r3.launches,
                                   "same_accepts_as_device_walk": r3.accepted_positions == r2.accepted_positions,
                                   "note": "hbx_eval_flips_psf + host decision + hbx_commit_flip_psf per batch"},
                               "note": "a flip moves the 1024x24 PSNR by a median 6.7e-7 dB; the incremental "
                                       "walk resolves a candidate's change to ~1e-12 dB (increment-form f64 "
                                       "sums) and equals the float64 oracle's accept sequence on the committed "
                                       "4096-candidate 1024x24 prefix, while the FFT mode (the reference's "
                                       "algorithm in f32) resolves ~1e-9 dB, so the two can order a near-tie "
                                       "differently (first_difference_change_db), after which the greedy "
                                       "sequences visit different states"}
    return out


def precision_sweep(mask1024, target1024, n_flips: int = 2048, n_constrained: int = 16384):
    """SURVEY 8d cfg 5 (BASELINE configs[4]): DBS_ratio_0.5.py's literal run -- 256x256x8
    mono greedy DBS until the PSNR has risen 0.5 dB (:366-372), FFT mode -- with f32 and
    with bf16-rounded pass intermediates (hbx_plan_set_precision), plus the per-flip PSNR
    change of n_flips random flips of the 1024x24 bench state under both."""
    import numpy as np
    import torch
    from hbx import dbs, pack_bits, PRECISION_BF16_STORE, PRECISION_F32
    from hbx.plan import Plan, mono_config, rgb_config
    mono = mono_config(256)
    pre = np.random.default_rng(0).random((8, 256, 256), np.float32)     # SURVEY 8d seeds
    tgt = np.random.default_rng(1).random((1, 256, 256), np.float32)
    order = np.random.default_rng(3).permutation(8 * 256 * 256)
    runs = {}
    for name, prec in (("f32", PRECISION_F32), ("bf16", PRECISION_BF16_STORE)):
        plan = Plan(mono, max_jobs=256, precision=prec)
        mask = pack_bits(torch.from_numpy(pre).cuda() >= 0.5)
        t0 = time.perf_counter()
        res = dbs.greedy(plan, mask, torch.from_numpy(tgt).cuda(), order, stop_diff=0.5, mode="fft")
        torch.cuda.synchronize()
        runs[name] = (res, time.perf_counter() - t0)
        plan.close()
    (r32, t32), (rbf, tbf) = runs["f32"], runs["bf16"]
    a32 = np.zeros(len(order), bool)
    abf = np.zeros(len(order), bool)
    a32[r32.accepted_positions] = True
    abf[rbf.accepted_positions] = True
    d = np.nonzero(a32 != abf)[0]
    out = {"workload": "DBS_ratio_0.5.py: 256x256x8 mono greedy DBS (seeds 0/1/3) until +0.5 dB, FFT mode",
           "f32": {"candidates": r32.steps, "accepts": len(r32.accepted_positions),
                   "initial_psnr": r32.initial_psnr, "final_psnr": r32.final_psnr, "seconds": round(t32, 3)},
           "bf16_intermediates": {"candidates": rbf.steps, "accepts": len(rbf.accepted_positions),
                                  "initial_psnr": rbf.initial_psnr, "final_psnr": rbf.final_psnr,
                                  "seconds": round(tbf, 3)},
           "initial_psnr_deviation_db": abs(rbf.initial_psnr - r32.initial_psnr),
           "final_psnr_deviation_db": abs(rbf.final_psnr - r32.final_psnr),
           "first_accept_sequence_difference": int(d[0]) if len(d) else None}
    cfg = rgb_config(1024)
    flips = torch.from_numpy(np.random.default_rng(4).integers(0, 24 * 1024 * 1024, n_flips)).cuda()
    deltas = {}
    for name, prec in (("f32", PRECISION_F32), ("bf16", PRECISION_BF16_STORE)):
        plan = Plan(cfg, max_jobs=256, precision=prec)
        _, st, p0 = plan.propagate(mask1024.unsqueeze(0), target1024.unsqueeze(0), want_intensity=False)
        ps, _ = plan.eval_flips(mask1024, target1024, st[0].contiguous(), flips)
        deltas[name] = (ps - p0).cpu().numpy()
        plan.close()
    e = deltas["bf16"] - deltas["f32"]
    out["per_flip_change_1024x24"] = {
        "flips": n_flips, "median_abs_change_db": float(np.median(np.abs(deltas["f32"]))),
        "bf16_rms_error_db": float(np.sqrt(np.mean(e * e))), "bf16_max_error_db": float(np.max(np.abs(e))),
        "bf16_sign_errors": float(np.mean(np.sign(deltas["bf16"]) != np.sign(deltas["f32"])))}
    # configs[4]'s own wording: 1024 x 1024 under a 50 % on-pixel constraint (the EXTENSION of DESIGN
    # 4k; the reference has no such constraint), fp32 vs bf16 intermediates over one candidate prefix
    order24 = np.random.default_rng(3).permutation(24 * 1024 * 1024)[:n_constrained]
    cons = {}
    for name, prec in (("f32", PRECISION_F32), ("bf16", PRECISION_BF16_STORE)):
        plan = Plan(cfg, max_jobs=256, precision=prec)
        m = mask1024.clone()
        t0 = time.perf_counter()
        res = dbs.greedy(plan, m, target1024, order24, mode="fft", fill_ratio=0.5, fill_tol=4)
        torch.cuda.synchronize()
        cons[name] = (res, time.perf_counter() - t0)
        plan.close()
    (c32, ct32), (cbf, ctbf) = cons["f32"], cons["bf16"]
    b32 = np.zeros(len(order24), bool)
    bbf = np.zeros(len(order24), bool)
    b32[c32.accepted_positions] = True
    bbf[cbf.accepted_positions] = True
    dd = np.nonzero(b32 != bbf)[0]
    out["constrained_1024x24"] = {
        "workload": f"1024x1024x24 FFT-mode greedy DBS over the first {len(order24)} candidates of rng(3), "
                    "on-pixel ratio 0.5 +- 4 pixels per colour group (extension, DESIGN 4k)",
        "f32": {"accepts": len(c32.accepted_positions), "psnr_gain_db": c32.final_psnr - c32.initial_psnr,
                "final_fill_counts": c32.fill_counts, "seconds": round(ct32, 3)},
        "bf16_intermediates": {"accepts": len(cbf.accepted_positions),
                               "psnr_gain_db": cbf.final_psnr - cbf.initial_psnr,
                               "final_fill_counts": cbf.fill_counts, "seconds": round(ctbf, 3)},
        "final_psnr_deviation_db": abs(cbf.final_psnr - c32.final_psnr),
        "first_accept_sequence_difference": int(dd[0]) if len(dd) else None}
    out["note"] = ("bf16 rounding of the stored intermediates (numerics only; layout and traffic stay f32). "
                   "The f32 path equals the float64 oracle's accept sequence on this run "
                   "(tests/test_gpu_dbs_headline.py::test_dbs_ratio05_256_literal_run)")
    return out


def probe_sweep(cfg, mask, target, reps: int = 5):
    """SURVEY 8(a) a12 / range.py:294-335: PSNR change of every single-pixel flip
    of one 1024x1024x24 state against that fixed state (25.2 M trials), by
    correlation (hbx_flip_map)."""
    import torch
    from hbx.plan import Plan
    plan = Plan(cfg, max_jobs=cfg.groups)
    dmap, _ = plan.flip_map(mask, target)          # warm-up: h-side spectra, workspace
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        plan.flip_map(mask, target, out=dmap)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    n = cfg.channels * cfg.height * cfg.width
    improved = int((dmap > 0).sum().item())
    plan.close()
    return {"flips": n, "ms": round(dt * 1e3, 3), "flips_per_s": round(n / dt, 1), "improving": improved,
            "note": "every flip's exact PSNR change against the fixed state from 2-D FFT correlations "
                    "with the single-pixel field (no per-flip propagation); matches the f64 oracle to "
                    "<1e-8 dB (tests/test_gpu_parity.py::test_flip_map_*)"}


def cpu_baseline(n_steps: int, N: int):
    """numpy float64 oracle env-step (one 8-plane group propagate + PSNR + reward), 1 core."""
    import numpy as np
    from oracle import hbx_oracle as O
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    cfg = O.rgb_config(N)
    pre, tgt = O.synthetic_inputs(cfg, 0)
    env = O.OracleEnv(cfg)
    env.reset(pre, tgt)
    acts = np.random.default_rng(2).integers(0, cfg.channels * N * N, n_steps + 2)
    env.step(int(acts[0]))      # warm-up (2 steps: SURVEY 8d)
    env.step(int(acts[1]))
    t0 = time.perf_counter()
    for a in acts[2:]:
        env.step(int(a))
    dt = time.perf_counter() - t0
    return {"value": n_steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus_visible": host_cpus(), "steps": n_steps, "warmup": 2,
            "sample": f"{n_steps} env-steps after 2 warm-ups of the {N}x{N}x24 RGB env (one 8-plane group propagate each), "
                      f"numpy.fft complex128 oracle (oracle/hbx_oracle.py), 1 thread, {dt:.1f} s"}


def cpu_baseline_mono(n_steps: int, N: int = 256):
    """configs[0] / the PPO shard: env.py's 256x256x8 mono env-step on the float64 numpy
    oracle (one 8-plane group propagate + PSNR + reward), 1 core."""
    import numpy as np
    from oracle import hbx_oracle as O
    cfg = O.mono_config(N)
    pre, tgt = O.synthetic_inputs(cfg, 0)
    env = O.OracleEnv(cfg)
    env.reset(pre, tgt)
    acts = np.random.default_rng(2).integers(0, cfg.channels * N * N, n_steps + 2)
    env.step(int(acts[0]))
    env.step(int(acts[1]))
    t0 = time.perf_counter()
    for a in acts[2:]:
        env.step(int(a))
    dt = time.perf_counter() - t0
    return {"value": n_steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus_visible": host_cpus(), "steps": n_steps, "warmup": 2,
            "sample": f"{n_steps} env-steps after 2 warm-ups of the {N}x{N}x8 mono env (env.py), numpy.fft complex128 oracle "
                      f"(oracle/hbx_oracle.py), 1 thread, {dt:.1f} s"}


def vecenv_step_obs(mcfg, B, steps, warmup, tsrc, psrc, bare_ms, seed, graph=False, reps=3, obs_format="torch"):
    """The step an SB3 learner calls (train-PPO.py:296-322): HologramVecEnv.step with all
    five observation keys (env.py:176-181) as device tensors, rewards / dones to the host,
    every step.  The observations are views of buffers the step kernels keep current
    (ABI v8), so the difference to the bare device step is the recon write, the per-step host
    round trip and the Python VecEnv bookkeeping.  `reps` timed runs of `steps` steps each,
    alternating with the same number of bare device steps (step_device of an env without
    observations, no pass timing, no metric gather) on a twin env; medians of both."""
    import statistics
    import torch
    from hbx.env import OBS_KEYS, HologramVecEnv
    vec = HologramVecEnv(mcfg, B, tsrc, pre_model_source=psrc, obs_keys=OBS_KEYS, obs_format=obs_format,
                         auto_reset=True, max_steps=10 ** 9, T_PSNR=1e9, T_PSNR_DIFF=1e9, refresh_every=0,
                         graph=graph)
    pure = HologramVecEnv(mcfg, B, tsrc, pre_model_source=psrc, obs_keys=(), auto_reset=False,
                          max_steps=10 ** 9, T_PSNR=1e9, T_PSNR_DIFF=1e9, refresh_every=0)
    vec.reset()
    pure.reset()
    gen = torch.Generator(device="cuda").manual_seed(seed)
    n_pix = mcfg.channels * mcfg.height * mcfg.width
    actions = torch.randint(0, n_pix, (warmup + steps, B), generator=gen, device="cuda", dtype=torch.int64)
    # the VecEnv gets numpy actions, as SB3's rollout hands them over (on_policy_algorithm.py:
    # actions.cpu().numpy() -> env.step); they go into the host-mapped action row
    actions_h = actions.cpu().numpy()
    for k in range(warmup):
        vec.step(actions_h[k])
        pure.step_device(actions[k])
    torch.cuda.synchronize()
    t_obs, t_pure = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        for k in range(warmup, warmup + steps):
            obs, rew, dones, infos = vec.step(actions_h[k])
        torch.cuda.synchronize()
        t_obs.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        for k in range(warmup, warmup + steps):
            pure.step_device(actions[k])
        torch.cuda.synchronize()
        t_pure.append(time.perf_counter() - t0)
    dt = statistics.median(t_obs)
    pure_ms = statistics.median(t_pure) / steps * 1e3
    pure.close()
    shapes = {k: list(v.shape) for k, v in obs.items()} if obs_format == "torch" else \
        {k: list(obs.device(k).shape) for k in obs.keys()}
    views = obs_format == "torch" and all(v.data_ptr() == getattr(vec.state, a).data_ptr() for k, v, a in
                                          ((k, obs[k], {"state_record": "record", "state": "state_bytes",
                                                        "pre_model": "pre_model", "recon_image": "recon",
                                                        "target_image": "target"}[k]) for k in obs))
    vec.close()
    ms = dt / steps * 1e3
    return {"value": round(B * steps / dt, 2), "unit": "env-steps/s", "envs": B, "steps": steps, "reps": reps,
            "graph": graph, "ms_per_step": round(ms, 4), "bare_step_ms": round(bare_ms, 4),
            "obs_overhead_frac": round(ms / bare_ms - 1.0, 4),
            "pure_device_step_ms": round(pure_ms, 4), "overhead_vs_pure_device_step": round(ms / pure_ms - 1.0, 4),
            "obs_format": obs_format, "obs_keys": list(obs.keys()), "obs_shapes": shapes, "obs_are_views": views,
            "actions": "numpy int64 [B] per step (SB3's form), written into the host-mapped action row",
            "note": "HologramVecEnv.step (SB3 VecEnv surface, obs_format='torch', auto_reset on): all five "
                    "observation keys returned as views of device buffers the step kernels keep current "
                    "(state as int8, stepped pre-rollback recon_image), rewards / dones / error word written "
                    "by the step kernels into host-mapped memory; median of `reps` runs.  bare_step_ms is the "
                    "ppo_mono_256 line's device step (same measurement as the headline: sampled pass timing "
                    "and the per-8-step metric gather included); pure_device_step_ms is step_device of a twin "
                    "env without observations, timing or gather, alternated with the VecEnv runs"}


def vecenv_step_obs_numpy(mcfg, B, steps, warmup, tsrc, psrc, seed, reps=2):
    """The SB3-ingestible step: HologramVecEnv(obs_format="numpy") -- host
    mirrors of state / state_record / pre_model / target_image updated by env.py:164-181's rules,
    recon_image the one device -> host copy per step -- against r05's numpy path (every key
    copied device -> host each step, emulated here as the torch-format step + .cpu().numpy() of
    all five keys).  Each is timed bare and with every key read as SB3's DictRolloutBuffer.add
    does (`observations[key][pos] = np.array(obs[key])`, buffers/rollout: one host copy per key
    into a 2-row ring here); medians of `reps`."""
    import statistics
    import numpy as np
    import torch
    from hbx.env import OBS_KEYS, HologramVecEnv
    kw = dict(pre_model_source=psrc, obs_keys=OBS_KEYS, auto_reset=True, max_steps=10 ** 9, T_PSNR=1e9,
              T_PSNR_DIFF=1e9)
    new = HologramVecEnv(mcfg, B, tsrc, obs_format="numpy", **kw)
    old = HologramVecEnv(mcfg, B, tsrc, obs_format="torch", **kw)
    o_new, o_old = new.reset(), old.reset()
    gen = torch.Generator(device="cuda").manual_seed(seed)
    n_pix = mcfg.channels * mcfg.height * mcfg.width
    acts = torch.randint(0, n_pix, (warmup + steps, B), generator=gen, device="cuda").cpu().numpy()
    ring = {k: np.empty((2,) + tuple(v.shape), v.dtype) for k, v in o_new.items()}

    def run(env, to_np, add):
        t0 = time.perf_counter()
        for j, k in enumerate(range(warmup, warmup + steps)):
            obs, _, _, _ = env.step(acts[k])
            if to_np:
                obs = {kk: v.cpu().numpy() for kk, v in obs.items()}
            if add:
                for kk in OBS_KEYS:
                    ring[kk][j % 2] = np.array(obs[kk])
        return (time.perf_counter() - t0) / steps * 1e3

    for k in range(warmup):
        new.step(acts[k])
        old.step(acts[k])
    res = {"mirror": [], "mirror_add": [], "r05_numpy": [], "r05_numpy_add": []}
    for _ in range(reps):
        res["mirror"].append(run(new, False, False))
        res["r05_numpy"].append(run(old, True, False))
        res["mirror_add"].append(run(new, False, True))
        res["r05_numpy_add"].append(run(old, True, True))
    d2h = new._mirror.d2h_bytes
    new.close()
    old.close()
    med = {k: round(statistics.median(v), 4) for k, v in res.items()}
    return {"value": round(B / med["mirror"] * 1e3, 2), "unit": "env-steps/s", "envs": B, "steps": steps,
            "reps": reps, "ms_per_step": med["mirror"], "ms_per_step_with_rollout_add": med["mirror_add"],
            "r05_numpy_ms_per_step": med["r05_numpy"], "r05_numpy_ms_per_step_with_rollout_add": med["r05_numpy_add"],
            "d2h_bytes_per_step": d2h,
            "r05_d2h_bytes_per_step": int(sum(np.prod(v.shape) * v.itemsize for v in o_new.values())),
            "note": "obs_format='numpy': only recon_image goes device -> host per step (d2h_bytes_per_step); "
                    "r05_* is the torch-format step with every key copied device -> host, as r05's numpy "
                    "format did; *_with_rollout_add also copies every key as SB3's DictRolloutBuffer.add"}


def dropin_env(N: int, G: int, steps: int, warmup: int):
    """configs[0] on the GPU: the drop-in single env hbx.env.BinaryHologramEnv (B = 1) -- the
    object train-PPO.py's DummyVecEnv(n_envs=1) steps (train-PPO.py:40,275-313) -- with the
    reference's numpy observation dict every step (env.py:154-259).  Synthetic seeded image
    (SURVEY 8d seeds 0 / 1 / 2); thresholds out of reach so no episode ends in the timed loop."""
    import numpy as np
    import torch
    from hbx.env import BinaryHologramEnv
    from hbx.plan import mono_config, rgb_config
    cfg = mono_config(N) if G == 1 else rgb_config(N)
    CH = cfg.channels
    pre = np.random.default_rng(0).random((CH, N, N), np.float32)
    tgt = np.random.default_rng(1).random((G, N, N), np.float32)
    loader = [(torch.from_numpy(tgt[None]), ["synthetic.png"])]
    env = BinaryHologramEnv(lambda t: torch.from_numpy(pre[None]).to(t.device), loader, max_steps=10 ** 9,
                            T_PSNR=1e9, T_PSNR_DIFF=1e9, config=cfg, verbose=False)
    env.reset()
    acts = np.random.default_rng(2).integers(0, CH * N * N, warmup + steps).tolist()
    for a in acts[:warmup]:
        env.step(a)
    s0 = env.host_syncs
    t0 = time.perf_counter()
    for a in acts[warmup:]:
        obs, reward, term, trunc, info = env.step(a)
    dt = time.perf_counter() - t0
    syncs = (env.host_syncs - s0) / steps
    mode = env._vec.mode
    env.close()
    return {"value": round(steps / dt, 2), "unit": "env-steps/s", "envs": 1, "steps": steps, "mode": mode,
            "ms_per_step": round(dt / steps * 1e3, 4), "host_syncs_per_step": syncs,
            "obs": {k: [list(v.shape), str(v.dtype)] for k, v in obs.items()},
            "note": "hbx.env.BinaryHologramEnv.step (gymnasium contract, numpy obs dict): action into "
                    "host-mapped memory, the device step, the recon D2H behind it, one wait; "
                    "state / state_record / pre_model / target are host mirrors (env.py:176-181)"}


def torch_reference_step(N: int, steps: int, warmup: int):
    """What the reference's env.step costs on THIS GPU with PyTorch-ROCm doing its physics:
    env.py:164-188 restated with torch ops (full int8 -> f32 mask H2D per step, torch.fft
    fft2 / x H / ifft2 of the 8 planes, |.|^2, plane mean, least-squares relative PSNR, the
    .item() sync of the comparison).  Not our path: a baseline for the drop-in env at B = 1
    (torchOptics itself is absent; this assumes it is torch.fft-based)."""
    import numpy as np
    import torch
    from hbx.plan import mono_config
    cfg = mono_config(N)
    P = cfg.planes
    fx = np.fft.fftfreq(N, cfg.dx)
    fy = np.fft.fftfreq(N, cfg.dy)
    arg = 1.0 / cfg.wavelengths[0] ** 2 - fx[None, :] ** 2 - fy[:, None] ** 2
    H = torch.from_numpy(np.exp(2j * np.pi * cfg.z * np.sqrt(np.maximum(arg, 0))).astype(np.complex64)).cuda()
    state = (np.random.default_rng(0).random((1, P, N, N), np.float32) >= 0.5).astype(np.int8)
    target = torch.from_numpy(np.random.default_rng(1).random((1, 1, N, N), np.float32)).cuda()
    acts = np.random.default_rng(2).integers(0, P * N * N, warmup + steps)

    def psnr_of(st):
        u = torch.tensor(st, dtype=torch.float32).cuda()
        f = torch.fft.ifft2(torch.fft.fft2(u) * H)
        res = torch.mean(f.abs() ** 2, dim=1, keepdim=True)
        x, y = res.double(), target.double()
        s = torch.sum(x * y) / torch.sum(x * x)
        mse = torch.mean((s * x - y) ** 2)
        return float((10 * torch.log10(1.0 / mse)).item())

    prev = psnr_of(state)

    def step(a):
        nonlocal prev
        c, k = divmod(int(a), N * N)
        r, col = divmod(k, N)
        state[0, c, r, col] ^= 1
        p = psnr_of(state)
        if p - prev < 0:
            state[0, c, r, col] ^= 1
        else:
            prev = p

    for a in acts[:warmup]:
        step(a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in acts[warmup:]:
        step(a)
    dt = time.perf_counter() - t0
    return {"value": round(steps / dt, 2), "unit": "env-steps/s", "steps": steps,
            "ms_per_step": round(dt / steps * 1e3, 4),
            "note": "env.py:164-196's step with torch.fft (hipFFT) on this GPU, B = 1: the reference's "
                    "algorithm as PyTorch would run it, for scale -- not the product path"}


def shim_dbs_loop(N: int, flips: int, warmup: int):
    """An unchanged DBS.py-style caller (DBS.py:247-294) driving the torchOptics shim: per flip,
    the numpy state flipped, torch.tensor(state).cuda(), tt.Tensor(meta), tt.simulate(., z).abs()**2,
    the plane mean, tt.relativeLoss(., target, tm.get_PSNR), strict accept or undo.  Builder-written
    against the contract, timed on env.py's 256x256x8 mono."""
    import numpy as np
    import torch
    import torchOptics.metrics as tm
    import torchOptics.optics as tt
    from hbx.plan import PIXEL_PITCH
    P = 8
    state = (np.random.default_rng(0).random((1, P, N, N), np.float32) >= 0.5).astype(np.int8)
    target = torch.from_numpy(np.random.default_rng(1).random((1, 1, N, N), np.float32)).cuda()
    order = np.random.default_rng(3).permutation(P * N * N)[:warmup + flips]
    meta = {"dx": (PIXEL_PITCH, PIXEL_PITCH), "wl": 515e-9}

    def psnr_of():
        x = tt.Tensor(torch.tensor(state, dtype=torch.float32).cuda(), meta=meta)
        res = torch.mean(tt.simulate(x, 2e-3).abs() ** 2, dim=1, keepdim=True)
        return tt.relativeLoss(res, target, tm.get_PSNR)

    prev = psnr_of()
    acc = 0

    def flip(a):
        nonlocal prev, acc
        c, k = divmod(int(a), N * N)
        r, col = divmod(k, N)
        state[0, c, r, col] = 1 - state[0, c, r, col]
        p = psnr_of()
        if p > prev:
            prev, acc = p, acc + 1
        else:
            state[0, c, r, col] = 1 - state[0, c, r, col]

    for a in order[:warmup]:
        flip(a)
    torch.cuda.synchronize()
    a0 = acc
    t0 = time.perf_counter()
    for a in order[warmup:]:
        flip(a)
    dt = time.perf_counter() - t0
    return {"value": round(flips / dt, 2), "unit": "candidates/s", "flips": flips, "accepted": acc - a0,
            "ms_per_flip": round(dt / flips * 1e3, 4),
            "note": "DBS.py:247-294's per-flip loop shape through torchOptics.optics.simulate / relativeLoss "
                    "(hbx_simulate underneath): full mask H2D, 8-plane propagation returning complex fields, "
                    "a host PSNR per flip -- the unchanged-caller path, not the device walk (dbs_greedy)"}


def reset_cost(cfg, n_env: int = 8, reps: int = 5):
    """Per-env HologramVecEnv.reset_envs time (env.py:90-152: threshold -> full propagation ->
    initial PSNR) with the pre-model / target already on the device, for the mask packing as
    shipped (hbx_pack_mask, one HIP launch, ABI v14) and as it was through r05 (torch ops:
    `(pre >= 0.5)` -> int64 -> shift -> sum, several kernels materialising 8 B per pixel) --
    the same reset otherwise, alternated, median of `reps`."""
    import statistics
    import torch
    import hbx.env as E
    from hbx.env import HologramVecEnv
    c = cfg
    gen = torch.Generator(device="cuda").manual_seed(77)
    pres = [torch.rand((c.channels, c.height, c.width), generator=gen, device="cuda") for _ in range(n_env)]
    tgts = [torch.rand((c.groups, c.height, c.width), generator=gen, device="cuda") for _ in range(n_env)]
    vec = HologramVecEnv(c, n_env, lambda i: tgts[i], pre_model_source=lambda i: pres[i], obs_keys=(),
                         auto_reset=False)
    shipped = E.pack_mask

    def legacy(pre, threshold, out):
        m = (pre >= threshold).to(torch.int64).reshape(*pre.shape[:-1], pre.shape[-1] // 64, 64)
        shifts = torch.arange(64, device=pre.device, dtype=torch.int64)
        out.copy_((m << shifts).sum(dim=-1, dtype=torch.int64))

    def timed(fn):
        E.pack_mask = fn
        try:
            vec.reset_envs(range(n_env))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            vec.reset_envs(range(n_env))
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / n_env * 1e3
        finally:
            E.pack_mask = shipped

    timed(shipped)
    new, old = [], []
    mask_new = None
    for _ in range(reps):
        new.append(timed(shipped))
        mask_new = vec.state.mask.clone()
        old.append(timed(legacy))
    same = bool(torch.equal(mask_new, vec.state.mask))
    vec.close()
    return {"ms_per_env": round(statistics.median(new), 4), "torch_pack_ms_per_env": round(statistics.median(old), 4),
            "envs": n_env, "reps": reps, "masks_equal": same, "size": c.height, "planes": c.channels,
            "note": "HologramVecEnv.reset_envs per env (pre-model and target resident on the GPU: threshold, full "
                    "propagation of every group, initial PSNR); ms_per_env packs the mask with hbx_pack_mask (one "
                    "HIP launch), torch_pack_ms_per_env with r05's torch ops -- alternated on the same env"}


def check_devices(rows, world: int, rehearse: bool, dev) -> int:
    """The number of distinct GPUs the ranks ran on (rank 0's view of hbx.dist.describe_devices
    rows, agreed by every rank).  Outside a rehearsal a line whose ranks did not run on `world`
    distinct GPUs is refused: every rank exits non-zero (SystemExit), so no number is printed
    for a world that time-shared devices."""
    from hbx import dist as hd
    n = hd.distinct_devices(rows) if rows else 0
    bad = 0.0 if (rehearse or n == world) else 1.0
    if hd.max_over_ranks(bad if rows else 0.0, dev) > 0:
        raise SystemExit(f"bench.py: {world} ranks ran on {n} distinct GPU(s) ({rows}); "
                         "a multi-GPU line needs one GPU per rank (HBX_BENCH_REHEARSE_ONE_GPU=1 rehearses)")
    return n


def vecenv_step_sharded(mcfg, B, steps, warmup, tsrc, psrc, every, dev, world):
    """world > 1 (BASELINE configs[3], train-PPO.py:275-322 at 128 envs per GPU): every rank's
    SB3-facing step (HologramVecEnv.step, all five observations, numpy rewards / dones on the
    host) with the rewards and done flags gathered to rank 0 every `every` steps over the
    group's backend; barrier-bracketed, max-over-ranks time.  Collective: every rank calls it."""
    import numpy as np
    import torch
    from hbx import dist as hd
    from hbx.env import OBS_KEYS, HologramVecEnv
    vec = HologramVecEnv(mcfg, B, tsrc, pre_model_source=psrc, obs_keys=OBS_KEYS, obs_format="torch",
                         auto_reset=True, max_steps=10 ** 9, T_PSNR=1e9, T_PSNR_DIFF=1e9)
    vec.reset()
    gen = torch.Generator(device="cuda").manual_seed(13 + 7919 * hd.env_rank_world()[0])
    n_pix = mcfg.channels * mcfg.height * mcfg.width
    actions = torch.randint(0, n_pix, (warmup + steps, B), generator=gen, device="cuda", dtype=torch.int64)
    actions_h = actions.cpu().numpy()          # SB3's numpy actions (host-mapped action row)
    buf = torch.zeros((every, 2, B), dtype=torch.float64, pin_memory=True)
    hb = buf.numpy()
    got = [0]

    def run(k0, k1):
        j = 0
        for k in range(k0, k1):
            obs, rew, dones, infos = vec.step(actions_h[k])
            hb[j, 0] = rew
            hb[j, 1] = dones
            j += 1
            if j == every:
                g = hd.gather_to_rank0(buf.to(dev, non_blocking=True))
                got[0] += 0 if g is None else g.shape[0]
                j = 0
        if j:
            g = hd.gather_to_rank0(buf[:j].to(dev))
            got[0] += 0 if g is None else g.shape[0]

    run(0, warmup)
    torch.cuda.synchronize()
    hd.barrier()
    got[0] = 0
    t0 = time.perf_counter()
    run(warmup, warmup + steps)
    torch.cuda.synchronize()
    hd.barrier()
    dt = hd.max_over_ranks(time.perf_counter() - t0, dev)
    vec.close()
    return {"value": round(B * world * steps / dt, 2), "unit": "env-steps/s", "envs_per_rank": B, "ranks": world,
            "steps": steps, "ms_per_step": round(dt / steps * 1e3, 4), "gather_every": every,
            "gathered_rows_rank0": got[0],
            "note": "HologramVecEnv.step on every rank (all five observations, numpy rewards / dones), the "
                    "per-step rewards and done flags gathered to rank 0 every `gather_every` steps; "
                    "barrier-bracketed, max over ranks"}


def psnr_check(vec, N):
    """PSNR delta vs the numpy oracle for env 0's initial state (full 24-plane propagate)."""
    import numpy as np
    from oracle import hbx_oracle as O
    cfg = O.rgb_config(N)
    mask = vec.state.mask[0].cpu().numpy().view("<u8")
    m = O.unpack_mask(mask, N)
    tgt = vec.state.target[0].cpu().numpy()
    prop = O.Propagator(cfg)
    inten = prop.all_intensity(m)
    st = np.stack([O.chan_stats(inten[g], tgt[g]) for g in range(3)])
    return abs(prop.psnr(st) - float(vec.state.init_psnr[0].item()))


def load_pmc_traffic(N: int = 1024):
    """Per-launch HBM bytes of the dominant kernels from the committed rocprofv3
    PMC summary (profiles/pmc_latest.json, written by tools/pmc_summary.py from
    separate FETCH_SIZE / WRITE_SIZE passes with the gfx950 x2 read correction)."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json" if N == 1024 else f"pmc_latest_{N}.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p))
    except Exception:
        return None


def pass_table(timing, abytes, jobs_override=None):
    """Per-pass average launch time and algorithmic GB/s.  jobs_override[name] replaces
    the jobs a pass is charged for (k_psf_commit only rewrites the ACCEPTED envs' planes)."""
    passes = {}
    for name, (ms, launches, jobs) in timing.items():
        if launches:
            avg = ms / launches
            if jobs_override and name in jobs_override:
                jobs = jobs_override[name]
            per_launch = abytes[name] * (jobs / launches)
            passes[name] = {"avg_ms": avg, "launches": launches, "jobs_per_launch": jobs / launches,
                            "alg_bytes_per_launch": per_launch,
                            "achieved_GBs": per_launch / (avg * 1e-3) / 1e9}
    return passes


def rounded(passes):
    return {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
            for k, v in passes.items()}


def main():
    args = parse()
    rc = launch_ranks(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    # the driver reads ONE JSON line from stdout: keep a handle on the real stdout and point
    # fd 1 at stderr, so library banners (RCCL prints its version block on stdout when the
    # communicator is created) cannot land on it
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    import torch
    from hbx import dist as hd
    from hbx.env import HologramVecEnv
    from hbx.plan import crop_config, mono_config, rgb_config

    # HBX_BENCH_REHEARSE_ONE_GPU=1: every rank on cuda:0 over gloo -- rehearses the world > 1
    # code path on a one-GPU box (RCCL refuses two ranks on one device); never a measurement
    rehearse = os.environ.get("HBX_BENCH_REHEARSE_ONE_GPU") == "1"
    # a process group at every world size (RCCL at N = 1 too): the N = 1 line runs the same
    # per-step metric gather, barrier and max-over-ranks collectives as the 8-GPU one
    rank, world, local = hd.init(backend="gloo" if rehearse else None, force=not args.no_pg)
    if rehearse:
        local = 0
    if world != args.gpus:
        # never measure a different number of ranks than asked for (a --gpus 8 line from one rank)
        raise SystemExit(f"bench.py: --gpus {args.gpus} but this run has WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    N, B = args.size, args.envs
    cfg = rgb_config(N)
    CH, G, P = cfg.channels, cfg.groups, cfg.planes
    gather = hd.active() and not args.no_gather

    # synthetic, seeded per global env index
    def target_source(i):
        g = torch.Generator(device="cuda").manual_seed(1_000_003 * (rank * B + i) + 1)
        return torch.rand((G, N, N), generator=g, device="cuda")

    def pre_model_source(i):
        g = torch.Generator(device="cuda").manual_seed(1_000_003 * (rank * B + i))
        return torch.rand((CH, N, N), generator=g, device="cuda")

    def measure(mode: str, steps: int, warmup: int, mcfg=None, timing_every=None, margin=0):
        mcfg = mcfg or cfg
        mG, mCH, mN = mcfg.groups, mcfg.channels, mcfg.height
        m0 = margin       # centre crop (env_1024_24_128.py:144-149) or the top-left corner

        def tsrc(i):
            return target_source(i)[:mG, m0:m0 + mN, m0:m0 + mN].contiguous()

        def psrc(i):
            return pre_model_source(i)[:mCH, m0:m0 + mN, m0:m0 + mN].contiguous()

        vec = HologramVecEnv(mcfg, B, tsrc, pre_model_source=psrc, obs_keys=(),
                             auto_reset=False, max_steps=10 ** 9, max_jobs=args.chunk or None, mode=mode,
                             refresh_every=0)
        vec.reset()
        gen = torch.Generator(device="cuda").manual_seed(2 + 7919 * rank)
        total = warmup + steps
        actions = torch.randint(0, mCH * mN * mN, (total, B), generator=gen, device="cuda", dtype=torch.int64)
        mg = hd.StepMetricGather(B, args.gather_every, dev) if gather else None

        def one_step(k):
            if mg is not None:
                mg.add(*vec.step_device(actions[k], out=mg.slot()))
            else:
                vec.step_device(actions[k])

        for k in range(warmup):
            one_step(k)
        if mg is not None:
            mg.flush()
        torch.cuda.synchronize()
        vec.plan.set_timing(steps * -(-B // (args.chunk or B)) + 1,
                            timing_every or args.timing_every)
        hd.barrier()
        torch.cuda.synchronize()
        acc0 = int(vec.state.flip_count.sum().item())
        t0 = time.perf_counter()
        for k in range(warmup, total):
            one_step(k)
        if mg is not None:
            mg.flush()
        torch.cuda.synchronize()
        hd.barrier()
        dt = hd.max_over_ranks(time.perf_counter() - t0, dev)
        timing = vec.plan.read_timing()
        vec.state.check_error()
        # accepted steps in the timed region (flip_count counts accepted flips, no resets here)
        vec.timed_accepts = int(vec.state.flip_count.sum().item()) - acc0
        acc_rate = float(vec.state.flip_count.sum().item()) / float(vec.state.steps.sum().item())
        return vec, dt, timing, acc_rate

    ranks_seen = hd.describe_devices(dev)
    n_devices = check_devices(ranks_seen, world, rehearse, dev)
    vec, dt, timing, acc_rate = measure("fft", args.steps, args.warmup)
    value = B * world * args.steps / dt
    ms_per_step = dt / args.steps * 1e3
    abytes = algorithmic_bytes(N, P)
    passes = pass_table(timing, abytes)
    out = None
    if rank == 0:
        dom = max(passes, key=lambda n: passes[n]["avg_ms"])
        d = passes[dom]
        pmc = load_pmc_traffic(N)
        traffic, traffic_src = None, None
        if pmc and dom in pmc.get("kernels", {}):
            kinfo = pmc["kernels"][dom]
            if kinfo.get("jobs_per_launch") == d["jobs_per_launch"] and kinfo.get("N") == N:
                traffic = kinfo.get("hbm_bytes_per_launch")
                traffic_src = (f"committed rocprofv3 PMC passes (profiles/pmc_latest{'' if N == 1024 else '_' + str(N)}"
                               f".json, source {pmc.get('source')}), a 1-GPU run of the same kernel and "
                               f"launch shape -- not measured in this run")
        roofline = {"bound": "hbm", "achieved": round(d["achieved_GBs"], 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(d["achieved_GBs"] / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "traffic_source": traffic_src,
                    "kernel": dom, "kernel_avg_ms": round(d["avg_ms"], 4),
                    "timing": f"hipEvent pairs on the launch stream around every {args.timing_every}-th launch "
                              f"of each pass inside the timed loop ({d['launches']} launches of {dom})"}
        step_bytes = sum(abytes[k] for k in timing if k in ("k_rowfwd", "k_col", "k_rowinv")) * B
        canon = canonical_step_bytes(N, P)
        out = {
            "metric": "env-steps/sec (1024x1024, 24-plane)" if N == 1024 else
                      f"env-steps/sec ({N}x{N} crop of 1024x1024, 24-plane)",
            "value": round(value, 2),
            "unit": "env-steps/s",
            "n_gpus": n_devices if rehearse else world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded U[0,1) pre-model/targets, uniform actions)",
            "config": {"workload": "configs[2]: batched VecEnv.step, 128 envs/GPU x 1024x1024x24-plane "
                                   "(3 colour groups x 8 planes), one action per env per step, FFT mode "
                                   "(whole touched group re-propagated)",
                       "envs_per_gpu": B, "global_envs": B * world, "size": N, "planes": CH,
                       "parallelism": f"env-sharded x{world}" + (
                           f" + metric gather to rank 0 every {args.gather_every} step(s)" if gather else ""),
                       "obs_keys": [],
                       "obs_note": "the headline times the device step (reward / psnr / accepted / terminated / "
                                   "truncated stay on the device, HologramVecEnv(obs_keys=())); the SB3-facing "
                                   "step with all five observations is `vecenv_step_obs`"},
            "ranks_seen": ranks_seen,
            "ranks_seen_note": "[rank, world, local_rank, backend, current device, PCI address, uuid] from "
                               "every rank (hbx.dist.describe_devices): the GPU each rank actually ran on",
            "roofline": roofline,
            "passes": rounded(passes),
            "step_alg_GBs": round(step_bytes / (ms_per_step * 1e-3) / 1e9, 1),
            "step_alg_frac": round(step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "step_canonical_equivalent": {
                "bytes_per_env_step": canon,
                "GBs_equivalent": round(canon * value / world / 1e9, 1),
                "note": "NOT bandwidth: SURVEY 8d's canonical bytes per env-step (two complex64 round trips "
                        "per plane + target + mask) x env-steps/s per GPU.  The kernels move fewer bytes "
                        "(half-spectrum intermediates): their achieved step bandwidth is step_alg_GBs / "
                        "step_alg_frac"},
            "accept_rate": round(acc_rate, 4),
        }
        if rehearse:
            out["rehearsal"] = True
            out["rehearsal_note"] = (f"HBX_BENCH_REHEARSE_ONE_GPU=1: {world} ranks time-sharing {n_devices} GPU(s) "
                                     "over gloo -- exercises the world > 1 code path, NOT a scaling measurement")
        if world == 1 and not args.no_psnr_check:
            out["psnr_delta_vs_numpy"] = psnr_check(vec, N)
    dbs_mask = vec.state.mask[0].clone()
    dbs_target = vec.state.target[0].clone()
    vec.close()
    del vec
    torch.cuda.empty_cache()

    if rank == 0 and world == 1 and not args.no_obs:
        out["vecenv_step_obs"] = vecenv_step_obs(
            cfg, B, args.steps, args.warmup, lambda i: target_source(i), lambda i: pre_model_source(i),
            ms_per_step, 11)
        out["vecenv_step_obs"]["graph_replay"] = {k: v for k, v in vecenv_step_obs(
            cfg, B, args.steps, args.warmup, lambda i: target_source(i), lambda i: pre_model_source(i),
            ms_per_step, 11, graph=True).items() if k in ("value", "ms_per_step", "obs_overhead_frac")}
        torch.cuda.empty_cache()

    if rank == 0 and world == 1 and args.dbs_flips > 0:
        out["dbs_greedy"] = dbs_prefix(cfg, dbs_mask, dbs_target, args.dbs_flips)
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_probe:
        out["probe_sweep"] = probe_sweep(cfg, dbs_mask, dbs_target)
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_precision and N == 1024:
        out["precision_sweep"] = precision_sweep(dbs_mask, dbs_target)
        torch.cuda.empty_cache()

    if not args.no_psf:
        vec, dt, timing, acc_rate = measure("psf", args.psf_steps, max(args.warmup, 5),
                                          timing_every=1)   # k_psf_commit is charged the timed accepts
        if rank == 0:
            ps = pass_table(timing, abytes, {"k_psf_commit": vec.timed_accepts})
            ev = ps.get("k_psf_eval")
            out["incremental_psf_mode"] = {
                "value": round(B * world * args.psf_steps / dt, 2), "unit": "env-steps/s",
                "steps": args.psf_steps, "ms_per_step": round(dt / args.psf_steps * 1e3, 4),
                "accept_rate": round(acc_rate, 4),
                "roofline": None if ev is None else {
                    "bound": "hbm", "kernel": "k_psf_eval", "achieved": round(ev["achieved_GBs"], 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ev["achieved_GBs"] / HBM_PEAK_GBS, 4),
                    "kernel_avg_ms": round(ev["avg_ms"], 4)},
                "passes": rounded(ps),
                "passes_note": "k_psf_commit is charged for the accepted envs only (24 N^2 B each); its "
                               "launch covers all envs but rejected ones return at once",
                "note": "same env semantics; a flip adds +-h_g(shifted) to the touched plane's cached field "
                        "(linearity of the propagation), no FFT per step; reported separately per SURVEY 8d"}
        vec.close()

    if not args.no_planes and N in (256, 1024):
        # plane-cached FFT mode: every result the FFT mode's bit for bit (tests/test_gpu_planes.py),
        # only the flipped plane's pair propagated per step
        psteps = 4 * args.steps
        vec, dt, timing, acc_rate = measure("planes", psteps, args.warmup)
        vec.close()
        if rank == 0:
            ps = pass_table(timing, plane_cached_bytes(N, P))
            step_b = sum(plane_cached_bytes(N, P).values()) * B
            pms = dt / psteps * 1e3
            out["plane_cached_mode"] = {
                "value": round(B * world * psteps / dt, 2), "unit": "env-steps/s", "steps": psteps,
                "ms_per_step": round(pms, 4), "accept_rate": round(acc_rate, 4),
                "vs_fft_mode": round((B * world * psteps / dt) / value, 3),
                "passes": rounded(ps),
                "step_alg_GBs": round(step_b / (pms * 1e-3) / 1e9, 1),
                "note": "same env semantics and the FFT mode's results bit for bit: a step propagates only "
                        "the flipped plane's pair and sums the other planes' cached |U|^2 in the FFT mode's "
                        "plane order (include/hbx.h ABI v9); reported separately, the headline stays the "
                        "literal re-propagation of the whole group"}
        torch.cuda.empty_cache()

    if not args.no_crop and N == 1024:
        # env_1024_24_128.py:144-149 (BASELINE configs[2]'s script): the centre 896 x 896 crop of
        # the 1024 masks, 24 planes, 128 envs per GPU, FFT mode -- the mixed-radix 28 x 32 passes
        ccfg = crop_config(cfg, 64)
        cN = ccfg.height
        vec, dt, timing, acc_rate = measure("fft", args.steps, args.warmup, mcfg=ccfg, margin=64)
        vec.close()
        if rank == 0:
            cb = algorithmic_bytes(cN, P)
            ps = pass_table(timing, cb)
            dom = max(ps, key=lambda n: ps[n]["avg_ms"])
            pmc = load_pmc_traffic(cN)
            ctraffic, csrc = None, None
            if pmc and dom in pmc.get("kernels", {}):
                kinfo = pmc["kernels"][dom]
                if kinfo.get("jobs_per_launch") == ps[dom]["jobs_per_launch"] and kinfo.get("N") == cN:
                    ctraffic = kinfo.get("hbm_bytes_per_launch")
                    csrc = (f"committed rocprofv3 PMC passes (profiles/pmc_latest_{cN}.json, source "
                            f"{pmc.get('source')}) -- not measured in this run")
            cms = dt / args.steps * 1e3
            cstep = sum(cb[k] for k in ("k_rowfwd", "k_col", "k_rowinv")) * B
            out["crop_896"] = {
                "value": round(B * world * args.steps / dt, 2), "unit": "env-steps/s", "envs_per_gpu": B,
                "steps": args.steps, "ms_per_step": round(cms, 4), "accept_rate": round(acc_rate, 4),
                "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ps[dom]["achieved_GBs"], 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(ps[dom]["achieved_GBs"] / HBM_PEAK_GBS, 4), "traffic": ctraffic,
                             "traffic_source": csrc, "kernel_avg_ms": round(ps[dom]["avg_ms"], 4)},
                "passes": rounded(ps),
                "step_alg_frac": round(cstep / (cms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "note": "env_1024_24_128.py:144-149: the centre 896 x 896 crop of 1024 x 1024 x 24 masks "
                        "(64 px per side), FFT mode, same env semantics; 896 = 28 x 32 mixed-radix passes "
                        "(csrc/hbx_passes896.hip)"}
        torch.cuda.empty_cache()
        if not args.no_planes:
            # (r06) the plane-cached FFT mode at 896: the FFT mode's bits (tests/test_gpu_planes.py)
            psteps = 4 * args.steps
            vec, dt, timing, acc_rate = measure("planes", psteps, args.warmup, mcfg=ccfg, margin=64)
            vec.close()
            if rank == 0:
                ps = pass_table(timing, plane_cached_bytes(cN, P))
                pms = dt / psteps * 1e3
                out["crop_896"]["plane_cached_mode"] = {
                    "value": round(B * world * psteps / dt, 2), "unit": "env-steps/s", "steps": psteps,
                    "ms_per_step": round(pms, 4), "accept_rate": round(acc_rate, 4),
                    "vs_fft_mode": round((B * world * psteps / dt) / out["crop_896"]["value"], 3),
                    "passes": rounded(ps),
                    "step_alg_GBs": round(sum(plane_cached_bytes(cN, P).values()) * B / (pms * 1e-3) / 1e9, 1)}
            torch.cuda.empty_cache()

    if not args.no_ppo:
        # SURVEY 3.2 / BASELINE configs[3]'s per-GPU shard: train-PPO.py's env (env.py, 256x256x8
        # mono), 128 envs per GPU, FFT mode -- a secondary line, not the headline metric; at world > 1
        # every rank steps its own 128 envs and the metrics are gathered to rank 0 (train-PPO.py:275-322)
        mono = mono_config(256)
        # a 0.35-ms step: 8x the headline's step count keeps the timed region ~0.1 s
        msteps = 8 * args.steps
        vec, dt, timing, acc_rate = measure("fft", msteps, args.warmup, mcfg=mono)
        ps = pass_table(timing, algorithmic_bytes(256, mono.planes))
        vec.close()
        mono_ms = dt / msteps * 1e3
        if rank == 0:
            dom = max(ps, key=lambda n: ps[n]["avg_ms"])
            pmc = load_pmc_traffic(256)
            mtraffic = None
            if pmc and dom in pmc.get("kernels", {}):
                kinfo = pmc["kernels"][dom]
                if kinfo.get("jobs_per_launch") == ps[dom]["jobs_per_launch"] and kinfo.get("N") == 256:
                    mtraffic = kinfo.get("hbm_bytes_per_launch")
            out["ppo_mono_256"] = {
                "value": round(B * world * msteps / dt, 2), "unit": "env-steps/s", "envs": B,
                "global_envs": B * world, "n_ranks": world, "steps": msteps,
                "ms_per_step": round(mono_ms, 4), "accept_rate": round(acc_rate, 4),
                "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ps[dom]["achieved_GBs"], 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(ps[dom]["achieved_GBs"] / HBM_PEAK_GBS, 4), "traffic": mtraffic,
                             "traffic_source": None if mtraffic is None else
                             f"committed rocprofv3 PMC passes (profiles/pmc_latest_256.json, source "
                             f"{pmc.get('source')}) -- not measured in this run",
                             "kernel_avg_ms": round(ps[dom]["avg_ms"], 4)},
                "passes": rounded(ps),
                "note": "configs[0] / train-PPO.py's env (env.py, 256x256, 1 colour group x 8 planes at 515 nm), "
                        "128 envs per GPU, FFT mode, same env semantics as the headline" +
                        (f"; {world} ranks, metric gather to rank 0 every {args.gather_every} steps" if world > 1 else "")}
        if not args.no_obs:
            mt = lambda i: target_source(i)[:1, :256, :256].contiguous()   # noqa: E731
            mp = lambda i: pre_model_source(i)[:8, :256, :256].contiguous()  # noqa: E731
            if world == 1:
                if rank == 0:
                    vo = vecenv_step_obs(mono, B, msteps, args.warmup, mt, mp, mono_ms, 12)
                    vo["graph_replay"] = {k: v for k, v in vecenv_step_obs(
                        mono, B, msteps, args.warmup, mt, mp, mono_ms, 12,
                        graph=True).items() if k in ("value", "ms_per_step", "obs_overhead_frac")}
                    vo["lazy_obs_unread"] = {k: v for k, v in vecenv_step_obs(
                        mono, B, msteps, args.warmup, mt, mp, mono_ms, 12,
                        obs_format="lazy").items() if k in ("value", "ms_per_step", "obs_overhead_frac",
                                                            "overhead_vs_pure_device_step")}
                    out["ppo_mono_256"]["vecenv_step_obs"] = vo
                    out["ppo_mono_256"]["vecenv_step_obs_numpy"] = vecenv_step_obs_numpy(
                        mono, B, 30, 5, mt, mp, 13)
            else:
                vo = vecenv_step_sharded(mono, B, msteps, args.warmup, mt, mp, args.gather_every, dev, world)
                if rank == 0:
                    out["ppo_mono_256"]["vecenv_step_obs"] = vo
        if rank == 0 and world == 1 and args.cpu_sample > 0:
            out["ppo_mono_256"]["cpu_baseline"] = cpu_baseline_mono(max(40, 25 * args.cpu_sample))
        if not args.no_planes:      # the same mono step in the plane-cached FFT mode (bit-exact)
            vec, dt, timing, _ = measure("planes", msteps, args.warmup, mcfg=mono)
            vec.close()
            if rank == 0:
                pps = pass_table(timing, plane_cached_bytes(256, mono.planes))
                out["ppo_mono_256"]["plane_cached_mode"] = {
                    "value": round(B * world * msteps / dt, 2), "unit": "env-steps/s",
                    "ms_per_step": round(dt / msteps * 1e3, 4),
                    "vs_fft_mode": round((B * world * msteps / dt) / out["ppo_mono_256"]["value"], 3),
                    "passes": rounded(pps)}

    if rank == 0 and world == 1 and not args.no_dropin:
        # configs[0] on the GPU: the drop-in single env an unchanged train-PPO.py binds, beside the
        # reference's algorithm on torch.fft and an unchanged DBS.py-style shim caller
        d = dropin_env(256, 1, max(1000, 20 * args.steps), 50)
        d["torch_reference_step"] = torch_reference_step(256, 300, 20)
        d["shim_dbs_loop"] = shim_dbs_loop(256, 300, 20)
        cb = out.get("ppo_mono_256", {}).get("cpu_baseline")
        if cb:
            d["cpu_baseline_mono"] = {"value": cb["value"], "unit": cb["unit"], "cores": cb["cores"],
                                      "vs_dropin": round(d["value"] / cb["value"], 1)}
        out["dropin_env_256"] = d
        out["dropin_env_1024x24"] = dropin_env(1024, 3, 60, 5)
        out["reset_1024x24"] = reset_cost(cfg)
        torch.cuda.empty_cache()

    if rank == 0:
        if world == 1 and args.cpu_sample > 0:
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample, N)
            if not args.no_scipy:
                try:
                    workers = min(16, host_cpus())
                    out["cpu_baseline_scipy"] = cpu_baseline_scipy(max(20, args.cpu_sample), N, workers)
                except Exception as e:  # scipy is optional on the box
                    out["cpu_baseline_scipy"] = {"error": str(e)}
        print(json.dumps(out), file=json_out, flush=True)
    hd.shutdown()


if __name__ == "__main__":
    main()
