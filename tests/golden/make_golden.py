"""Generate the committed golden fixtures from the oracle (oracle/hbx_oracle.py).

The reference cannot run here (torchOptics / gymnasium / SB3 / torchvision
absent), so these vectors are the oracle's own float64 outputs on
seeded inputs, plus the reference's stated known answers (env.py:228-229).
They pin (a) the oracle against silent drift and (b) the HIP path in the
-m gpu parity tests.  Run:  python tests/golden/make_golden.py
(the headline-size DBS fixtures: python tests/golden/make_golden.py --large)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import hbx_oracle as O  # noqa: E402

COMBOS = [(tf, fk, rs) for tf in (O.TF_ASM, O.TF_FRESNEL)
          for fk in (O.FIELD_AMPLITUDE, O.FIELD_PHASE) for rs in (O.REL_LSQ, O.REL_NONE)]


def small_rgb_cfg(**kw):
    # 64x64, 3 colour groups x 2 planes: the smallest shape exercising every
    # code path of the RGB env (group selection, cached other-group stats)
    return O.OpticsConfig(64, 64, 3, 2, O.WL_RGB, **kw)


def decode_table():
    rows = []
    rng = np.random.default_rng(7)
    for (n, ch) in ((256, 8), (1024, 24)):
        hw = n * n
        edges = [0, hw - 1, hw, ch * hw - 1, n - 1, n, 5 * hw + 3 * n + 7]
        rand = rng.integers(0, ch * hw, 25).tolist()
        for a in edges + rand:
            c, r, col = O.decode_action(a, n, n)
            rows.append((n, ch, a, int(c), int(r), int(col)))
    return np.array(rows, np.int64)


def reward_table():
    s = np.array([1.0, 0.5, 0.25, 0.125, 0.0, 0.3333333333333333])
    return s, np.array([O.success_cubic(v) for v in s]), np.array([O.max_steps_cubic(v) for v in s])


def prop_fixture(cfg_fn, seed):
    cfg = cfg_fn()
    pre, tgt = O.synthetic_inputs(cfg, seed)
    mask = (pre >= 0.5).astype(np.uint8)
    out = {"mask_bits": O.pack_mask(mask), "target": tgt, "seed": np.int64(seed),
           "combos": np.array(COMBOS, np.int64)}
    stats_all, psnr_all = [], []
    for (tf, fk, rs) in COMBOS:
        c = cfg_fn(tf_kind=tf, field_kind=fk, rel_scale=rs)
        prop = O.Propagator(c)
        inten = prop.all_intensity(mask)
        st = np.stack([O.chan_stats(inten[g], tgt[g]) for g in range(c.groups)])
        stats_all.append(st)
        psnr_all.append(prop.psnr(st))
        if (tf, fk, rs) == COMBOS[0]:
            out["intensity"] = inten.astype(np.float32)
            out["psnr_direct"] = np.float64(O.relative_psnr(inten, tgt, rs))
    out["stats"] = np.array(stats_all)
    out["psnr"] = np.array(psnr_all)
    return out


def env_trace(steps=200):
    cfg = small_rgb_cfg()
    pre, tgt = O.synthetic_inputs(cfg, 11)
    env = O.OracleEnv(cfg, max_steps=150, T_PSNR=30.0, T_steps=1, T_PSNR_DIFF=0.08)
    env.reset(pre, tgt)
    acts = np.random.default_rng(12).integers(0, cfg.channels * 64 * 64, steps)
    rec = [env.step(int(a)) for a in acts]
    return {"pre_model": pre, "target": tgt, "actions": acts.astype(np.int64),
            "initial_psnr": np.float64(env.initial_psnr),
            "psnr": np.array([r.psnr for r in rec]), "reward": np.array([r.reward for r in rec]),
            "accepted": np.array([r.accepted for r in rec]),
            "terminated": np.array([r.terminated for r in rec]),
            "truncated": np.array([r.truncated for r in rec]),
            "final_mask_bits": O.pack_mask(env.state.astype(np.uint8)),
            "final_record": env.state_record.copy(),
            "params": np.array([150, 30.0, 1, 0.08])}


def dbs_trace(n=4096):
    cfg = small_rgb_cfg()
    pre, tgt = O.synthetic_inputs(cfg, 21)
    env = O.OracleEnv(cfg, accept_rule=1)
    env.reset(pre, tgt)
    order = np.random.default_rng(3).permutation(cfg.channels * 64 * 64)[:n].astype(np.int64)
    acc, psnrs, final = O.dbs_greedy(env, order)
    return {"pre_model": pre, "target": tgt, "order": order, "accepted": acc, "psnr": psnrs,
            "initial_psnr": np.float64(env.initial_psnr), "final_psnr": np.float64(final),
            "final_mask_bits": O.pack_mask(env.state.astype(np.uint8))}


def probe_fixture(n=2048):
    cfg = small_rgb_cfg()
    pre, tgt = O.synthetic_inputs(cfg, 31)
    env = O.OracleEnv(cfg)
    base = env.reset(pre, tgt)
    flips = np.random.default_rng(32).integers(0, cfg.channels * 64 * 64, n).astype(np.int64)
    ps = O.probe_sweep(env, flips)
    improved = ps > base
    att, imp, dsum = O.premodel_histogram(pre, flips, improved, ps - base, 64, 64)
    return {"pre_model": pre, "target": tgt, "flips": flips, "psnr": ps, "base_psnr": np.float64(base),
            "attempted": att, "improved": imp, "delta_sum": dsum}


def env_group_trace(steps=260, k=512, seed=77):
    """env_group.py importance-reward episode: K sampled flips at reset,
    nearest-change rewards, dynamic T_PSNR_DIFF, linear bonuses."""
    cfg = small_rgb_cfg()
    pre, tgt = O.synthetic_inputs(cfg, 51)
    env = O.OracleEnvGroup(cfg, max_steps=250, T_PSNR=30.0, T_steps=1)
    n_pix = cfg.channels * 64 * 64
    sample = O.importance_sample(n_pix, k, seed)
    env.reset_group(pre, tgt, sample)
    acts = np.random.default_rng(52).integers(0, n_pix, steps)
    rec = [env.step(int(a)) for a in acts]
    return {"pre_model": pre, "target": tgt, "sample": sample.astype(np.int64),
            "changes": np.asarray(env.psnr_change_list, np.float64),
            "importance": np.asarray(env.importance_ranks, np.float64),
            "t_psnr_diff": np.float64(env.T_PSNR_DIFF), "seed": np.int64(seed),
            "initial_psnr": np.float64(env.initial_psnr), "actions": acts.astype(np.int64),
            "psnr": np.array([r.psnr for r in rec]), "reward": np.array([r.reward for r in rec]),
            "accepted": np.array([r.accepted for r in rec]),
            "terminated": np.array([r.terminated for r in rec]),
            "truncated": np.array([r.truncated for r in rec]),
            "params": np.array([250, 30.0, 1])}


def dbs_prefix_large(cfg, n, seed=0, order_seed=3, stop_diff=None, n_probe=0):
    """Greedy DBS at a full reference size by the float64 linear evaluator
    (O.LinearGreedy): the accept sequence, every candidate's PSNR and its
    PSNR change against the running base, over the first ``n`` candidates of
    rng(order_seed).permutation(CH*N^2) of the seeded synthetic
    image.  The inputs are regenerated from the seeds, so only the outputs
    are stored."""
    pre, tgt = O.synthetic_inputs(cfg, seed)
    order = np.random.default_rng(order_seed).permutation(cfg.channels * cfg.height * cfg.width)
    if n is not None:
        order = order[:n]
    lg = O.LinearGreedy(cfg, pre, tgt)
    # PSNR change of the first n_probe candidates against the INITIAL state (no commits):
    # pins each candidate's evaluation, accepted or not (probe sweep / eval_flips)
    probe = np.array([lg.evaluate(int(a))[0] - lg.initial_psnr for a in order[:n_probe]], np.float64)
    acc, ps, delta = lg.run(order, stop_diff=stop_diff)
    return {"seed": np.int64(seed), "order_seed": np.int64(order_seed),
            "size": np.int64(cfg.height), "groups": np.int64(cfg.groups), "planes": np.int64(cfg.planes),
            "field_kind": np.int64(cfg.field_kind), "n": np.int64(len(acc)),
            "stop_diff": np.float64(np.nan if stop_diff is None else stop_diff),
            "accepted": acc, "psnr": ps, "delta": delta,
            "initial_psnr": np.float64(lg.initial_psnr), "final_psnr": np.float64(lg.previous_psnr),
            "probe_delta": probe}


def env_trace_large(cfg, n_steps, seed=0, action_seed=2):
    """The env step (env.py:154-214) at a full reference size: n_steps seeded random
    actions (rng(2).integers) on the seeded synthetic image, accept iff the
    PSNR change is >= 0, by the float64 linear evaluator."""
    pre, tgt = O.synthetic_inputs(cfg, seed)
    actions = np.random.default_rng(action_seed).integers(0, cfg.channels * cfg.height * cfg.width, n_steps)
    lg = O.LinearGreedy(cfg, pre, tgt)
    acc, ps, delta = lg.run_env(actions)
    return {"seed": np.int64(seed), "action_seed": np.int64(action_seed), "size": np.int64(cfg.height),
            "groups": np.int64(cfg.groups), "planes": np.int64(cfg.planes),
            "field_kind": np.int64(cfg.field_kind), "n": np.int64(n_steps), "actions": actions.astype(np.int64),
            "accepted": acc, "psnr": ps, "delta": delta, "initial_psnr": np.float64(lg.initial_psnr),
            "final_psnr": np.float64(lg.previous_psnr)}


def build_large(only=()):
    """The headline-size fixtures (minutes of CPU; not rebuilt by the CPU tests):
    DBS_1024_24.py greedy prefixes (amplitude 4096 and 16384 candidates, phase 4096) and the
    literal DBS_ratio_0.5.py run (256x256x8 mono until +0.5 dB, :366-372)."""
    specs = {
        "dbs_prefix_1024x24.npz": lambda: dbs_prefix_large(O.rgb_config(1024), 4096, n_probe=512),
        "dbs_prefix_1024x24_phase.npz":
            lambda: dbs_prefix_large(O.rgb_config(1024, field_kind=O.FIELD_PHASE), 4096),
        "dbs_ratio05_256.npz": lambda: dbs_prefix_large(O.mono_config(256), None, stop_diff=0.5),
        # the 896 x 896 x 24 crop size (env_1024_24_128.py / DBS_1024_24-128.py), 2,048 candidates
        "dbs_prefix_896x24.npz": lambda: dbs_prefix_large(O.rgb_config(896), 2048, seed=7),
        # the headline env step (BASELINE configs[2] semantics) over 2,000 random actions
        "env_trace_1024x24.npz": lambda: env_trace_large(O.rgb_config(1024), 2000),
        # the same amplitude prefix four times longer (~15 min of CPU): its first 4096
        # candidates are dbs_prefix_1024x24.npz's
        "dbs_prefix_1024x24_16k.npz": lambda: dbs_prefix_large(O.rgb_config(1024), 16384),
    }
    return {k: f() for k, f in specs.items() if not only or k in only}


def build_all():
    dt = decode_table()
    s, succ, maxs = reward_table()
    return {
        "decode.npz": {"table": dt},
        "reward.npz": {"success_ratio": s, "success_cubic": succ, "max_steps_cubic": maxs},
        "prop_64_rgb.npz": prop_fixture(small_rgb_cfg, 101),
        "prop_256_mono.npz": prop_fixture(lambda **kw: O.mono_config(256, **kw), 202),
        "env_trace_64.npz": env_trace(),
        "dbs_trace_64.npz": dbs_trace(),
        "probe_64.npz": probe_fixture(),
        "env_group_trace_64.npz": env_group_trace(),
    }


def main():
    large = "--large" in sys.argv
    only = [a for a in sys.argv[1:] if a.endswith(".npz")]
    for name, arrays in (build_large(only) if large else build_all()).items():
        np.savez_compressed(os.path.join(HERE, name), **arrays)
        print("wrote", name)


if __name__ == "__main__":
    main()
