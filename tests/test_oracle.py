"""Oracle pinning (CPU): known answers stated by the reference, analytic
properties of the restated physics, and the committed golden vectors.

Parity note: the floating-point physics (torchOptics) is unpinned -- see the
oracle header; these tests pin what can be pinned."""
import math
import os

import numpy as np
import pytest

from oracle import hbx_oracle as O


# -- known answers from the reference -------------------------------------------------
def test_reward_cubic_known_answers():
    # env.py:228-229: "1 = +300, 1/2 = +100, 1/4 = -100, 1/8 = -300"
    for s, want in ((1.0, 300.0), (0.5, 100.0), (0.25, -100.0), (0.125, -300.0)):
        assert abs(O.success_cubic(s) - want) < 0.05
        assert abs(O.max_steps_cubic(s) - want) < 0.05
    # exact values of the reference's literal coefficients
    assert O.success_cubic(1.0) == pytest.approx(300.04, abs=1e-9)
    assert O.max_steps_cubic(1.0) == pytest.approx(300.0, abs=1e-9)
    assert O.success_cubic(0.5) == pytest.approx(100.03875, abs=1e-9)
    assert O.success_cubic(0.125) == pytest.approx(-299.96185546875, abs=1e-9)


@pytest.mark.parametrize("n,ch", [(256, 8), (1024, 24)])
def test_decode_edges(n, ch):
    hw = n * n
    assert tuple(int(v) for v in O.decode_action(0, n, n)) == (0, 0, 0)
    assert tuple(int(v) for v in O.decode_action(hw - 1, n, n)) == (0, n - 1, n - 1)
    assert tuple(int(v) for v in O.decode_action(hw, n, n)) == (1, 0, 0)
    assert tuple(int(v) for v in O.decode_action(ch * hw - 1, n, n)) == (ch - 1, n - 1, n - 1)
    a = np.random.default_rng(0).integers(0, ch * hw, 1000)
    c, r, col = O.decode_action(a, n, n)
    assert np.array_equal(O.encode_action(c, r, col, n, n), a)


def test_decode_matches_reference_formula():
    # the literal python of env.py:158-161 on python ints
    for a in (0, 1, 65535, 65536, 524287, 25165823, 12345678):
        for ips in (256, 1024):
            ch, pi = a // (ips * ips), a % (ips * ips)
            want = (ch, pi // ips, pi % ips)
            assert tuple(int(v) for v in O.decode_action(a, ips, ips)) == want


def test_pack_roundtrip():
    m = (np.random.default_rng(1).random((3, 5, 128)) > 0.5).astype(np.uint8)
    bits = O.pack_mask(m)
    assert bits.shape == (3, 5, 2) and bits.dtype == np.dtype("<u8")
    assert np.array_equal(O.unpack_mask(bits, 128), m)
    # bit j of word w is column 64 w + j
    one = np.zeros((1, 128), np.uint8)
    one[0, 70] = 1
    assert O.pack_mask(one)[0, 1] == np.uint64(1 << 6)


# -- analytic properties of the restated physics ---------------------------------------
def test_parseval_energy_conserved():
    cfg = O.rgb_config(64, planes=2)
    pre, _ = O.synthetic_inputs(cfg, 5)
    mask = (pre >= 0.5).astype(np.uint8)
    prop = O.Propagator(cfg)
    for g in range(3):
        inten = prop.group_intensity(mask, g)
        # |H| = 1 on the propagating band (no evanescent cut at these params)
        assert np.sum(inten) == pytest.approx(mask[2 * g:2 * g + 2].sum() / 2.0, rel=1e-12)


def test_plane_wave_invariant():
    cfg = O.mono_config(64)
    mask = np.ones((8, 64, 64), np.uint8)
    inten = O.Propagator(cfg).group_intensity(mask, 0)
    assert np.allclose(inten, 1.0, atol=1e-12)


def test_asm_close_to_fresnel_at_small_angle():
    h_asm = O.transfer_function(64, 64, 7.56e-6, 7.56e-6, 515e-9, 2e-3, O.TF_ASM)
    h_fr = O.transfer_function(64, 64, 7.56e-6, 7.56e-6, 515e-9, 2e-3, O.TF_FRESNEL)
    # identical up to the global phase and the O((lambda f)^4) term
    ratio = h_asm / h_fr
    ratio /= ratio[0, 0]
    assert np.max(np.abs(np.angle(ratio))) < 0.05


def test_transfer_function_even():
    h = O.transfer_function(64, 64, 7.56e-6, 7.56e-6, 638e-9, 2e-3)
    idx = (-np.arange(64)) % 64
    assert np.allclose(h, h[idx][:, idx])


def test_psnr_stats_identity():
    rng = np.random.default_rng(3)
    x = rng.random((3, 32, 32))
    y = rng.random((3, 32, 32)).astype(np.float32)
    st = np.stack([O.chan_stats(x[g], y[g]) for g in range(3)])
    for rs in (O.REL_LSQ, O.REL_NONE):
        assert O.psnr_from_stats(st, x.size, rs) == pytest.approx(O.relative_psnr(x, y, rs), abs=1e-10)


def test_phase_field_mapping():
    m = np.array([[0, 1]], np.uint8)
    assert np.array_equal(O.mask_to_field(m, O.FIELD_PHASE), np.array([[1.0, -1.0]]))
    assert np.array_equal(O.mask_to_field(m, O.FIELD_AMPLITUDE), np.array([[0.0, 1.0]]))


# -- env semantics quirks (env.py:184-259) -----------------------------------------------
def _small_env(**kw):
    cfg = O.OpticsConfig(64, 64, 3, 2, O.WL_RGB)
    pre, tgt = O.synthetic_inputs(cfg, 9)
    env = O.OracleEnv(cfg, **kw)
    env.reset(pre, tgt)
    return env, cfg


def test_rollback_keeps_record_and_never_terminates():
    env, cfg = _small_env(max_steps=3)
    rng = np.random.default_rng(4)
    saw_rollback_at_max = False
    for _ in range(40):
        a = int(rng.integers(0, cfg.channels * 64 * 64))
        c, r, col = (int(v) for v in O.decode_action(a, 64, 64))
        before = env.state_record[c, r, col]
        res = env.step(a)
        assert env.state_record[c, r, col] == np.int8(before + 1)      # record never decremented
        if not res.accepted:
            assert not res.terminated and not res.truncated           # early return (env.py:196)
            if env.steps >= env.max_steps:
                saw_rollback_at_max = True
        else:
            assert res.truncated == (env.steps >= 3)
    assert saw_rollback_at_max


def test_reward_is_800_delta_when_rejected():
    env, cfg = _small_env()
    prev = env.previous_psnr
    for a in range(0, 5000, 97):
        res = env.step(a)
        if not res.accepted:
            assert res.reward == pytest.approx(800.0 * (res.psnr - prev))
        prev = env.previous_psnr


def test_dbs_accept_strict_vs_env_nonstrict():
    assert O.OracleEnv.__dataclass_fields__["accept_rule"].default == 0


def test_premodel_bins():
    assert O.premodel_bin(0.0) == 0 and O.premodel_bin(0.0999) == 0 and O.premodel_bin(0.1) == 1
    assert O.premodel_bin(0.95) == 9 and O.premodel_bin(1.0) == 9 and O.premodel_bin(1.01) == -1


def test_importance_ranks_threshold():
    d = np.array([-0.1, 0.2, 0.05, -0.3, 0.4])
    ranks, thr = O.importance_ranks(d)
    assert thr == pytest.approx((0.2 + 0.05 + 0.4) / 4)
    assert ranks[np.argmax(d)] == pytest.approx(np.poly1d(np.polyfit(
        [10000, 9000, 8000, 5000, 2500, 1], [-0.5, -0.48, -0.45, -0.35, 0, 1], 5))(1.0))


# -- golden vectors: the oracle reproduces the committed fixtures --------------------------
def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def test_golden_decode_and_reward(golden_dir):
    t = _load(golden_dir, "decode.npz")["table"]
    for n, ch, a, c, r, col in t:
        assert tuple(int(v) for v in O.decode_action(a, n, n)) == (c, r, col)
    rw = _load(golden_dir, "reward.npz")
    for s, a, b in zip(rw["success_ratio"], rw["success_cubic"], rw["max_steps_cubic"]):
        assert O.success_cubic(s) == a and O.max_steps_cubic(s) == b


def test_golden_propagation(golden_dir):
    import tests.golden.make_golden as G
    for name, fn in (("prop_64_rgb.npz", G.small_rgb_cfg),
                     ("prop_256_mono.npz", lambda **kw: O.mono_config(256, **kw))):
        d = _load(golden_dir, name)
        mask = O.unpack_mask(d["mask_bits"], d["target"].shape[-1])
        for i, (tf, fk, rs) in enumerate(d["combos"]):
            if i > 1 and name.startswith("prop_256"):
                break   # keep the CPU suite fast; the GPU tests cover every combo
            c = fn(tf_kind=int(tf), field_kind=int(fk), rel_scale=int(rs))
            prop = O.Propagator(c)
            inten = prop.all_intensity(mask)
            st = np.stack([O.chan_stats(inten[g], d["target"][g]) for g in range(c.groups)])
            assert np.allclose(st, d["stats"][i], rtol=1e-12, atol=1e-9)
            assert prop.psnr(st) == pytest.approx(float(d["psnr"][i]), abs=1e-10)


def test_golden_env_trace(golden_dir):
    d = _load(golden_dir, "env_trace_64.npz")
    cfg = O.OpticsConfig(64, 64, 3, 2, O.WL_RGB)
    ms, tp, ts, td = d["params"]
    env = O.OracleEnv(cfg, max_steps=int(ms), T_PSNR=float(tp), T_steps=int(ts), T_PSNR_DIFF=float(td))
    assert env.reset(d["pre_model"], d["target"]) == pytest.approx(float(d["initial_psnr"]), abs=1e-10)
    for k, a in enumerate(d["actions"][:60]):
        r = env.step(int(a))
        assert r.psnr == pytest.approx(float(d["psnr"][k]), abs=1e-10)
        assert r.reward == pytest.approx(float(d["reward"][k]), abs=1e-7)
        assert (r.accepted, r.terminated, r.truncated) == (
            bool(d["accepted"][k]), bool(d["terminated"][k]), bool(d["truncated"][k]))


def test_golden_dbs_prefix(golden_dir):
    d = _load(golden_dir, "dbs_trace_64.npz")
    cfg = O.OpticsConfig(64, 64, 3, 2, O.WL_RGB)
    env = O.OracleEnv(cfg, accept_rule=1)
    env.reset(d["pre_model"], d["target"])
    acc, ps, _ = O.dbs_greedy(env, d["order"][:300])
    assert np.array_equal(acc, d["accepted"][:300])
    assert np.allclose(ps, d["psnr"][:300], atol=1e-10)


def test_env_group_trace_golden(golden_dir):
    """The importance-reward oracle (env_group.py) reproduces its committed trace."""
    import importlib.util, os
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(golden_dir, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    d = np.load(os.path.join(golden_dir, "env_group_trace_64.npz"))
    got = mg.env_group_trace()
    for k in ("sample", "changes", "importance", "actions", "accepted", "terminated", "truncated"):
        assert np.array_equal(got[k], d[k]), k
    assert np.allclose(got["reward"], d["reward"], rtol=0, atol=1e-12)
    assert float(got["t_psnr_diff"]) == float(d["t_psnr_diff"])


def test_importance_values_match_reference_formula():
    """hbx/importance.py vs the oracle (env_group.py:121-143,198), incl. ties."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "binary-hologram-reinforcement-learning_amd"))
    from hbx.importance import importance_values
    rng = np.random.default_rng(3)
    ch = rng.normal(0, 1e-3, 10000)
    ch[5:50] = ch[0]                      # duplicated draws (ties)
    v, t = importance_values(ch)
    w, u = O.importance_ranks(ch)
    assert np.array_equal(v, w) and t == u
    # the polynomial passes through the reference's six anchor points
    from hbx.importance import rank_polynomial, STEP_POLY, REWARDS_POLY
    assert np.allclose(rank_polynomial()(STEP_POLY), REWARDS_POLY, atol=1e-9)


@pytest.mark.parametrize("field_kind", [O.FIELD_AMPLITUDE, O.FIELD_PHASE])
def test_linear_greedy_equals_repropagating_oracle(field_kind):
    """O.LinearGreedy (increments by linearity of tt.simulate) reproduces the
    re-propagating serial DBS (DBS_1024_24.py:313-422) decision for decision."""
    cfg = O.OpticsConfig(64, 64, 3, 2, O.WL_RGB, field_kind=field_kind)
    pre, tgt = O.synthetic_inputs(cfg, 21)
    env = O.OracleEnv(cfg, accept_rule=1)
    env.reset(pre, tgt)
    order = np.random.default_rng(3).permutation(cfg.channels * 64 * 64)[:400]
    acc, ps, final = O.dbs_greedy(env, order)
    lg = O.LinearGreedy(cfg, pre, tgt)
    acc2, ps2, delta = lg.run(order)
    assert np.array_equal(acc, acc2)
    assert np.max(np.abs(ps - ps2)) <= 1e-12
    assert np.max(np.abs(lg.intensity - env.intensity)) <= 1e-12
    assert np.array_equal(lg.state, env.state)
    assert abs(lg.previous_psnr - final) <= 1e-12


def test_fill_admissible_rule_and_host_copy_agree():
    """The on-pixel ratio constraint (EXTENSION, BASELINE configs[4]; no reference counterpart,
    SURVEY F7): within tol of the target, or closer to it.  hbx.dbs.fill_admissible (the host
    decisions) and the oracle's are the same rule (the device's is hbx_walk_planes.hpp's)."""
    from hbx.dbs import fill_admissible as host_rule
    for count in range(0, 12):
        for target in (4, 5, 6):
            for tol in (0, 1, 2):
                for bit in (0, 1):
                    d = -1 if bit else 1
                    want = abs(count + d - target) <= tol or abs(count + d - target) < abs(count - target)
                    assert O.fill_admissible(count, target, tol, bit) == want == host_rule(count, target, tol, bit)


@pytest.mark.parametrize("field_kind", [O.FIELD_AMPLITUDE, O.FIELD_PHASE])
def test_fill_constrained_greedy_linear_equals_repropagating(field_kind):
    """The constrained serial loop: LinearGreedy and the re-propagating dbs_greedy make the same
    decisions, rejected candidates are NaN and were never accepted, and the per-group on-pixel
    deviation from the target never grows past max(initial deviation, tol)."""
    cfg = O.OpticsConfig(64, 64, 3, 2, O.WL_RGB, field_kind=field_kind)
    pre, tgt = O.synthetic_inputs(cfg, 23)
    env = O.OracleEnv(cfg, accept_rule=1)
    env.reset(pre, tgt)
    order = np.random.default_rng(5).permutation(cfg.channels * 64 * 64)[:500]
    per_group = cfg.planes * 64 * 64
    target, tol = per_group // 2, 1
    dev0 = np.abs(O.group_fill_counts(env.state, cfg.groups) - target)
    acc, ps, _ = O.dbs_greedy(env, order, fill=(target, tol))
    lg = O.LinearGreedy(cfg, pre, tgt)
    acc2, ps2, _ = lg.run(order, fill=(target, tol))
    assert np.array_equal(acc, acc2)
    assert np.array_equal(np.isnan(ps), np.isnan(ps2))
    ok = ~np.isnan(ps)
    assert np.max(np.abs(ps[ok] - ps2[ok])) <= 1e-12
    assert np.isnan(ps).any() and not acc[np.isnan(ps)].any()
    counts = O.group_fill_counts(env.state, cfg.groups)
    assert np.array_equal(counts, lg.fill_counts)
    assert np.all(np.abs(counts - target) <= np.maximum(dev0, tol))
    # unconstrained, the same order accepts differently (the constraint binds)
    env2 = O.OracleEnv(cfg, accept_rule=1)
    env2.reset(pre, tgt)
    acc3, _, _ = O.dbs_greedy(env2, order)
    assert not np.array_equal(acc, acc3)


@pytest.mark.parametrize("name,n_check", [("dbs_prefix_1024x24.npz", 12), ("dbs_ratio05_256.npz", 300)])
def test_large_dbs_fixtures_reproduce(golden_dir, name, n_check):
    """The headline-size DBS fixtures (make_golden.py --large) against a fresh
    oracle run of their first candidates (the full runs take minutes)."""
    import os
    d = np.load(os.path.join(golden_dir, name), allow_pickle=False)
    n, g = int(d["size"]), int(d["groups"])
    cfg = O.OpticsConfig(n, n, g, int(d["planes"]), O.WL_RGB if g == 3 else O.WL_MONO,
                         field_kind=int(d["field_kind"]))
    pre, tgt = O.synthetic_inputs(cfg, int(d["seed"]))
    order = np.random.default_rng(int(d["order_seed"])).permutation(cfg.channels * n * n)[:n_check]
    lg = O.LinearGreedy(cfg, pre, tgt)
    assert lg.initial_psnr == pytest.approx(float(d["initial_psnr"]), abs=1e-10)
    acc, ps, delta = lg.run(order)
    assert np.array_equal(acc, d["accepted"][:n_check])
    assert np.allclose(delta, d["delta"][:n_check], rtol=0, atol=1e-12)


def test_long_dbs_prefix_extends_the_4096_fixture(golden_dir):
    """dbs_prefix_1024x24_16k.npz (16,384 candidates) and dbs_prefix_1024x24.npz (4,096)
    come from the same seeded image and order: the long run's first 4,096 decisions,
    PSNRs and changes are the short one's."""
    import os
    a = np.load(os.path.join(golden_dir, "dbs_prefix_1024x24.npz"), allow_pickle=False)
    b = np.load(os.path.join(golden_dir, "dbs_prefix_1024x24_16k.npz"), allow_pickle=False)
    n = int(a["n"])
    assert int(b["n"]) == 16384 and n == 4096
    for k in ("seed", "order_seed", "size", "groups", "planes", "field_kind"):
        assert int(a[k]) == int(b[k])
    assert np.array_equal(a["accepted"], b["accepted"][:n])
    assert np.array_equal(a["psnr"], b["psnr"][:n]) and np.array_equal(a["delta"], b["delta"][:n])
    assert float(a["initial_psnr"]) == float(b["initial_psnr"])


def test_env_trace_1024x24_matches_the_stepping_env(golden_dir):
    """env_trace_1024x24.npz (LinearGreedy.run_env, 2,000 steps) against the
    re-propagating OracleEnv.step (env.py:154-258) over its first steps: same accept
    flags, PSNRs and rewards (reward = 800 * change, no terminal bonus inside the trace)."""
    import os
    d = np.load(os.path.join(golden_dir, "env_trace_1024x24.npz"), allow_pickle=False)
    n = int(d["size"])
    cfg = O.OpticsConfig(n, n, int(d["groups"]), int(d["planes"]), O.WL_RGB, field_kind=int(d["field_kind"]))
    pre, tgt = O.synthetic_inputs(cfg, int(d["seed"]))
    acts = np.random.default_rng(int(d["action_seed"])).integers(0, cfg.channels * n * n, int(d["n"]))
    assert np.array_equal(acts, d["actions"])
    env = O.OracleEnv(cfg)
    assert env.reset(pre, tgt) == pytest.approx(float(d["initial_psnr"]), abs=1e-10)
    for i in range(6):
        s = env.step(int(acts[i]))
        assert s.accepted == bool(d["accepted"][i]) and not s.terminated
        assert s.psnr == pytest.approx(float(d["psnr"][i]), abs=1e-10)
        assert s.reward == pytest.approx(O.RW * float(d["delta"][i]), abs=1e-8)
    assert 0.3 < d["accepted"].mean() < 0.7
    assert float(d["final_psnr"]) - float(d["initial_psnr"]) < 0.1     # stays short of T_PSNR_DIFF
