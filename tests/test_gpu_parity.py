"""Parity of the HIP path (libhbx.so via hbx) with the float64 oracle.

Tolerances (north_star: "PSNR within 1e-4 of numpy"):
  PSNR            |gpu - oracle| <= 1e-4 dB
  channel stats   relative 2e-5 (fp32 FFT, f64 accumulation)
  intensity       max |gpu - oracle| <= 2e-5 * max(oracle)
  flip indexing, masks, records, accept / terminate / truncate flags: bit-exact
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import hbx_oracle as O  # noqa: E402

PSNR_TOL = 1e-4
STATS_RTOL = 2e-5


def _require_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm GPU")


def dev_cfg(o: O.OpticsConfig):
    import hbx
    return hbx.OpticsConfig(o.height, o.width, o.groups, o.planes, tuple(o.wavelengths), o.dx, o.dy, o.z,
                            o.tf_kind, o.field_kind, o.rel_scale, o.peak)


def small_rgb(**kw):
    return O.OpticsConfig(64, 64, 3, 2, O.WL_RGB, **kw)


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def to_dev_bits(bits: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(bits).view(np.int64)).cuda()


@pytest.fixture(scope="module", autouse=True)
def gpu():
    _require_gpu()
    import hbx
    hbx.load_library()
    yield


# -- propagation -------------------------------------------------------------------------
@pytest.mark.parametrize("name,fn", [("prop_64_rgb.npz", small_rgb),
                                     ("prop_256_mono.npz", lambda **kw: O.mono_config(256, **kw))])
def test_propagate_golden_all_switches(golden_dir, name, fn):
    import hbx
    d = load(golden_dir, name)
    bits = to_dev_bits(d["mask_bits"])[None]
    tgt = torch.from_numpy(d["target"]).cuda()[None]
    for i, (tf, fk, rs) in enumerate(d["combos"]):
        cfg = dev_cfg(fn(tf_kind=int(tf), field_kind=int(fk), rel_scale=int(rs)))
        plan = hbx.Plan(cfg, max_jobs=cfg.groups)
        inten, stats, psnr = plan.propagate(bits, tgt)
        torch.cuda.synchronize()
        st = stats[0].cpu().numpy()
        assert np.allclose(st, d["stats"][i], rtol=STATS_RTOL), (tf, fk, rs)
        assert abs(float(psnr[0]) - float(d["psnr"][i])) <= PSNR_TOL, (tf, fk, rs)
        if i == 0:
            ref = d["intensity"]
            got = inten[0].cpu().numpy()
            assert np.max(np.abs(got - ref)) <= 2e-5 * np.max(ref)
        plan.close()


def test_propagate_1024_rgb_vs_oracle():
    import hbx
    ocfg = O.rgb_config(1024)
    pre, tgt = O.synthetic_inputs(ocfg, 0)
    mask = (pre >= 0.5).astype(np.uint8)
    prop = O.Propagator(ocfg)
    ref_i = prop.all_intensity(mask)
    ref_st = np.stack([O.chan_stats(ref_i[g], tgt[g]) for g in range(3)])
    plan = hbx.Plan(dev_cfg(ocfg), max_jobs=3)
    inten, stats, psnr = plan.propagate(to_dev_bits(O.pack_mask(mask))[None], torch.from_numpy(tgt).cuda()[None])
    torch.cuda.synchronize()
    assert np.allclose(stats[0].cpu().numpy(), ref_st, rtol=STATS_RTOL)
    assert abs(float(psnr[0]) - prop.psnr(ref_st)) <= PSNR_TOL
    got = inten[0].cpu().numpy()
    assert np.max(np.abs(got - ref_i)) <= 2e-5 * np.max(ref_i)


def test_parseval_full_size_batch():
    """Size-independent property at the benchmark size (1024 x 24, B=4):
    sum_xy I_g = popcount(group) / P exactly (|H| = 1, no evanescent cut)."""
    import hbx
    cfg = hbx.rgb_config(1024)
    g = torch.Generator(device="cuda").manual_seed(5)
    pre = torch.rand((4, 24, 1024, 1024), generator=g, device="cuda")
    bits = hbx.pack_bits(pre >= 0.5)
    tgt = torch.rand((4, 3, 1024, 1024), generator=g, device="cuda")
    plan = hbx.Plan(cfg, max_jobs=6)
    inten, stats, psnr = plan.propagate(bits, tgt)
    pop = (pre >= 0.5).reshape(4, 3, 8, -1).sum(dim=(2, 3)).double() / 8.0
    s = inten.double().sum(dim=(2, 3))
    assert torch.allclose(s, pop, rtol=2e-6)
    # the stats' sum I^2 matches the returned intensity
    assert torch.allclose(stats[..., 1], (inten.double() ** 2).sum(dim=(2, 3)), rtol=1e-9)


def test_deterministic_bitwise():
    import hbx
    cfg = hbx.rgb_config(256)
    g = torch.Generator(device="cuda").manual_seed(1)
    bits = hbx.pack_bits(torch.rand((2, 24, 256, 256), generator=g, device="cuda") >= 0.5)
    tgt = torch.rand((2, 3, 256, 256), generator=g, device="cuda")
    plan = hbx.Plan(cfg, max_jobs=4)   # forces two chunks
    a = plan.propagate(bits, tgt)
    b = plan.propagate(bits, tgt)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])


def test_pack_bits_matches_oracle():
    import hbx
    m = (np.random.default_rng(2).random((3, 4, 128)) > 0.5).astype(np.uint8)
    got = hbx.pack_bits(torch.from_numpy(m).cuda()).cpu().numpy().view("<u8")
    assert np.array_equal(got, O.pack_mask(m))
    assert np.array_equal(hbx.unpack_bits(torch.from_numpy(got.view(np.int64)).cuda(), 128).cpu().numpy(), m)


# -- trial flips ---------------------------------------------------------------------------
def test_eval_flips_probe_golden(golden_dir):
    import hbx
    from hbx import dbs
    d = load(golden_dir, "probe_64.npz")
    cfg = dev_cfg(small_rgb())
    plan = hbx.Plan(cfg, max_jobs=256)
    mask = hbx.pack_bits(torch.from_numpy(d["pre_model"]).cuda() >= 0.5)
    res = dbs.probe(plan, mask, torch.from_numpy(d["target"]).cuda(), d["flips"], pre_model=d["pre_model"])
    assert abs(res.base_psnr - float(d["base_psnr"])) <= PSNR_TOL
    assert np.max(np.abs(res.psnr - d["psnr"])) <= PSNR_TOL
    delta = d["psnr"] - d["base_psnr"]
    clear = np.abs(delta) > 1e-5          # fp32 cannot order ties below this
    assert np.array_equal(res.improved[clear], (delta > 0)[clear])
    assert np.array_equal(res.attempted_bins, d["attempted"])
    assert np.sum(np.abs(res.improved_bins - d["improved"])) <= np.sum(~clear)


def test_eval_flips_1024_vs_oracle():
    import hbx
    ocfg = O.rgb_config(1024)
    pre, tgt = O.synthetic_inputs(ocfg, 3)
    env = O.OracleEnv(ocfg)
    env.reset(pre, tgt)
    flips = np.array([0, 1024 * 1024 - 1, 9 * 1024 * 1024 + 5 * 1024 + 77, 24 * 1024 * 1024 - 1], np.int64)
    want = [env.evaluate_flip(int(a))[0] for a in flips]
    plan = hbx.Plan(dev_cfg(ocfg), max_jobs=4)
    bits = to_dev_bits(O.pack_mask((pre >= 0.5).astype(np.uint8)))
    _, st, _ = plan.propagate(bits[None], torch.from_numpy(tgt).cuda()[None])
    got, _ = plan.eval_flips(bits, torch.from_numpy(tgt).cuda(), st[0].contiguous(),
                             torch.from_numpy(flips).cuda())
    assert np.max(np.abs(got.cpu().numpy() - np.array(want))) <= PSNR_TOL


# -- env semantics ---------------------------------------------------------------------------
def test_env_trace_golden(golden_dir):
    import hbx
    from hbx.env import HologramVecEnv
    d = load(golden_dir, "env_trace_64.npz")
    ms, tp, ts, td = d["params"]
    cfg = dev_cfg(small_rgb())
    env = HologramVecEnv(cfg, 1, lambda i: d["target"], pre_model_source=lambda i: d["pre_model"],
                         max_steps=int(ms), T_PSNR=float(tp), T_steps=int(ts), T_PSNR_DIFF=float(td),
                         auto_reset=False)
    env.reset()
    assert abs(float(env.state.init_psnr[0]) - float(d["initial_psnr"])) <= PSNR_TOL
    for k, a in enumerate(d["actions"]):
        r, ps, acc, term, trunc = env.step_device(torch.tensor([int(a)], device="cuda"))
        assert abs(float(ps[0]) - float(d["psnr"][k])) <= PSNR_TOL, k
        assert abs(float(r[0]) - float(d["reward"][k])) <= 800 * PSNR_TOL, k
        assert (bool(acc[0]), bool(term[0]), bool(trunc[0])) == (
            bool(d["accepted"][k]), bool(d["terminated"][k]), bool(d["truncated"][k])), k
    fm = env.state.mask[0].cpu().numpy().view("<u8")
    assert np.array_equal(fm, d["final_mask_bits"])
    assert np.array_equal(env.state.record[0].cpu().numpy(), d["final_record"])
    assert int(env.state.steps[0]) == len(d["actions"])


def test_vecenv_batch_matches_oracle_per_env():
    import hbx
    from hbx.env import HologramVecEnv
    ocfg = small_rgb()
    B = 6
    ins = [O.synthetic_inputs(ocfg, 100 + b) for b in range(B)]
    env = HologramVecEnv(dev_cfg(ocfg), B, lambda i: ins[i][1], pre_model_source=lambda i: ins[i][0],
                         auto_reset=False)
    env.reset()
    oenvs = [O.OracleEnv(ocfg) for _ in range(B)]
    for b in range(B):
        oenvs[b].reset(*ins[b])
    rng = np.random.default_rng(8)
    for _ in range(25):
        acts = rng.integers(0, ocfg.channels * 64 * 64, B)
        r, ps, acc, term, trunc = env.step_device(torch.from_numpy(acts).cuda())
        ps, acc = ps.cpu().numpy(), acc.cpu().numpy()
        for b in range(B):
            want = oenvs[b].step(int(acts[b]))
            assert abs(ps[b] - want.psnr) <= PSNR_TOL
            assert bool(acc[b]) == want.accepted


@pytest.mark.parametrize("size,mono", [(1024, False), (256, True)])
def test_env_steps_full_size_vs_oracle(size, mono):
    """The headline configuration (1024x1024x24 RGB) and env.py's 256x256x8 mono:
    per-step PSNR and reward against the float64 oracle evaluated on the SAME
    state (the oracle follows the GPU's accept decisions), and the decisions
    themselves wherever the PSNR change is clear of fp32 resolution (1e-5 dB;
    a single flip moves the 1024x24 PSNR by ~1e-6 dB, below what an f32 field
    can order against an f64 reference)."""
    from hbx.env import HologramVecEnv
    ocfg = O.mono_config(size) if mono else O.rgb_config(size)
    pre, tgt = O.synthetic_inputs(ocfg, 3)
    env = HologramVecEnv(dev_cfg(ocfg), 1, lambda i: tgt, pre_model_source=lambda i: pre, auto_reset=False,
                         obs_keys=())
    env.reset()
    oe = O.OracleEnv(ocfg)
    oe.reset(pre, tgt)
    assert abs(float(env.state.init_psnr[0]) - oe.initial_psnr) <= PSNR_TOL
    rng = np.random.default_rng(4)
    clear = 0
    for _ in range(8):
        a = int(rng.integers(0, ocfg.channels * size * size))
        r, ps, acc, _, _ = env.step_device(torch.tensor([a], device="cuda"))
        want, g, ig, st = oe.evaluate_flip(a)
        change = want - oe.previous_psnr
        assert abs(float(ps[0]) - want) <= PSNR_TOL
        assert abs(float(r[0]) - O.RW * change) <= O.RW * 2 * PSNR_TOL
        if abs(change) > 1e-5:
            clear += 1
            assert bool(acc[0]) == (change >= 0)
        if bool(acc[0]):                       # follow the GPU's decision
            ch, row, col = (int(v) for v in O.decode_action(a, size, size))
            oe.state[ch, row, col] ^= 1
            oe.stats, oe.intensity[g], oe.previous_psnr = st, ig, want
    assert torch.equal(env.state.mask[0].cpu(), torch.from_numpy(O.pack_mask(oe.state.astype(np.uint8)).view(np.int64)))
    if mono:
        assert clear > 0


def test_invalid_action_raises():
    from hbx.env import HologramVecEnv
    ocfg = small_rgb()
    pre, tgt = O.synthetic_inputs(ocfg, 1)
    env = HologramVecEnv(dev_cfg(ocfg), 1, lambda i: tgt, pre_model_source=lambda i: pre, auto_reset=False)
    env.reset()
    with pytest.raises(ValueError):
        env.step(np.array([ocfg.channels * 64 * 64]))


def test_vecenv_auto_reset_and_obs():
    from hbx.env import HologramVecEnv
    ocfg = small_rgb()
    pre, tgt = O.synthetic_inputs(ocfg, 2)
    env = HologramVecEnv(dev_cfg(ocfg), 2, lambda i: tgt, pre_model_source=lambda i: pre, max_steps=3)
    obs = env.reset()
    assert obs["state"].shape == (2, 1, 6, 64, 64) and obs["recon_image"].shape == (2, 1, 3, 64, 64)
    assert np.array_equal(obs["state"][0, 0].cpu().numpy(), (pre >= 0.5).astype(np.int8))
    seen_done = False
    rng = np.random.default_rng(0)
    for _ in range(40):
        obs, rew, dones, infos = env.step(rng.integers(0, 6 * 4096, 2))
        if dones.any():
            seen_done = True
            i = int(np.nonzero(dones)[0][0])
            assert "terminal_observation" in infos[i]
            assert int(env.state.steps[i]) == 0       # auto-reset happened
    assert seen_done


@pytest.mark.parametrize("mode", ["fft", "psf"])
def test_vecenv_save_load_resume(tmp_path, mode):
    """HologramVecEnv.save / load: a restored env continues bit-identically."""
    from hbx.env import HologramVecEnv
    cfg = dev_cfg(small_rgb())
    B = 3
    gens = [torch.Generator(device="cuda").manual_seed(40 + i) for i in range(B)]
    pres = [torch.rand((cfg.channels, 64, 64), generator=g, device="cuda") for g in gens]
    tgts = [torch.rand((cfg.groups, 64, 64), generator=g, device="cuda") for g in gens]
    keys = ("state_record", "state") if mode == "psf" else ("state_record", "state", "recon_image")
    kw = dict(pre_model_source=lambda i: pres[i], obs_keys=keys, auto_reset=False, mode=mode, refresh_every=0)
    a = HologramVecEnv(cfg, B, lambda i: tgts[i], **kw)
    a.reset()
    acts = torch.randint(0, cfg.channels * 64 * 64, (24, B), generator=gens[0], device="cuda")
    for k in range(12):
        a.step_device(acts[k])
    if mode == "psf":
        a.refresh()
    path = str(tmp_path / "env.npz")
    a.save(path)
    b = HologramVecEnv(cfg, B, lambda i: tgts[(i + 1) % B], **kw)
    b.reset()
    b.load(path)
    for k in range(12, 24):
        ra, rb = a.step_device(acts[k]), b.step_device(acts[k])
        for x, y in zip(ra, rb):
            assert torch.equal(x, y)
    for name in ("mask", "record", "chan_stats", "steps", "flip_count", "prev_psnr"):
        assert torch.equal(getattr(a.state, name), getattr(b.state, name)), name
    c = HologramVecEnv(cfg, B + 1, lambda i: tgts[0], **kw)
    with pytest.raises(ValueError):
        c.load(path)
    for e in (a, b, c):
        e.close()


# -- DBS --------------------------------------------------------------------------------------
def test_dbs_greedy_speculative_equals_serial(golden_dir):
    import hbx
    from hbx import dbs
    d = load(golden_dir, "dbs_trace_64.npz")
    plan = hbx.Plan(dev_cfg(small_rgb()), max_jobs=128)
    mask = hbx.pack_bits(torch.from_numpy(d["pre_model"]).cuda() >= 0.5)
    res = dbs.greedy(plan, mask, torch.from_numpy(d["target"]).cuda(), d["order"])
    want_pos = np.nonzero(d["accepted"])[0]
    assert np.array_equal(np.array(res.accepted_positions), want_pos)
    assert abs(res.final_psnr - float(d["final_psnr"])) <= PSNR_TOL
    assert np.array_equal(mask.cpu().numpy().view("<u8"), d["final_mask_bits"])
    assert res.launches < len(d["order"])      # speculation batched the walk


def test_dbs_early_stop():
    import hbx
    from hbx import dbs
    ocfg = small_rgb()
    pre, tgt = O.synthetic_inputs(ocfg, 21)
    order = np.random.default_rng(3).permutation(ocfg.channels * 64 * 64)
    plan = hbx.Plan(dev_cfg(ocfg), max_jobs=64)
    mask = hbx.pack_bits(torch.from_numpy(pre).cuda() >= 0.5)
    res = dbs.greedy(plan, mask, torch.from_numpy(tgt).cuda(), order, stop_diff=0.05)
    env = O.OracleEnv(ocfg, accept_rule=1)
    env.reset(pre, tgt)
    acc, ps, final = O.dbs_greedy(env, order, stop_diff=0.05)
    assert res.stopped_early
    assert res.steps == len(acc)
    assert abs(res.final_psnr - final) <= PSNR_TOL


# -- incremental-field (PSF) mode --------------------------------------------------------------
def test_psf_env_trace_golden(golden_dir):
    from hbx.env import HologramVecEnv
    d = load(golden_dir, "env_trace_64.npz")
    ms, tp, ts, td = d["params"]
    env = HologramVecEnv(dev_cfg(small_rgb()), 1, lambda i: d["target"],
                         pre_model_source=lambda i: d["pre_model"], max_steps=int(ms), T_PSNR=float(tp),
                         T_steps=int(ts), T_PSNR_DIFF=float(td), auto_reset=False, mode="psf",
                         obs_keys=("state", "target_image"), refresh_every=64)
    env.reset()
    for k, a in enumerate(d["actions"]):
        r, ps, acc, term, trunc = env.step_device(torch.tensor([int(a)], device="cuda"))
        assert abs(float(ps[0]) - float(d["psnr"][k])) <= PSNR_TOL, k
        assert (bool(acc[0]), bool(term[0]), bool(trunc[0])) == (
            bool(d["accepted"][k]), bool(d["terminated"][k]), bool(d["truncated"][k])), k
    assert np.array_equal(env.state.mask[0].cpu().numpy().view("<u8"), d["final_mask_bits"])
    assert np.array_equal(env.state.record[0].cpu().numpy(), d["final_record"])


def test_psf_field_matches_oracle():
    from hbx.env import HologramVecEnv
    ocfg = small_rgb()
    pre, tgt = O.synthetic_inputs(ocfg, 4)
    env = HologramVecEnv(dev_cfg(ocfg), 1, lambda i: tgt, pre_model_source=lambda i: pre, mode="psf",
                         obs_keys=(), auto_reset=False)
    env.reset()
    mask = (pre >= 0.5).astype(np.uint8)
    prop = O.Propagator(ocfg)
    for g in range(3):
        u = O.propagate(O.mask_to_field(mask[2 * g:2 * g + 2]), prop.h[g])
        got = env.state.field[0, 2 * g:2 * g + 2].cpu().numpy()
        got = got[..., 0] + 1j * got[..., 1]
        assert np.max(np.abs(got - u)) <= 2e-5 * np.max(np.abs(u))
        assert np.allclose(env.state.intensity[0, g].cpu().numpy(), prop.group_intensity(mask, g),
                           atol=2e-5 * np.max(np.abs(u)) ** 2)


@pytest.mark.parametrize("field_kind", [O.FIELD_AMPLITUDE, O.FIELD_PHASE])
def test_psf_matches_fft_full_size(field_kind):
    """1024 x 24, 4 envs, 40 steps: the incremental mode and the FFT mode agree."""
    import hbx
    from hbx.env import HologramVecEnv
    cfg = hbx.rgb_config(1024, field_kind=field_kind)
    B = 4
    gens = [torch.Generator(device="cuda").manual_seed(50 + i) for i in range(B)]
    pres = [torch.rand((24, 1024, 1024), generator=g, device="cuda") for g in gens]
    tgts = [torch.rand((3, 1024, 1024), generator=g, device="cuda") for g in gens]
    kw = dict(pre_model_source=lambda i: pres[i], obs_keys=(), auto_reset=False)
    fft = HologramVecEnv(cfg, B, lambda i: tgts[i], **kw)
    psf = HologramVecEnv(cfg, B, lambda i: tgts[i], mode="psf", refresh_every=16, **kw)
    fft.reset()
    psf.reset()
    assert torch.allclose(fft.state.init_psnr, psf.state.init_psnr, atol=1e-9)
    acts = torch.randint(0, 24 * 1024 * 1024, (40, B), generator=gens[0], device="cuda")
    for k in range(40):
        _, p1, a1, _, _ = fft.step_device(acts[k])
        _, p2, a2, _, _ = psf.step_device(acts[k])
        assert torch.max(torch.abs(p1 - p2)).item() <= PSNR_TOL
        d = torch.abs(p1 - fft.state.prev_psnr)
        assert torch.equal(a1, a2) or bool((d < 1e-5).any())
    assert torch.equal(fft.state.mask, psf.state.mask)
    fft.close()
    psf.close()


def test_psf_matches_fft_many_envs():
    """300 envs at 64 x 64 x (3 x 2): more jobs than one 256-job chunk of k_psf_order's
    ballot sort (hbx_psf.hip), all three colour groups mixed in every step; the
    incremental and FFT modes agree step by step (PSNR, accept flags) and end on the
    same masks."""
    from hbx.env import HologramVecEnv
    cfg = dev_cfg(small_rgb())
    B = 300
    g = torch.Generator(device="cuda").manual_seed(7)
    pres = torch.rand((B, 6, 64, 64), generator=g, device="cuda")
    tgts = torch.rand((B, 3, 64, 64), generator=g, device="cuda")
    kw = dict(pre_model_source=lambda i: pres[i], obs_keys=(), auto_reset=False)
    fft = HologramVecEnv(cfg, B, lambda i: tgts[i], **kw)
    psf = HologramVecEnv(cfg, B, lambda i: tgts[i], mode="psf", refresh_every=8, **kw)
    fft.reset()
    psf.reset()
    acts = torch.randint(0, 6 * 64 * 64, (12, B), generator=g, device="cuda")
    for k in range(12):
        prev = fft.state.prev_psnr.clone()
        _, p1, a1, _, _ = fft.step_device(acts[k])
        _, p2, a2, _, _ = psf.step_device(acts[k])
        assert torch.max(torch.abs(p1 - p2)).item() <= PSNR_TOL
        differ = a1 != a2
        assert bool((torch.abs(p1 - prev)[differ] < 1e-5).all()), f"step {k}: decisions differ"
    assert torch.equal(fft.state.mask, psf.state.mask)
    fft.close()
    psf.close()


# ---------------------------------------------------------------------------
# all-flip PSNR-change map (hbx_flip_map, correlation evaluation)
# ---------------------------------------------------------------------------
MAP_TOL = 1e-8   # dB: the map evaluates each flip's increments directly (measured
                 # <= 1e-9 dB at 64^2 / 256^2 and ~1e-12 dB at 1024^2 against the f64 oracle)


def test_flip_map_probe_golden(golden_dir):
    import hbx
    from hbx import dbs
    d = load(golden_dir, "probe_64.npz")
    cfg = dev_cfg(small_rgb())
    plan = hbx.Plan(cfg, max_jobs=8)
    mask = hbx.pack_bits(torch.from_numpy(d["pre_model"]).cuda() >= 0.5)
    res = dbs.probe_map(plan, mask, torch.from_numpy(d["target"]).cuda(), d["flips"], pre_model=d["pre_model"])
    assert abs(res.base_psnr - float(d["base_psnr"])) <= PSNR_TOL
    delta = d["psnr"] - d["base_psnr"]
    err = np.max(np.abs((res.psnr - res.base_psnr) - delta))
    assert err <= MAP_TOL, err
    clear = np.abs(delta) > MAP_TOL
    assert np.array_equal(res.improved[clear], (delta > 0)[clear])
    assert np.array_equal(res.attempted_bins, d["attempted"])
    assert np.sum(np.abs(res.improved_bins - d["improved"])) <= np.sum(~clear)
    assert np.allclose(res.delta_bins, d["delta_sum"], rtol=0, atol=2048 * MAP_TOL)


@pytest.mark.parametrize("field", ["amplitude", "phase"])
def test_flip_map_every_flip_256(field):
    """Every one of the 524 288 flips of a 256x256x8 mono state vs the oracle
    on a sample, and vs hbx_eval_flips (brute-force propagation) on another."""
    import hbx
    fk = O.FIELD_AMPLITUDE if field == "amplitude" else O.FIELD_PHASE
    ocfg = O.mono_config(256, field_kind=fk)
    pre, tgt = O.synthetic_inputs(ocfg, 41)
    env = O.OracleEnv(ocfg)
    base = env.reset(pre, tgt)
    plan = hbx.Plan(dev_cfg(ocfg), max_jobs=256)
    bits = to_dev_bits(O.pack_mask((pre >= 0.5).astype(np.uint8)))
    t = torch.from_numpy(tgt).cuda()
    dmap, b = plan.flip_map(bits, t)
    assert abs(float(b.item()) - base) <= PSNR_TOL
    flat = dmap.reshape(-1).cpu().numpy().astype(np.float64)
    assert np.all(np.isfinite(flat))
    rng = np.random.default_rng(42)
    sample = rng.integers(0, ocfg.channels * 256 * 256, 48)
    want = np.array([env.evaluate_flip(int(a))[0] - base for a in sample])
    err = np.max(np.abs(flat[sample] - want))
    assert err <= MAP_TOL, (err, np.max(np.abs(want)))
    # brute force on the GPU for 256 more
    s2 = torch.from_numpy(rng.integers(0, ocfg.channels * 256 * 256, 256)).cuda()
    _, st, _ = plan.propagate(bits[None], t[None])
    ps, _ = plan.eval_flips(bits, t, st[0].contiguous(), s2)
    assert np.max(np.abs(flat[s2.cpu().numpy()] - (ps.cpu().numpy() - base))) <= PSNR_TOL


def test_flip_map_1024_rgb_vs_eval_flips():
    """Full size (24 x 1024 x 1024 = 25.2 M flips in one call) against brute-force
    propagation of 256 random flips plus the corners of every plane."""
    import hbx
    ocfg = O.rgb_config(1024)
    pre, tgt = O.synthetic_inputs(ocfg, 5)
    plan = hbx.Plan(dev_cfg(ocfg), max_jobs=256)
    bits = to_dev_bits(O.pack_mask((pre >= 0.5).astype(np.uint8)))
    t = torch.from_numpy(tgt).cuda()
    dmap, base = plan.flip_map(bits, t)
    n = 1024 * 1024
    corners = [c * n + off for c in range(24) for off in (0, 1023, n - 1024, n - 1)]
    flips = np.concatenate([np.random.default_rng(6).integers(0, 24 * n, 256), corners]).astype(np.int64)
    f_t = torch.from_numpy(flips).cuda()
    _, st, _ = plan.propagate(bits[None], t[None])
    ps, _ = plan.eval_flips(bits, t, st[0].contiguous(), f_t)
    got = dmap.reshape(-1)[f_t].double().cpu().numpy()
    want = ps.cpu().numpy() - float(base.item())
    err = np.max(np.abs(got - want))
    assert err <= PSNR_TOL, err
    assert bool(torch.isfinite(dmap).all())
    # the map is the more precise of the two (it sums each flip's increment
    # directly; eval_flips subtracts two full-image PSNRs): f64 oracle check
    env = O.OracleEnv(ocfg)
    b0 = env.reset(pre, tgt)
    few = np.array([0, 5 * n + 77, 13 * n + 512 * 1024 + 3, 24 * n - 1])
    exact = np.array([env.evaluate_flip(int(a))[0] - b0 for a in few])
    got = dmap.reshape(-1)[torch.from_numpy(few).cuda()].double().cpu().numpy()
    assert np.max(np.abs(got - exact)) <= MAP_TOL


# ---------------------------------------------------------------------------
# env_group.py importance rewards
# ---------------------------------------------------------------------------
def test_env_group_importance_trace(golden_dir):
    from hbx.env import HologramVecEnv
    d = load(golden_dir, "env_group_trace_64.npz")
    cfg = dev_cfg(small_rgb())
    k = d["sample"].shape[0]
    vec = HologramVecEnv(cfg, 1, lambda i: torch.from_numpy(d["target"]).cuda(),
                         pre_model_source=lambda i: torch.from_numpy(d["pre_model"]).cuda(),
                         max_steps=250, T_PSNR=30.0, T_steps=1, obs_keys=(), auto_reset=False,
                         reward="importance", importance_samples=k, importance_seed=int(d["seed"]))
    vec.reset()
    st = vec.state
    changes = st.imp_changes[0].cpu().numpy()
    assert np.max(np.abs(changes - d["changes"])) <= 1e-8          # read out of the flip map
    tpd = float(st.t_psnr_diff[0].item())
    assert abs(tpd - float(d["t_psnr_diff"])) <= k * 1e-8
    vals = st.imp_values[0].cpu().numpy()
    clear = np.array([np.sum(np.abs(d["changes"] - c) <= 1e-8) == 1 for c in d["changes"]])
    assert np.allclose(vals[clear], d["importance"][clear], rtol=0, atol=1e-9)
    rewards, n_checked = [], 0
    for t, a in enumerate(d["actions"]):
        r, ps, acc, term, trunc = vec.step_device(torch.tensor([int(a)], device="cuda"))
        ps = float(ps.item())
        assert abs(ps - d["psnr"][t]) <= PSNR_TOL
        rewards.append(float(r.item()))
        if abs(float(d["psnr"][t]) - ps) > 1e-7:
            continue
        n_checked += 1
        assert bool(acc.item()) == bool(d["accepted"][t]), t
        assert bool(term.item()) == bool(d["terminated"][t]), t
        assert bool(trunc.item()) == bool(d["truncated"][t]), t
    # reward = importance of the sampled change nearest to the step's change (+ bonus):
    # the device may pick a neighbour rank when two sampled changes are closer than
    # its PSNR error, so compare against every candidate within that margin
    prev = float(d["initial_psnr"])
    for t in range(len(d["actions"])):
        c = d["psnr"][t] - prev
        dist = np.abs(d["changes"] - c)
        cand = d["importance"][dist <= dist.min() + 2 * 1e-7]
        bonus = d["reward"][t] - d["importance"][np.argmin(dist)]
        assert np.min(np.abs(cand + bonus - rewards[t])) <= 1e-6, t
        if d["accepted"][t]:
            prev = d["psnr"][t]
    assert n_checked > 200
    vec.close()


def test_multidiscrete_actions_match_discrete(golden_dir):
    """env_md.py: MultiDiscrete([CH, IPS, IPS]) actions step exactly like the
    flat Discrete index c*H*W + r*W + col."""
    from hbx.env import HologramVecEnv
    d = load(golden_dir, "env_trace_64.npz")
    cfg = dev_cfg(small_rgb())
    mk = lambda fmt: HologramVecEnv(cfg, 1, lambda i: torch.from_numpy(d["target"]).cuda(),  # noqa: E731
                                    pre_model_source=lambda i: torch.from_numpy(d["pre_model"]).cuda(),
                                    obs_keys=(), auto_reset=False, action_format=fmt)
    a, b = mk("discrete"), mk("multidiscrete")
    a.reset(), b.reset()
    assert tuple(b.action_space.nvec) == (cfg.channels, 64, 64)
    for act in d["actions"][:60]:
        c, k = divmod(int(act), 64 * 64)
        ra = [t.cpu().numpy() for t in a.step_device(torch.tensor([int(act)], device="cuda"))]
        rb = [t.cpu().numpy() for t in b.step_device(torch.tensor([[c, k // 64, k % 64]], device="cuda"))]
        for x, y in zip(ra, rb):
            assert np.array_equal(x, y)
    b.step_device(torch.tensor([[cfg.channels, 0, 0]], device="cuda"))
    with pytest.raises(ValueError):
        b.state.check_error()
    a.close(), b.close()


def test_premodel_on_gpu_feeds_env_reset():
    """BinaryNet (PyTorch-ROCm / MIOpen) as the env's pre_model_fn
    (env.py:109-120): GPU output vs the CPU module, then the reset state's PSNR
    vs the oracle on the same binarised mask."""
    from hbx.env import HologramVecEnv
    from hbx.premodel import premodel_fn, reference_premodel
    torch.manual_seed(0)
    m = reference_premodel(num_hologram=8, in_planes=1)
    tgt = torch.rand(1, 1, 64, 64)
    want = m(tgt)
    mg = m.cuda()
    got = premodel_fn(mg)(tgt.cuda())
    assert torch.allclose(got.cpu(), want, atol=1e-4)
    assert premodel_fn(mg, torch.bfloat16)(tgt.cuda()).shape == (1, 8, 64, 64)
    ocfg = O.mono_config(64)
    vec = HologramVecEnv(dev_cfg(ocfg), 1, lambda i: tgt[0].cuda(), pre_model_fn=premodel_fn(mg), obs_keys=("pre_model",))
    obs = vec.reset()
    pre = obs["pre_model"][0, 0].cpu().numpy()
    env = O.OracleEnv(ocfg)
    base = env.reset(pre, tgt[0].numpy())
    assert abs(float(vec.state.init_psnr[0].item()) - base) <= PSNR_TOL
    vec.close()


@pytest.mark.parametrize("mode", ["psf", "psf_host"])
@pytest.mark.parametrize("refresh", [0, 64])
def test_dbs_greedy_incremental_mode(golden_dir, refresh, mode):
    """Greedy DBS with candidates on the incremental-field path -- the
    device-resident walk (hbx_dbs_walk_psf) and the host-decided batches
    (hbx_eval_flips_psf / hbx_commit_flip_psf): the serial accept sequence of
    the 4096-flip oracle trace, with and without periodic exact refresh."""
    import hbx
    from hbx import dbs
    d = load(golden_dir, "dbs_trace_64.npz")
    plan = hbx.Plan(dev_cfg(small_rgb()), max_jobs=128)
    mask = hbx.pack_bits(torch.from_numpy(d["pre_model"]).cuda() >= 0.5)
    res = dbs.greedy(plan, mask, torch.from_numpy(d["target"]).cuda(), d["order"], mode=mode,
                     refresh_every=refresh)
    want_pos = np.nonzero(d["accepted"])[0]
    got = np.array(res.accepted_positions)
    assert len(got) == len(want_pos) and np.array_equal(got, want_pos)
    assert abs(res.final_psnr - float(d["final_psnr"])) <= PSNR_TOL
    assert np.array_equal(mask.cpu().numpy().view("<u8"), d["final_mask_bits"])


@pytest.mark.parametrize("refresh", [4096, 7])
def test_walk_repeated_positions_fused_split_host_oracle(monkeypatch, refresh):
    """Orders that revisit pixels: consecutive repeats, a period-3 cycle
    over three pixels and revisits one candidate apart, so a batch holds a candidate on
    the first accept's pixel (the fused step breaks there and re-evaluates it in the next
    launch) and pending commits sit on a candidate's pixel (the WalkPre sign toggle).
    K cycles through the fused depths 2, 3, 4 every chunk.  The fused walk, the split
    three-launch walk (HBX_WALK_SPLIT=1) and the host-decided batches accept exactly the
    same positions, and all of them the serial float64 oracle's wherever its change is
    resolved (|change| > 1e-7 dB)."""
    import hbx
    from hbx import dbs
    ocfg = O.OpticsConfig(64, 64, 3, 2, O.WL_RGB)
    pre, tgt = O.synthetic_inputs(ocfg, 33)
    cfg = dev_cfg(ocfg)
    n_pix = ocfg.channels * 64 * 64
    base = np.random.default_rng(9).integers(0, n_pix, 400)
    i = np.arange(600)
    order = np.concatenate([base[i // 3 + (i % 3 == 2)],           # b0 b0 b1 b1 b1 b2 ...
                            base[400 - 3:][i % 3],                   # a b c a b c ...
                            base[(i // 2) + (i % 2) * 2]])           # b0 b2 b1 b3 b2 b4 ...
    ks = [2, 3, 4]
    it = iter(range(10 ** 6))
    monkeypatch.setattr(dbs, "walk_k", lambda *a, **k: ks[next(it) % len(ks)])
    env = O.OracleEnv(ocfg)
    env.reset(pre, tgt)
    want, psnrs, _ = O.dbs_greedy(env, order)
    prev = np.maximum.accumulate(np.concatenate([[env.initial_psnr], psnrs]))[:-1]
    clear = np.abs(psnrs - prev) > 1e-7
    runs = {}
    for name in ("psf", "split", "psf_host"):
        if name == "split":
            monkeypatch.setenv("HBX_WALK_SPLIT", "1")
        plan = hbx.Plan(cfg, max_jobs=16)
        monkeypatch.delenv("HBX_WALK_SPLIT", raising=False)
        mask = hbx.pack_bits(torch.from_numpy(pre).cuda() >= 0.5)
        res = dbs.greedy(plan, mask, torch.from_numpy(tgt).cuda(), order,
                         mode="psf_host" if name == "psf_host" else "psf", refresh_every=refresh)
        plan.close()
        got = np.zeros(len(order), bool)
        got[res.accepted_positions] = True
        runs[name] = (got, mask.cpu().numpy())
        assert res.steps == len(order)
        assert np.array_equal(got[clear], want[clear]), (name, int(np.nonzero(got[clear] != want[clear])[0][0]))
    assert np.array_equal(runs["psf"][0], runs["split"][0]) and np.array_equal(runs["psf"][1], runs["split"][1])
    assert np.array_equal(runs["psf"][0], runs["psf_host"][0])
    assert 0 < want.sum() < len(order) and (~clear).sum() < 5


def test_dbs_walk_early_stop_and_prefix():
    """Device walk: DBS_ratio_0.5.py's early stop (stop_diff) against the serial
    oracle, and a max_candidates prefix ends exactly at the prefix."""
    import hbx
    from hbx import dbs
    ocfg = small_rgb()
    pre, tgt = O.synthetic_inputs(ocfg, 21)
    order = np.random.default_rng(3).permutation(ocfg.channels * 64 * 64)
    plan = hbx.Plan(dev_cfg(ocfg), max_jobs=8)
    env = O.OracleEnv(ocfg, accept_rule=1)
    env.reset(pre, tgt)
    acc, ps, final = O.dbs_greedy(env, order, stop_diff=0.05)
    mask = hbx.pack_bits(torch.from_numpy(pre).cuda() >= 0.5)
    res = dbs.greedy(plan, mask, torch.from_numpy(tgt).cuda(), order, stop_diff=0.05, mode="psf")
    assert res.stopped_early
    assert res.steps == len(acc)
    assert abs(res.final_psnr - final) <= PSNR_TOL
    mask = hbx.pack_bits(torch.from_numpy(pre).cuda() >= 0.5)
    res = dbs.greedy(plan, mask, torch.from_numpy(tgt).cuda(), order, mode="psf", max_candidates=777)
    assert res.steps == 777 and not res.stopped_early
    assert all(p < 777 for p in res.accepted_positions)


def test_dbs_walk_graph_replay_matches(golden_dir):
    """The walk's chunks captured into hipGraphs (one per speculation depth K)
    and replayed give the eager walk's accept sequence: the C-ABI enqueues
    capture-safe work (no allocation, copy or sync inside a launch)."""
    import hbx
    from hbx import dbs
    d = load(golden_dir, "dbs_trace_64.npz")
    plan = hbx.Plan(dev_cfg(small_rgb()), max_jobs=8)
    res = []
    for graphs in (False, True):
        mask = hbx.pack_bits(torch.from_numpy(d["pre_model"]).cuda() >= 0.5)
        res.append(dbs.greedy(plan, mask, torch.from_numpy(d["target"]).cuda(), d["order"], mode="psf",
                              refresh_every=64, graphs=graphs))
    assert res[0].accepted_positions == res[1].accepted_positions == np.nonzero(d["accepted"])[0].tolist()
    assert res[0].final_psnr == res[1].final_psnr


def test_dbs_greedy_many_equals_single_walks():
    """dbs.greedy_many (several images' walks side by side, one stream each)
    returns exactly what greedy(mode="psf") returns for each image alone,
    including a walk that halts for exact refreshes and one that stops early."""
    import hbx
    from hbx import dbs
    ocfg = small_rgb()
    cfg = dev_cfg(ocfg)
    n = ocfg.channels * 64 * 64
    ins = [O.synthetic_inputs(ocfg, 60 + i) for i in range(3)]
    orders = [np.random.default_rng(70 + i).permutation(n)[:3000] for i in range(3)]
    masks = [hbx.pack_bits(torch.from_numpy(p).cuda() >= 0.5) for p, _ in ins]
    tgts = [torch.from_numpy(t).cuda() for _, t in ins]
    single = []
    for i in range(3):
        plan = hbx.Plan(cfg, max_jobs=cfg.groups)
        m = masks[i].clone()
        single.append((dbs.greedy(plan, m, tgts[i], orders[i], mode="psf", refresh_every=256), m))
        plan.close()
    plans = [hbx.Plan(cfg, max_jobs=cfg.groups) for _ in range(3)]
    ms = [m.clone() for m in masks]
    many = dbs.greedy_many(plans, ms, tgts, orders, refresh_every=256)
    for (want, wm), got, gm in zip(single, many, ms):
        assert got.accepted_positions == want.accepted_positions
        assert got.final_psnr == want.final_psnr and got.steps == want.steps
        assert torch.equal(gm, wm)
    stop = dbs.greedy_many(plans[:2], [m.clone() for m in masks[:2]], tgts[:2], orders[:2], stop_diff=0.02)
    for i, r in enumerate(stop):
        w = dbs.greedy(plans[i], masks[i].clone(), tgts[i], orders[i], mode="psf", stop_diff=0.02)
        assert r.stopped_early == w.stopped_early and r.accepted_positions == w.accepted_positions
    for p in plans:
        p.close()


def test_dbs_dataset_single_rank_equals_single_walks(tmp_path):
    """dbs.greedy_dataset (the per-folder loop, images sharded over ranks; world 1 here)
    gives each image exactly its greedy(mode="psf") result, two images side by side."""
    import hbx
    from hbx import dbs
    ocfg = small_rgb()
    cfg = dev_cfg(ocfg)
    n = ocfg.channels * 64 * 64
    ins = [O.synthetic_inputs(ocfg, 80 + i) for i in range(3)]
    orders = [np.random.default_rng(90 + i).permutation(n)[:2000] for i in range(3)]

    def load(i):
        return hbx.pack_bits(torch.from_numpy(ins[i][0]).cuda() >= 0.5), torch.from_numpy(ins[i][1]).cuda()

    rows = dbs.greedy_dataset(3, load, lambda i: orders[i], lambda: hbx.Plan(cfg, max_jobs=cfg.groups),
                              per_gpu=2, save_dir=str(tmp_path))
    assert [r["image"] for r in rows] == [0, 1, 2] and all(r["rank"] == 0 for r in rows)
    for i, r in enumerate(rows):
        plan = hbx.Plan(cfg, max_jobs=cfg.groups)
        m, t = load(i)
        w = dbs.greedy(plan, m, t, orders[i], mode="psf")
        plan.close()
        assert r["accepted"] == len(w.accepted_positions) and r["final_psnr"] == w.final_psnr
        assert r["candidates"] == w.steps == 2000
        z = np.load(tmp_path / f"dbs_image{i}_accepted.npz")
        assert z["positions"].tolist() == w.accepted_positions


@pytest.mark.parametrize("field_kind", [0, 1])
def test_dbs_walk_matches_host_batches_1024(field_kind):
    """1024 x 24 RGB: the device-resident walk and the host-decided psf batches
    accept the same positions over a 3000-candidate prefix and end on the same
    mask; the final PSNR agrees with an exact re-propagation."""
    import hbx
    from hbx import dbs
    cfg = hbx.rgb_config(1024, field_kind=field_kind)
    g = torch.Generator(device="cuda").manual_seed(31)
    pre = torch.rand((24, 1024, 1024), generator=g, device="cuda")
    tgt = torch.rand((3, 1024, 1024), generator=g, device="cuda")
    order = np.random.default_rng(3).permutation(24 * 1024 * 1024)[:3000]
    plan = hbx.Plan(cfg, max_jobs=64)
    m1 = hbx.pack_bits(pre >= 0.5)
    m2 = m1.clone()
    r1 = dbs.greedy(plan, m1, tgt, order, mode="psf")
    r2 = dbs.greedy(plan, m2, tgt, order, mode="psf_host")
    assert r1.steps == r2.steps == 3000
    assert r1.accepted_positions == r2.accepted_positions
    assert torch.equal(m1, m2)
    _, _, ps = plan.propagate(m1[None], tgt[None], want_intensity=False)
    assert abs(float(ps[0]) - r1.final_psnr) <= PSNR_TOL


# ---------------------------------------------------------------------------
# N = 896: the 64-pixel crop of a 1024 mask (env_1024_24_128.py:144-149,
# DBS_1024_24-128.py:210-216) on the generic 28 x 32 mixed-radix path
# ---------------------------------------------------------------------------
def _crop_inputs(seed):
    import hbx
    full = O.rgb_config(1024)
    pre, tgt = O.synthetic_inputs(full, seed)
    ocfg = O.rgb_config(896)
    pre_c, tgt_c = O.crop(pre, 64), O.crop(tgt, 64)
    bits_full = to_dev_bits(O.pack_mask((pre >= 0.5).astype(np.uint8)))
    bits = hbx.crop_bits(bits_full, 64)
    return ocfg, pre_c, tgt_c, bits


@pytest.mark.parametrize("field_kind", [O.FIELD_AMPLITUDE, O.FIELD_PHASE])
def test_crop_896_lane_class_edges_vs_oracle(field_kind):
    """N = 896 (the fused mixed-radix passes, hbx_passes896.hip) against the float64
    oracle at the row / column edges of every slot lane class (x, y = 27 / 28 / 447 /
    448 / 895 ...): the plane field of hbx_simulate (2e-6 * max), the propagated
    statistics, and flips there (1e-4 dB).  Round 2 checked the fused path against a
    composed one; that path is gone and the oracle pins 896 directly."""
    import hbx
    _, pre, tgt, bits = _crop_inputs(12)
    ocfg = O.rgb_config(896, field_kind=field_kind)
    mask = (pre >= 0.5).astype(np.uint8)
    plan = hbx.Plan(dev_cfg(ocfg), max_jobs=12)
    t = torch.from_numpy(tgt).cuda()
    fld, _ = plan.simulate(bits[None])
    want_f = O.propagate(O.mask_to_field(mask[:2], field_kind), ocfg.transfer(0))
    got_f = fld[0, :2].cpu().numpy()
    assert np.max(np.abs(got_f - want_f)) <= 2e-6 * np.max(np.abs(want_f))
    env = O.OracleEnv(ocfg)
    base = env.reset(pre, tgt)
    _, st, p0 = plan.propagate(bits[None], t[None])
    assert abs(float(p0[0]) - base) <= PSNR_TOL
    n = 896 * 896
    fl = np.array([c * n + r * 896 + x for c in (0, 7, 16, 23) for (r, x) in
                   ((0, 0), (895, 895), (447, 27), (448, 28), (300, 448), (1, 895 - 31))], np.int64)
    want = np.array([env.evaluate_flip(int(a))[0] for a in fl])
    got, _ = plan.eval_flips(bits, t, st[0].contiguous(), torch.from_numpy(fl).cuda())
    assert np.max(np.abs(got.cpu().numpy() - want)) <= PSNR_TOL
    plan.close()


def test_crop_896_propagate_vs_oracle():
    import hbx
    ocfg, pre, tgt, bits = _crop_inputs(7)
    mask = (pre >= 0.5).astype(np.uint8)
    assert np.array_equal(bits.cpu().numpy().view("<u8"), O.pack_mask(mask))
    prop = O.Propagator(ocfg)
    ref_i = prop.all_intensity(mask)
    ref_st = np.stack([O.chan_stats(ref_i[g], tgt[g]) for g in range(3)])
    plan = hbx.Plan(dev_cfg(ocfg), max_jobs=6)
    inten, stats, psnr = plan.propagate(bits[None], torch.from_numpy(tgt).cuda()[None])
    torch.cuda.synchronize()
    assert np.allclose(stats[0].cpu().numpy(), ref_st, rtol=STATS_RTOL)
    assert abs(float(psnr[0]) - prop.psnr(ref_st)) <= PSNR_TOL
    got = inten[0].cpu().numpy()
    assert np.max(np.abs(got - ref_i)) <= 2e-5 * np.max(ref_i)
    plan.close()


@pytest.mark.parametrize("field_kind", [O.FIELD_AMPLITUDE, O.FIELD_PHASE])
def test_crop_896_eval_flips_and_map_vs_oracle(field_kind):
    import hbx
    _, pre, tgt, bits = _crop_inputs(8)
    ocfg = O.rgb_config(896, field_kind=field_kind)
    env = O.OracleEnv(ocfg)
    base = env.reset(pre, tgt)
    n = 896 * 896
    flips = np.array([0, n - 1, 895, n - 896, 5 * n + 448 * 896 + 447, 13 * n + 77, 24 * n - 1], np.int64)
    want = np.array([env.evaluate_flip(int(a))[0] for a in flips])
    plan = hbx.Plan(dev_cfg(ocfg), max_jobs=8)
    t = torch.from_numpy(tgt).cuda()
    _, st, p0 = plan.propagate(bits[None], t[None])
    assert abs(float(p0[0]) - base) <= PSNR_TOL
    got, _ = plan.eval_flips(bits, t, st[0].contiguous(), torch.from_numpy(flips).cuda())
    assert np.max(np.abs(got.cpu().numpy() - want)) <= PSNR_TOL
    dmap, b = plan.flip_map(bits, t)
    assert abs(float(b.item()) - base) <= PSNR_TOL
    assert bool(torch.isfinite(dmap).all())
    d = dmap.reshape(-1)[torch.from_numpy(flips).cuda()].double().cpu().numpy()
    assert np.max(np.abs(d - (want - base))) <= MAP_TOL
    plan.close()


def test_crop_896_psf_matches_fft():
    """Incremental-field mode at 896 (folded h offsets, non-power-of-2 N)
    agrees with the FFT mode step by step."""
    import hbx
    from hbx.env import HologramVecEnv
    cfg = hbx.rgb_config(896)
    B = 2
    gens = [torch.Generator(device="cuda").manual_seed(70 + i) for i in range(B)]
    pres = [torch.rand((24, 896, 896), generator=g, device="cuda") for g in gens]
    tgts = [torch.rand((3, 896, 896), generator=g, device="cuda") for g in gens]
    kw = dict(pre_model_source=lambda i: pres[i], obs_keys=(), auto_reset=False)
    fft = HologramVecEnv(cfg, B, lambda i: tgts[i], **kw)
    psf = HologramVecEnv(cfg, B, lambda i: tgts[i], mode="psf", refresh_every=8, **kw)
    fft.reset()
    psf.reset()
    assert torch.allclose(fft.state.init_psnr, psf.state.init_psnr, atol=1e-9)
    acts = torch.randint(0, 24 * 896 * 896, (24, B), generator=gens[0], device="cuda")
    for k in range(24):
        _, p1, a1, _, _ = fft.step_device(acts[k])
        _, p2, a2, _, _ = psf.step_device(acts[k])
        assert torch.max(torch.abs(p1 - p2)).item() <= PSNR_TOL
    assert torch.equal(fft.state.mask, psf.state.mask)
    fft.close()
    psf.close()


def test_crop_896_dbs_greedy_vs_oracle():
    """DBS on the crop (DBS_1024_24-128.py:210-300): FFT-mode and
    incremental-mode greedy runs against the serial f64 oracle."""
    import hbx
    from hbx import dbs
    ocfg, pre, tgt, bits = _crop_inputs(9)
    env = O.OracleEnv(ocfg)
    env.reset(pre, tgt)
    order = np.random.default_rng(3).integers(0, 24 * 896 * 896, 40)
    acc, psnrs, final = O.dbs_greedy(env, order)
    prev = np.maximum.accumulate(np.concatenate([[env.initial_psnr], psnrs]))[:-1]
    clear = np.abs(psnrs - prev) > 1e-5      # fp32 fields cannot order ties below this
    plan = hbx.Plan(dev_cfg(ocfg), max_jobs=16)
    t = torch.from_numpy(tgt).cuda()
    for mode in ("fft", "psf"):
        m = bits.clone()
        res = dbs.greedy(plan, m, t, order, mode=mode)
        got = np.zeros(len(order), bool)
        got[res.accepted_positions] = True
        assert np.array_equal(got[clear], acc[clear]), mode
        assert abs(res.final_psnr - final) <= PSNR_TOL, mode
        if np.array_equal(got, acc):
            assert np.array_equal(m.cpu().numpy().view("<u8"), O.pack_mask(env.state)), mode
    plan.close()


def test_empty_batches_and_chunked_invalid_flips():
    """Edge cases at the C-ABI: zero-sized batches are no-ops (torch hands
    null data pointers for empty tensors), a flip batch larger than max_jobs
    runs in max_jobs chunks, and out-of-range flip indices (negative, or
    >= CH*N^2, which env.py:157-161's decode would carry into a non-existent
    plane) come back as NaN without disturbing their neighbours."""
    import hbx
    ocfg = small_rgb()
    pre, tgt = O.synthetic_inputs(ocfg, 5)
    plan = hbx.Plan(dev_cfg(ocfg), max_jobs=3)
    bits = to_dev_bits(O.pack_mask((pre >= 0.5).astype(np.uint8)))
    t = torch.from_numpy(tgt).cuda()

    inten, st0, ps0 = plan.propagate(bits[None][:0], t[None][:0])
    assert inten.shape[0] == 0 and st0.shape[0] == 0 and ps0.shape[0] == 0
    assert plan.psnr(st0).shape == (0,)

    _, st, ps = plan.propagate(bits[None], t[None])
    got0, gs0 = plan.eval_flips(bits, t, st[0].contiguous(), torch.empty((0,), dtype=torch.int64, device="cuda"))
    assert got0.shape == (0,) and gs0.shape == (0, 3)

    env = O.OracleEnv(ocfg)
    env.reset(pre, tgt)
    assert abs(float(ps[0]) - env.initial_psnr) <= PSNR_TOL
    total = ocfg.channels * 64 * 64
    flips = np.array([0, -1, total - 1, total, 4095, 4096, 2 * 4096 + 65], np.int64)   # K = 7 > max_jobs
    got, _ = plan.eval_flips(bits, t, st[0].contiguous(), torch.from_numpy(flips).cuda())
    got = got.cpu().numpy()
    for a, g in zip(flips, got):
        if 0 <= a < total:
            assert abs(g - env.evaluate_flip(int(a))[0]) <= PSNR_TOL, int(a)
        else:
            assert np.isnan(g), int(a)
    # the base mask is untouched by evaluation
    assert np.array_equal(bits.cpu().numpy(), to_dev_bits(O.pack_mask((pre >= 0.5).astype(np.uint8))).cpu().numpy())


@pytest.mark.timeout(240)
def test_sharded_envs_world2_match_single_process():
    """SURVEY 8e on the device: 4 envs split 2 + 2 over a world of 2 (gloo,
    both ranks on cuda:0 -- the one-GPU stand-in for one rank per GPU over
    RCCL), each rank stepping its own envs and gathering every step's metrics
    to rank 0, reproduce a single process stepping all 4 envs bit for bit."""
    import socket
    import torch.multiprocessing as mp
    from tests import _shard_worker as W

    want = np.stack([r.cpu().numpy() for r in W.run_envs(0, W.TOTAL)])
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=W.worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    got = next(r for r in res if r is not None)
    assert got.shape == want.shape == (W.STEPS, W.TOTAL, 5)
    assert np.array_equal(got, want)
    assert 0 < want[:, :, 2].sum() < want[:, :, 2].size   # both accepts and rollbacks occurred
