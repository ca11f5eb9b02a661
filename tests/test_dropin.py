"""The drop-in env classes (hbx.env.BinaryHologramEnv / Group / MD) under the
reference's own contracts, and a builder-written driver with DBS_1024_24.py's
contract (not its text) running against them through the torchOptics shim.

Reference contracts checked:
  env.py:42-52      observation_space Dict / Discrete action_space
  env.py:135-140    reset obs: state / state_record / pre_model (1, CH, N, N),
                    recon_image / target_image (1, G, N, N); info {"state": ...}
  env.py:154-259    step -> (obs, reward float, terminated bool, truncated bool, {})
  env_md.py:54,160  MultiDiscrete([CH, N, N]) actions
  DBS_1024_24.py:221-422  the driver reads obs["state"].shape[1], slices colour
                    groups, propagates them with tt.simulate, caches the group
                    means and runs the greedy loop on current_state[0, c, r, col]
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import hbx_oracle as O  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm GPU")
    import hbx
    hbx.load_library()
    yield


class _Loader:
    """A DataLoader(batch_size=1) stand-in: (target [1, G, N, N], [path]) items."""

    def __init__(self, targets):
        self.targets = targets

    def __iter__(self):
        for i, t in enumerate(self.targets):
            yield torch.from_numpy(t[None]), [f"/data/valid/{801 + i:04d}.png"]


def _setup(ocfg, n_images=2, seed=40):
    ins = [O.synthetic_inputs(ocfg, seed + 2 * i) for i in range(n_images)]
    pres = {float(t[0, 0, 0]): p for p, t in ins}     # target -> pre-model output (BinaryNet stand-in)

    def target_function(target):
        key = float(target.reshape(-1)[0])
        return torch.from_numpy(pres[key][None]).to(target.device)

    return _Loader([t for _, t in ins]), target_function, ins


def _dev_cfg(ocfg):
    import hbx
    return hbx.OpticsConfig(ocfg.height, ocfg.width, ocfg.groups, ocfg.planes, tuple(ocfg.wavelengths))


@pytest.mark.parametrize("rgb", [False, True])
def test_binary_hologram_env_contract_and_trace(rgb, capsys):
    from hbx.env import BinaryHologramEnv
    ocfg = O.OpticsConfig(64, 64, 3, 8, O.WL_RGB) if rgb else O.mono_config(64)
    loader, tf, ins = _setup(ocfg)
    env = BinaryHologramEnv(tf, loader, max_steps=30, T_PSNR_DIFF=0.05, config=_dev_cfg(ocfg), verbose=True)
    obs, info = env.reset()
    CH, G, N = ocfg.channels, ocfg.groups, 64
    shapes = {"state": (1, CH, N, N), "state_record": (1, CH, N, N), "pre_model": (1, CH, N, N),
              "recon_image": (1, G, N, N), "target_image": (1, G, N, N)}
    assert {k: v.shape for k, v in obs.items()} == shapes
    assert obs["state"].dtype == np.int8 and obs["pre_model"].dtype == np.float32
    assert env.observation_space.contains(obs)
    assert np.array_equal(info["state"], obs["state"])
    pre, tgt = ins[0]
    assert np.array_equal(obs["state"][0], (pre >= 0.5).astype(np.int8))       # env.py:120
    assert np.allclose(obs["target_image"][0], tgt)
    oe = O.OracleEnv(ocfg, max_steps=30, T_PSNR_DIFF=0.05)
    oe.reset(pre, tgt)
    assert abs(env.initial_psnr - oe.initial_psnr) <= 1e-4
    rng = np.random.default_rng(5)
    for _ in range(30):
        a = int(rng.integers(0, env.action_space.n))
        obs, reward, term, trunc, info = env.step(a)
        want = oe.step(a)
        assert isinstance(reward, float) and isinstance(term, bool) and isinstance(trunc, bool) and info == {}
        assert env.observation_space.contains(obs)
        assert abs(reward - want.reward) <= 800 * 2e-4
        assert (term, trunc) == (want.terminated, want.truncated)
        assert np.array_equal(obs["state"][0], oe.state)                        # rollback applied
        assert env.previous_psnr == pytest.approx(oe.previous_psnr, abs=1e-4)
        if term or trunc:
            break
    out = capsys.readouterr().out
    # the DataLoader yields a batch of paths, printed as the list (env.py:104 formats current_file as is)
    assert "[Episode Start] Currently using dataset file: ['/data/valid/0801.png'], Episode count: 1" in out
    assert "PSNR After:" in out and "| Flip Count:" in out                      # env.py:206-212 blocks
    assert "Initial PSNR:" in out and "Initial MSE:" in out
    env.close()


def test_debug_timing_lines_parse(capsys):
    """debug_env.py's per-phase timing lines, in the format log_py/debug_log.py:37-38 parses."""
    import re
    from hbx.env import BinaryHologramEnv
    ocfg = O.mono_config(64)
    loader, tf, _ = _setup(ocfg, 1)
    env = BinaryHologramEnv(tf, loader, config=_dev_cfg(ocfg), debug_timing=True)
    env.reset()
    for a in (3, 4000, 70000 % (8 * 4096)):
        env.step(a)
    out = capsys.readouterr().out
    rx = re.compile(r"Step:\s*(\d+)\s*\|\s*Time\s*(.+?)\s*:\s*([\d\.]+)\s*seconds")
    phases = {m.group(2) for m in rx.finditer(out)}
    assert {"action", "simulate", "obs", "reward", "k_rowfwd", "k_col", "k_rowinv"} <= phases
    assert {int(m.group(1)) for m in rx.finditer(out)} == {1, 2, 3}
    env.close()


def test_group_and_md_contracts():
    from hbx.env import BinaryHologramEnvGroup, BinaryHologramEnvMD
    ocfg = O.mono_config(64)
    loader, tf, ins = _setup(ocfg)
    g = BinaryHologramEnvGroup(tf, loader, config=_dev_cfg(ocfg), importance_samples=256)
    obs, info = g.reset()
    assert g.observation_space.contains(obs) and obs["state"].shape == (1, 8, 64, 64)
    assert g.psnr_change_list.shape == (256,) and g.importance_ranks.shape == (256,)
    obs, r, term, trunc, info = g.step(17)
    assert g.observation_space.contains(obs) and isinstance(r, float)
    g.close()
    loader, tf, ins = _setup(ocfg)
    md = BinaryHologramEnvMD(tf, loader, config=_dev_cfg(ocfg), max_steps=10)
    obs, _ = md.reset()
    assert list(md.action_space.nvec) == [8, 64, 64]
    oe = O.OracleEnv(ocfg, max_steps=10)
    oe.reset(*ins[0])
    rng = np.random.default_rng(9)
    for _ in range(10):
        c, r, col = int(rng.integers(8)), int(rng.integers(64)), int(rng.integers(64))
        obs, rew, term, trunc, _ = md.step((c, r, col))                       # env_md.py:159
        want = oe.step(int(O.encode_action(c, r, col, 64, 64)))
        assert md.observation_space.contains(obs)
        assert abs(rew - want.reward) <= 800 * 2e-4 and (term, trunc) == (want.terminated, want.truncated)
    with pytest.raises(ValueError):
        md.step((8, 0, 0))
    md.close()


def test_shim_greedy_contract_rgb():
    """What a DBS-style caller of the drop-in env relies on (the per-flip loop of
    DBS_1024_24.py:313-422), written against the contract rather than the script:
    obs["state"] is (1, CH, N, N) with CH = 3 colour groups x P planes in channel
    order; tt.simulate of one group's slice at that group's wavelength, |.|^2 and the
    plane mean give the group's reconstruction; tt.relativeLoss over the three
    group means reproduces the env's initial PSNR; and a strict-improvement walk over
    single flips that re-simulates only the touched group (the other two means
    cached) makes the float64 oracle's decisions, except at a candidate whose PSNR
    change is below the f32 resolution of a full-image PSNR (1e-6 dB), after which
    the comparison stops."""
    import torchOptics.metrics as tm
    import torchOptics.optics as tt
    from hbx.env import BinaryHologramEnv
    ocfg = O.OpticsConfig(64, 64, 3, 8, O.WL_RGB)
    loader, tf, ins = _setup(ocfg, 1, seed=60)
    env = BinaryHologramEnv(tf, loader, config=_dev_cfg(ocfg))
    obs, _ = env.reset()
    state = np.array(obs["state"], copy=True)
    n_ch, side = state.shape[1], state.shape[2]
    assert state.shape == (1, 24, 64, 64) and state.dtype == np.int8
    per = n_ch // ocfg.groups
    target = torch.tensor(obs["target_image"], dtype=torch.float32).cuda()
    dx = (ocfg.dx, ocfg.dy)

    def group_mean(g):
        field = tt.simulate(tt.Tensor(state[:, g * per:(g + 1) * per], meta={"wl": ocfg.wavelengths[g], "dx": dx}),
                            ocfg.z)
        return torch.mean(field.abs() ** 2, dim=1, keepdim=True)

    def psnr_of(means):
        rgb = tt.Tensor(torch.cat(means, dim=1), meta={"wl": tuple(ocfg.wavelengths), "dx": dx})
        return float(tt.relativeLoss(rgb, target, tm.get_PSNR))

    means = [group_mean(g) for g in range(ocfg.groups)]
    best = psnr_of(means)
    assert best == pytest.approx(env.initial_psnr, abs=1e-5)
    _, names = next(iter(env.trainloader))
    assert names[0].endswith("0801.png")

    order = np.random.default_rng(3).permutation(n_ch * side * side)[:400]
    decisions = []
    for a in order:
        ch, pix = divmod(int(a), side * side)
        r, col = divmod(pix, side)
        state[0, ch, r, col] ^= 1
        g = ch // per
        trial = means[:g] + [group_mean(g)] + means[g + 1:]
        p = psnr_of(trial)
        keep = p > best                                   # strict improvement
        if keep:
            means, best = trial, p
        else:
            state[0, ch, r, col] ^= 1                     # roll the flip back
        decisions.append(keep)

    pre, tgt = ins[0]
    lg = O.LinearGreedy(ocfg, pre, tgt)
    want, _, delta = lg.run(order)
    got = np.array(decisions)
    diff = np.nonzero(got != want)[0]
    upto = len(want) if len(diff) == 0 else int(diff[0])
    if len(diff):
        assert abs(delta[upto]) <= 1e-6, (upto, delta[upto])
    assert upto >= 200 and int(got.sum()) > 50
    if len(diff) == 0:
        assert np.array_equal(state[0], lg.state)
        assert best == pytest.approx(lg.previous_psnr, abs=1e-5)
    env.close()


def test_dbs_rgb_artifacts(tmp_path, capsys):
    """DBS_1024_24.py:280-286 / :444-451: the reconstructed RGB saved before and after the
    greedy loop, under the reference's file names, equal to the oracle's group means."""
    import hbx
    from hbx import dbs
    ocfg = O.OpticsConfig(64, 64, 3, 2, O.WL_RGB)
    pre, tgt = O.synthetic_inputs(ocfg, 11)
    cfg = hbx.OpticsConfig(64, 64, 3, 2, O.WL_RGB)
    plan = hbx.Plan(cfg, max_jobs=16)
    mask = hbx.pack_bits(torch.from_numpy(pre).cuda() >= 0.5)
    target = torch.from_numpy(tgt).cuda()
    before, after = dbs.rgb_artifact_paths("0801", str(tmp_path / "DBS"))
    assert before.endswith("DBS/episode_0801png_rgb_before.npy") and after.endswith("DBS/episode_0801_rgb_after.npy")
    m0 = (pre >= 0.5).astype(np.float32)
    dbs.save_rgb(plan, mask, target, before)
    order = np.random.default_rng(5).permutation(ocfg.channels * 64 * 64)[:300]
    res = dbs.greedy(plan, mask, target, order, mode="psf")
    dbs.save_rgb(plan, mask, target, after)
    out = capsys.readouterr().out
    assert f"RGB data saved to {before}" in out and f"RGB data saved to {after}" in out
    prop = O.Propagator(ocfg)
    m1 = O.unpack_mask(mask.cpu().numpy().view("<u8"), 64).astype(np.float32)
    assert int(np.sum(m1 != m0)) == len(res.accepted_positions)
    for path, m in ((before, m0), (after, m1)):
        got = np.load(path)
        want = prop.all_intensity(m)[None]
        assert got.shape == (1, 3, 64, 64) and got.dtype == np.float32
        assert np.max(np.abs(got - want)) <= 2e-5 * np.max(want)
    plan.close()
