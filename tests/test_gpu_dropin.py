"""The drop-in single env (hbx.env.BinaryHologramEnv -- the object an unchanged
train-PPO.py binds through DummyVecEnv(n_envs=1), and whose reset() the DBS
drivers call) at the sizes its callers use, against the float64 oracle.

  256x256x8 mono (env.py, train-PPO.py:40,275):  >= 200 steps vs O.OracleEnv, every
      observation compared at every step, the rollback-at-max_steps quirk
      (env.py:191-196: a rolled-back step at max_steps neither terminates nor
      truncates; the next accepted one does, with the -595.24 bonus), the success
      termination path (T_steps sustained steps past T_PSNR_DIFF, the -595.2 bonus),
      one blocking wait per step (host_syncs) and no hidden torch sync
      (torch.cuda.set_sync_debug_mode("error")), host counters == device counters.
  1024x1024x24 RGB (env_1024_24.py / DBS_1024_24.py:213-224): >= 20 steps vs
      O.LinearGreedy following the GPU's decisions (as tests/test_gpu_batch128.py).

Tolerances (north_star "PSNR within 1e-4 of numpy"):
  PSNR after each step          |gpu - oracle| <= 1e-4 dB
  PSNR change (decision)        decisions equal wherever |change| > CLEAR_DB (the f32
                                resolution of a change: 256 mono 1e-6 dB, 1024x24 4e-9 dB)
  reward                        |gpu - oracle| <= 800 * 1e-4
  recon_image                   max |gpu - oracle| <= 2e-5 * max(oracle)
  state / state_record / pre_model / target, counters, flags: exact
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import hbx_oracle as O  # noqa: E402

PSNR_TOL = 1e-4
CLEAR_256 = 1e-6
CLEAR_1024 = 4e-9      # ENV_FFT_TOL_DB, tests/test_gpu_dbs_headline.py
RECON_RTOL = 2e-5


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


def _setup(ocfg, n_images=2, seed=70):
    ins = [O.synthetic_inputs(ocfg, seed + 2 * i) for i in range(n_images)]
    pres = {float(t[0, 0, 0]): p for p, t in ins}     # target -> pre-model output (BinaryNet stand-in)

    def target_function(target):
        return torch.from_numpy(pres[float(target.reshape(-1)[0])][None]).to(target.device)

    return _Loader([t for _, t in ins]), target_function, ins


def _dev_cfg(ocfg):
    import hbx
    return hbx.OpticsConfig(ocfg.height, ocfg.width, ocfg.groups, ocfg.planes, tuple(ocfg.wavelengths))


def _check_obs(obs, oe, pre, tgt, recon_want):
    assert np.array_equal(obs["state"][0], oe.state)
    assert np.array_equal(obs["state_record"][0], oe.state_record)
    assert np.array_equal(obs["pre_model"][0], pre) and np.array_equal(obs["target_image"][0], tgt)
    assert obs["recon_image"].shape == (1,) + recon_want.shape and obs["recon_image"].dtype == np.float32
    assert np.max(np.abs(obs["recon_image"][0] - recon_want)) <= RECON_RTOL * np.max(recon_want)


def _pick(oe, rng, sign, n_pix):
    """An action whose change against the oracle's current state is clearly `sign`."""
    for _ in range(64):
        a = int(rng.integers(0, n_pix))
        p, _, _, _ = oe.evaluate_flip(a)
        if sign * (p - oe.previous_psnr) > 10 * CLEAR_256:
            return a
    raise AssertionError("no clear candidate found")


def _step_both(env, oe, a, clear_db):
    """One step of both envs; the oracle follows the GPU's decision at a sub-resolution tie."""
    obs, reward, term, trunc, info = env.step(a)
    gpu_acc = env.flip_count == oe.flip_count + 1
    want = oe.step(a, accept=gpu_acc)
    ch = oe.last_change
    if abs(ch) > clear_db:
        assert gpu_acc == (ch >= 0), (a, ch)                    # env.py:191: roll back iff change < 0
    assert isinstance(reward, float) and isinstance(term, bool) and isinstance(trunc, bool) and info == {}
    assert abs(reward - want.reward) <= O.RW * PSNR_TOL
    assert (term, trunc) == (want.terminated, want.truncated)
    return obs, reward, term, trunc, want


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", [None, "fft"])   # None: the default (plane-cached FFT mode at 256 / 1024)
def test_dropin_env_256_mono_vs_oracle_with_max_steps_rollback(mode):
    from hbx.env import BinaryHologramEnv
    ocfg = O.mono_config(256)
    n_pix = ocfg.channels * 256 * 256
    loader, tf, ins = _setup(ocfg)
    max_steps = 200
    kw = {} if mode is None else {"mode": mode}
    env = BinaryHologramEnv(tf, loader, max_steps=max_steps, config=_dev_cfg(ocfg), verbose=False, **kw)
    assert env._vec.mode == (mode or "planes")
    obs, info = env.reset()
    pre, tgt = ins[0]
    assert info["state"] is obs["state"] is env.state                          # env.py:152,177 alias
    oe = O.OracleEnv(ocfg, max_steps=max_steps)
    oe.reset(pre, tgt)
    assert abs(env.initial_psnr - oe.initial_psnr) <= PSNR_TOL
    _check_obs(obs, oe, pre, tgt, oe.intensity)
    rng = np.random.default_rng(11)
    clear = accepted = 0
    syncs0 = env.host_syncs
    torch.cuda.set_sync_debug_mode("error")        # a hidden torch sync in step() raises
    try:
        for k in range(max_steps - 1):
            obs, reward, term, trunc, want = _step_both(env, oe, int(rng.integers(0, n_pix)), CLEAR_256)
            clear += abs(oe.last_change) > CLEAR_256
            accepted += want.accepted
            assert not term and not trunc
            assert obs["state"] is env.state and obs["state_record"] is env.state_record
            _check_obs(obs, oe, pre, tgt, oe.last_group_intensity[1][None])
            assert env.previous_psnr == pytest.approx(oe.previous_psnr, abs=PSNR_TOL)
            assert (env.steps, env.flip_count, env.psnr_sustained_steps) == \
                (oe.steps, oe.flip_count, oe.psnr_sustained_steps)
        # step max_steps: a clearly negative change is rolled back and does NOT end the episode
        a = _pick(oe, rng, -1, n_pix)
        obs, reward, term, trunc, want = _step_both(env, oe, a, CLEAR_256)
        assert env.steps == max_steps and not want.accepted and reward < 0 and (term, trunc) == (False, False)
        _check_obs(obs, oe, pre, tgt, oe.last_group_intensity[1][None])
        # step max_steps + 1: accepted -> terminated and truncated, with the -595.24 bonus
        a = _pick(oe, rng, +1, n_pix)
        obs, reward, term, trunc, want = _step_both(env, oe, a, CLEAR_256)
        assert want.accepted and term and trunc
        ratio = oe.flip_count / oe.steps
        assert abs(reward - (O.RW * oe.last_change + O.max_steps_cubic(ratio))) <= O.RW * PSNR_TOL
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert env.host_syncs - syncs0 == max_steps + 1            # one blocking wait per step
    assert clear >= 150 and 0 < accepted < max_steps
    dc = env.device_counters()
    assert (dc["steps"], dc["flip_count"], dc["psnr_sustained_steps"]) == \
        (env.steps, env.flip_count, env.psnr_sustained_steps)
    assert dc["previous_psnr"] == env.previous_psnr and dc["max_psnr_diff"] == env.max_psnr_diff
    # the device mask is the host mirror
    import hbx
    got = hbx.unpack_bits(env._vec.state.mask[0], 256).cpu().numpy()
    assert np.array_equal(got, env.state[0])
    # the next episode: the loader's second image, fresh mirrors
    obs, info = env.reset()
    pre2, tgt2 = ins[1]
    assert env.episode_num_count == 2 and env.steps == 0 and not env.state_record.any()
    assert np.array_equal(obs["state"][0], (pre2 >= 0.5).astype(np.int8))
    assert np.array_equal(obs["target_image"][0], tgt2)
    env.close()


@pytest.mark.timeout(300)
def test_dropin_env_256_success_termination():
    """env.py:216-235,257: T_steps accepted steps past T_PSNR_DIFF end the episode with the
    success cubic.  T_PSNR_DIFF is placed between two oracle PSNR gains of a dry run (at a
    clear distance from every gain the run reaches), so both envs cross it on the same step."""
    from hbx.env import BinaryHologramEnv
    ocfg = O.mono_config(256)
    n_pix = ocfg.channels * 256 * 256
    loader, tf, ins = _setup(ocfg, 1, seed=90)
    pre, tgt = ins[0]
    acts = np.random.default_rng(12).integers(0, n_pix, 160)
    dry = O.OracleEnv(ocfg, T_PSNR_DIFF=1e9)
    dry.reset(pre, tgt)
    gains = []
    for a in acts:
        r = dry.step(int(a))
        if r.accepted:
            gains.append(r.psnr - dry.initial_psnr)
    g = np.sort(np.array(gains[40:]))
    gaps = np.diff(g)
    j = int(np.argmax(gaps[:len(gaps) // 2]))              # a wide gap in the lower half
    thr = float(g[j] + gaps[j] / 2)
    assert gaps[j] > 20 * CLEAR_256
    env = BinaryHologramEnv(tf, loader, T_PSNR_DIFF=thr, T_steps=2, config=_dev_cfg(ocfg), verbose=False)
    env.reset()
    oe = O.OracleEnv(ocfg, T_PSNR_DIFF=thr, T_steps=2)
    oe.reset(pre, tgt)
    ended = False
    for a in acts:
        obs, reward, term, trunc, want = _step_both(env, oe, int(a), CLEAR_256)
        assert env.psnr_sustained_steps == oe.psnr_sustained_steps
        if term:
            ended = True
            assert not trunc and oe.psnr_sustained_steps == 2
            ratio = oe.flip_count / oe.steps
            assert abs(reward - (O.RW * oe.last_change + O.success_cubic(ratio))) <= O.RW * PSNR_TOL
            break
    assert ended
    dc = env.device_counters()
    assert (dc["steps"], dc["flip_count"], dc["psnr_sustained_steps"]) == \
        (env.steps, env.flip_count, env.psnr_sustained_steps)
    env.close()


@pytest.mark.timeout(300)
def test_dropin_env_1024x24_rgb_vs_linear_oracle():
    """env_1024_24.py's env with DBS_1024_24.py's per-flip semantics: 24 steps of
    the drop-in env against O.LinearGreedy (float64 by linearity) following the GPU's
    decisions; every observation compared."""
    import hbx
    from hbx.env import BinaryHologramEnv
    ocfg = O.rgb_config(1024)
    N, CH, G = 1024, ocfg.channels, ocfg.groups
    loader, tf, ins = _setup(ocfg, 1, seed=80)
    env = BinaryHologramEnv(tf, loader, config=hbx.rgb_config(N), verbose=False)
    obs, _ = env.reset()
    pre, tgt = ins[0]
    lg = O.LinearGreedy(ocfg, pre, tgt)
    assert abs(env.initial_psnr - lg.initial_psnr) <= PSNR_TOL
    assert obs["state"].shape == (1, CH, N, N) and obs["recon_image"].shape == (1, G, N, N)
    assert np.max(np.abs(obs["recon_image"][0] - lg.intensity)) <= RECON_RTOL * np.max(lg.intensity)
    record = np.zeros((CH, N, N), np.int8)
    rng = np.random.default_rng(13)
    clear = 0
    syncs0 = env.host_syncs
    for k in range(24):
        a = int(rng.integers(0, CH * N * N))
        ev = lg.evaluate(a)
        change = ev[0] - lg.previous_psnr
        fc = env.flip_count
        obs, reward, term, trunc, info = env.step(a)
        accepted = env.flip_count == fc + 1
        assert abs(reward - O.RW * change) <= O.RW * PSNR_TOL and not term and not trunc
        if abs(change) > CLEAR_1024:
            clear += 1
            assert accepted == (change >= 0), (k, change)
        ch, r, col = (int(v) for v in O.decode_action(a, N, N))
        record[ch, r, col] += 1
        g = ch // ocfg.planes
        want_recon = lg.intensity.copy()
        want_recon[g] = lg.intensity[g] + ev[5]                   # the stepped (pre-rollback) group
        assert np.max(np.abs(obs["recon_image"][0] - want_recon)) <= RECON_RTOL * np.max(want_recon)
        if accepted:
            lg.commit(a, ev)
        assert np.array_equal(obs["state"][0], lg.state) and np.array_equal(obs["state_record"][0], record)
        assert obs["pre_model"] is env.observation and obs["target_image"] is env.target_image_np
        assert env.previous_psnr == pytest.approx(lg.previous_psnr, abs=PSNR_TOL)
    assert env.host_syncs - syncs0 == 24 and clear >= 12
    got = hbx.unpack_bits(env._vec.state.mask[0], N).cpu().numpy()
    assert np.array_equal(got, env.state[0])
    dc = env.device_counters()
    assert (dc["steps"], dc["flip_count"]) == (env.steps, env.flip_count)
    env.close()
