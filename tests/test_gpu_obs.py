"""Zero-copy observations (ABI v8, env.py:135-140,176-181).

The reference hands out env.state itself as obs["state"] and the stepped
reconstruction as obs["recon_image"].  HologramVecEnv now returns views of
device buffers the reset / step kernels keep current (state_bytes, recon);
these tests check the mirrors against what they mirror after many random
steps with rollbacks:

  obs["state"]        == unpack_bits(mask)                         bit-exact
  obs["recon_image"]  stepped group == the propagated intensity of the stepped
                      (pre-rollback) mask; other groups == the propagated
                      intensity of the current mask                 bit-exact (same kernels)
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import hbx_oracle as O  # noqa: E402


def _env(cfg, B, seed, **kw):
    from hbx.env import HologramVecEnv
    g = torch.Generator(device="cuda").manual_seed(seed)
    pres = [torch.rand((cfg.channels, cfg.height, cfg.width), generator=g, device="cuda") for _ in range(B)]
    tgts = [torch.rand((cfg.groups, cfg.height, cfg.width), generator=g, device="cuda") for _ in range(B)]
    env = HologramVecEnv(cfg, B, lambda i: tgts[i], pre_model_source=lambda i: pres[i], auto_reset=False, **kw)
    return env, g


def _flip_words(mask, actions, cfg):
    """mask (B, CH, H, W/64) with each env's action pixel toggled."""
    m = mask.clone()
    hw = cfg.height * cfg.width
    for b, a in enumerate(actions.tolist()):
        ch, pix = divmod(a, hw)
        r, col = divmod(pix, cfg.width)
        w = col // 64
        bit = torch.tensor(1, dtype=torch.int64, device=m.device) << (col % 64)
        m[b, ch, r, w] ^= bit
    return m


@pytest.mark.parametrize("N,steps", [(1024, 200), (256, 300)])
def test_obs_mirrors_follow_steps_and_rollbacks(N, steps):
    import hbx
    from hbx.plan import unpack_bits
    cfg = hbx.rgb_config(1024) if N == 1024 else hbx.mono_config(256)
    B = 4
    env, g = _env(cfg, B, 17 + N)
    obs = env.reset()
    st = env.state
    assert obs["state"].data_ptr() == st.state_bytes.data_ptr()          # views, not copies
    assert obs["recon_image"].data_ptr() == st.recon.data_ptr()
    assert obs["state"].shape == (B, 1, cfg.channels, N, N) and obs["state"].dtype == torch.int8
    assert torch.equal(st.state_bytes, unpack_bits(st.mask, N))
    assert torch.equal(st.recon, st.intensity)
    plan = hbx.Plan(cfg, max_jobs=B * cfg.groups)
    acts = torch.randint(0, cfg.channels * N * N, (steps, B), generator=g, device="cuda")
    n_acc = n_rej = 0
    for k in range(steps):
        pre_mask = st.mask.clone()
        obs, r, dones, infos = env.step(acts[k])
        assert obs["state"].data_ptr() == st.state_bytes.data_ptr()
        assert torch.equal(st.state_bytes, unpack_bits(st.mask, N)), k
        acc = env.last_step()["accepted"]
        n_acc += int(acc.sum())
        n_rej += int((~acc).sum())
        if k % 20 == 0 or k == steps - 1:
            stepped = _flip_words(pre_mask, acts[k], cfg)
            tgt = st.target
            i_step, _, _ = plan.propagate(stepped, tgt)
            i_now, _, _ = plan.propagate(st.mask, tgt)
            gidx = (acts[k] // (N * N)) // cfg.planes
            for b in range(B):
                for gg in range(cfg.groups):
                    want = i_step[b, gg] if gg == int(gidx[b]) else i_now[b, gg]
                    assert torch.equal(obs["recon_image"][b, 0, gg], want), (k, b, gg)
    assert n_acc > 0 and n_rej > 0
    # the accepted-state cache is current after the next step's reconcile; a reset re-syncs
    env.reset_envs([1])
    assert torch.equal(st.recon[1], st.intensity[1]) and int(st.recon_pending[1]) == 0
    assert torch.equal(st.state_bytes, unpack_bits(st.mask, N))
    plan.close()
    env.close()


def test_obs_state_mirror_incremental_mode():
    """mode='psf' keeps obs["state"] in the same step kernel (k_env_step_finalize)."""
    import hbx
    from hbx.plan import unpack_bits
    cfg = hbx.rgb_config(1024)
    B = 3
    env, g = _env(cfg, B, 5, mode="psf", refresh_every=64,
                  obs_keys=("state_record", "state", "pre_model", "target_image"))
    env.reset()
    acts = torch.randint(0, cfg.channels * 1024 * 1024, (200, B), generator=g, device="cuda")
    for k in range(200):
        obs, _, _, _ = env.step(acts[k])
    assert obs["state"].data_ptr() == env.state.state_bytes.data_ptr()
    assert torch.equal(env.state.state_bytes, unpack_bits(env.state.mask, 1024))
    assert 0 < int(env.state.flip_count.sum()) < 200 * B
    env.close()


def test_obs_step_matches_oracle_small():
    """64 x 64 RGB: the observation dict after every step against the float64
    oracle env (state exact, recon_image within 2e-5 * max, stepped group
    pre-rollback), including rollbacks."""
    import hbx
    from hbx.env import HologramVecEnv
    ocfg = O.OpticsConfig(64, 64, 3, 2, O.WL_RGB)
    pre, tgt = O.synthetic_inputs(ocfg, 21)
    cfg = hbx.OpticsConfig(64, 64, 3, 2, O.WL_RGB)
    env = HologramVecEnv(cfg, 1, lambda i: tgt, pre_model_source=lambda i: pre, auto_reset=False)
    env.reset()
    ref = O.OracleEnv(ocfg)
    ref.reset(pre, tgt)
    prop = O.Propagator(ocfg)
    rng = np.random.default_rng(4)
    saw = set()
    for a in rng.integers(0, ocfg.channels * 64 * 64, 40):
        obs, _, _, _ = env.step(torch.tensor([int(a)], device="cuda"))
        before = ref.state.copy()
        res = ref.step(int(a))
        saw.add(res.accepted)
        c, r, col = O.decode_action(int(a), 64, 64)
        stepped = before.copy()
        stepped[c, r, col] ^= 1
        want_rec = prop.all_intensity(ref.state)
        gs = c // ocfg.planes
        want_rec[gs] = prop.group_intensity(stepped, gs)
        got = obs["recon_image"][0, 0].cpu().numpy()
        assert np.max(np.abs(got - want_rec)) <= 2e-5 * np.max(want_rec)
        assert np.array_equal(obs["state"][0, 0].cpu().numpy(), ref.state.astype(np.int8))
    assert saw == {True, False}
    env.close()


@pytest.mark.parametrize("mode,src", [("fft", "tensor"), ("planes", "tensor"), ("fft", "numpy"),
                                      ("planes", "numpy")])
def test_graph_replayed_step_equals_eager(mode, src):
    """HologramVecEnv(graph=True): the device step captured once into a HIP graph and replayed
    gives the eager step's rewards, flags, observations and state at every step, across
    auto-resets of env subsets (which run eagerly between replays).  src="numpy": the graph env
    gets numpy actions (what SB3 passes), read by the kernels from the host-mapped action row
    (r05, its own graph), against the eager env's device-tensor actions."""
    import hbx
    from hbx.env import HologramVecEnv, OBS_KEYS
    cfg = hbx.mono_config(256)
    B = 8
    g = torch.Generator(device="cuda").manual_seed(23)
    pres = [torch.rand((cfg.channels, 256, 256), generator=g, device="cuda") for _ in range(B)]
    tgts = [torch.rand((cfg.groups, 256, 256), generator=g, device="cuda") for _ in range(B)]
    kw = dict(pre_model_source=lambda i: pres[i], auto_reset=True, max_steps=25, obs_keys=OBS_KEYS, mode=mode)
    eager = HologramVecEnv(cfg, B, lambda i: tgts[i], **kw)
    graph = HologramVecEnv(cfg, B, lambda i: tgts[i], graph=True, **kw)
    eager.reset()
    graph.reset()
    acts = torch.randint(0, cfg.channels * 256 * 256, (80, B), generator=g, device="cuda")
    n_done = 0
    acts_h = acts.cpu().numpy()
    for k in range(80):
        o1, r1, d1, _ = eager.step(acts[k])
        o2, r2, d2, _ = graph.step(acts[k] if src == "tensor" else acts_h[k])
        assert np.array_equal(r1, r2) and np.array_equal(d1, d2), k
        for key in OBS_KEYS:
            assert torch.equal(o1[key], o2[key]), (k, key)
        n_done += int(d1.sum())
    assert (graph._graph if src == "tensor" else graph._graph_h) is not None and n_done > 0
    for key in ("mask", "chan_stats", "prev_psnr", "steps", "flip_count"):
        assert torch.equal(getattr(eager.state, key), getattr(graph.state, key)), key


@pytest.mark.parametrize("src", ["tensor", "numpy"])
def test_graph_step_follows_set_attr_and_plan_changes(src):
    """a HIP graph keeps the kernel arguments it was captured with, and
    EnvParams go to k_env_step_finalize by value.  After set_attr('max_steps' / 'T_PSNR', ...)
    or a plan timing change the graph-replayed env must behave as the eager env does."""
    import hbx
    from hbx.env import HologramVecEnv
    cfg = hbx.mono_config(256)
    B = 6
    g = torch.Generator(device="cuda").manual_seed(31)
    pres = [torch.rand((cfg.channels, 256, 256), generator=g, device="cuda") for _ in range(B)]
    tgts = [torch.rand((cfg.groups, 256, 256), generator=g, device="cuda") for _ in range(B)]
    kw = dict(pre_model_source=lambda i: pres[i], auto_reset=True, max_steps=1000, T_PSNR=1e9,
              T_PSNR_DIFF=1e9)
    eager = HologramVecEnv(cfg, B, lambda i: tgts[i], **kw)
    graph = HologramVecEnv(cfg, B, lambda i: tgts[i], graph=True, **kw)
    eager.reset()
    graph.reset()
    acts = torch.randint(0, cfg.channels * 256 * 256, (60, B), generator=g, device="cuda")
    acts_h = acts.cpu().numpy()
    ended = 0
    for k in range(60):
        if k == 5:                                      # after the graph has been captured
            assert (graph._graph if src == "tensor" else graph._graph_h) is not None
            for e in (eager, graph):
                e.set_attr("max_steps", 12)
        if k == 30:
            for e in (eager, graph):
                e.set_attr("max_steps", 1000)
                e.set_attr("T_PSNR", 0.0)               # every accepted step now counts as sustained
                e.set_attr("T_PSNR_DIFF", -1e9)
        if k == 40:
            graph.plan.set_timing(64, 2)                # plan per-call state changes: recapture
        o1, r1, d1, i1 = eager.step(acts[k])
        o2, r2, d2, i2 = graph.step(acts[k] if src == "tensor" else acts_h[k])
        assert np.array_equal(r1, r2) and np.array_equal(d1, d2), k
        assert [x.get("TimeLimit.truncated") for x in i1] == [x.get("TimeLimit.truncated") for x in i2], k
        assert [("terminal_observation" in x) for x in i1] == [("terminal_observation" in x) for x in i2], k
        if 5 <= k < 30:
            ended += int(d1.sum())
    assert ended > 0                                    # max_steps = 12 ended episodes (env.py:216-246)
    for key in ("mask", "chan_stats", "prev_psnr", "steps", "flip_count", "sustained"):
        assert torch.equal(getattr(eager.state, key), getattr(graph.state, key)), key
    eager.close()
    graph.close()


@pytest.mark.parametrize("G", [1, 3])
def test_obs_sync_resolve_right_after_accepted_step(G):
    """hbx_env_obs_sync(HBX_OBS_RECON) right after an accepted step used to copy
    the stale intensity cache over the correct recon and drop the pending reconcile.  With
    HBX_OBS_RESOLVE (ABI v10) the pending group goes recon -> intensity first; afterwards recon and
    the intensity cache both equal the propagation of the accepted mask, pending is 0, and the env
    keeps stepping exactly like an untouched twin.  ABI v12: at one colour group nothing is ever
    pending (every step rewrites recon whole) and HBX_OBS_RECON re-propagates the cache; the
    RGB case keeps the pending reconcile."""
    import hbx
    from hbx import _lib
    cfg = hbx.mono_config(256) if G == 1 else hbx.OpticsConfig(64, 64, 3, 2, (638e-9, 515e-9, 450e-9))
    N = cfg.height
    B = 4
    env, g = _env(cfg, B, 77)
    twin, _ = _env(cfg, B, 77)
    env.reset()
    twin.reset()
    st = env.state
    plan = hbx.Plan(cfg, max_jobs=B)
    acts = torch.randint(0, cfg.channels * N * N, (40, B), generator=g, device="cuda")
    synced = 0
    for k in range(40):
        # step_device: VecEnv.step settles accepted steps itself (HBX_OBS_SETTLE), this test
        # wants the pending reconcile an accepted step leaves behind
        env.step_device(acts[k])
        twin.step_device(acts[k])
        # the two agree after every step (a re-sync only changes what the previous step's
        # reconcile would have restored anyway)
        assert torch.equal(env.state.recon, twin.state.recon), k
        assert torch.equal(env.state.prev_psnr, twin.state.prev_psnr), k
        acc = env._acc.bool()
        if acc.any() and k % 3 == 0:
            if G > 1:
                assert int(st.recon_pending[acc].min()) > 0
            else:
                assert int(st.recon_pending.abs().sum()) == 0
            plan.env_obs_sync(st.bufs, B, _lib.OBS_RECON | _lib.OBS_RESOLVE)
            # recon now shows the CURRENT (accepted) state of every group, and so does the cache
            i_now, _, _ = plan.propagate(st.mask, st.target)
            assert torch.equal(st.recon, i_now) and torch.equal(st.intensity, i_now), k
            assert int(st.recon_pending.abs().sum()) == 0
            synced += 1
    assert synced > 0
    with pytest.raises(_lib.HbxError):
        plan.env_obs_sync(st.bufs, B, _lib.OBS_RESOLVE)         # a modifier of OBS_RECON only
    plan.close()
    env.close()
    twin.close()


@pytest.mark.parametrize("N", [256, 1024])
def test_step_host_row_equals_device_row(N):
    """ABI v11: step() has the step kernels write reward / psnr / flags and the error mirror
    straight into host-mapped memory (no device -> host copy).  Against a twin stepped through
    step_device (the device row): every result equal at every step; an out-of-range action
    still raises through the mirrored error word, and the env steps on afterwards."""
    import hbx
    cfg = hbx.rgb_config(1024) if N == 1024 else hbx.mono_config(256)
    B = 6
    a, g = _env(cfg, B, 91)
    b, _ = _env(cfg, B, 91)
    a.reset()
    b.reset()
    acts = torch.randint(0, cfg.channels * N * N, (40, B), generator=g, device="cuda")
    n_acc = 0
    for k in range(40):
        _, r, d, _ = a.step(acts[k])
        rew, psnr, acc, term, trunc = (t.cpu().numpy() for t in b.step_device(acts[k]))
        last = a.last_step()
        assert np.array_equal(r, rew) and np.array_equal(last["psnr"], psnr), k
        assert np.array_equal(last["accepted"], acc != 0), k
        assert np.array_equal(d, (term != 0) | (trunc != 0)), k
        n_acc += int(last["accepted"].sum())
    assert 0 < n_acc < 40 * B
    bad = acts[0].clone()
    bad[2] = cfg.channels * N * N          # out of range
    with pytest.raises(ValueError):
        a.step(bad)
    _, r, _, _ = a.step(acts[1])           # the word was cleared: the next step is clean
    assert np.isfinite(r).all()
    a.close()
    b.close()


def test_step_settles_accepted_groups():
    """VecEnv.step queues HBX_OBS_SETTLE behind its readback (ABI v11): after every step the
    accepted envs' intensity cache already holds the stepped group (= recon) with recon_pending
    cleared, rolled-back envs keep -(g + 1) and their cache; recon, the returned observation, is
    the stepped intensity either way, and the env steps exactly like a twin driven through
    step_device (which leaves the reconcile to the next step's k_rowinv)."""
    import hbx
    cfg = hbx.rgb_config(1024)
    B = 4
    env, g = _env(cfg, B, 29)
    twin, _ = _env(cfg, B, 29)
    env.reset()
    twin.reset()
    st = env.state
    acts = torch.randint(0, cfg.channels * 1024 * 1024, (60, B), generator=g, device="cuda")
    n_acc = n_rej = 0
    for k in range(60):
        before = st.intensity.clone()
        obs, _, _, _ = env.step(acts[k])
        twin.step_device(acts[k])
        acc = env.last_step()["accepted"]
        gidx = ((acts[k] // (1024 * 1024)) // cfg.planes).tolist()
        for b in range(B):
            gb = int(gidx[b])
            if acc[b]:
                n_acc += 1
                assert int(st.recon_pending[b]) == 0, (k, b)
                assert torch.equal(st.intensity[b, gb], st.recon[b, gb]), (k, b)
            else:
                n_rej += 1
                assert int(st.recon_pending[b]) == -(gb + 1), (k, b)
                assert torch.equal(st.intensity[b], before[b]), (k, b)
        assert torch.equal(obs["recon_image"][:, 0], twin.state.recon), k
        assert torch.equal(st.prev_psnr, twin.state.prev_psnr), k
    assert n_acc > 0 and n_rej > 0
    env.close()
    twin.close()


def test_step_chunked_batches_equal_one_batch():
    """A VecEnv whose plan holds fewer jobs than envs (max_jobs 4, 10 envs: three chunks per step,
    each decoding its actions in the first pass and reducing in its finalize) steps exactly like
    the one-chunk env: rewards, PSNRs, accept flags, observations; an out-of-range action in the
    last chunk raises through the mirrored error word."""
    import hbx
    cfg = hbx.mono_config(256)
    B = 10
    a, g = _env(cfg, B, 41, max_jobs=4)
    b, _ = _env(cfg, B, 41)
    oa, ob = a.reset(), b.reset()
    assert torch.equal(oa["recon_image"], ob["recon_image"])
    acts = torch.randint(0, cfg.channels * 256 * 256, (60, B), generator=g, device="cuda")
    for k in range(60):
        oa, ra, da, _ = a.step(acts[k])
        ob, rb, db, _ = b.step(acts[k])
        la, lb = a.last_step(), b.last_step()
        assert np.array_equal(ra, rb) and np.array_equal(da, db), k
        assert np.array_equal(la["psnr"], lb["psnr"]) and np.array_equal(la["accepted"], lb["accepted"]), k
        assert torch.equal(oa["recon_image"], ob["recon_image"]) and torch.equal(oa["state"], ob["state"]), k
    bad = acts[0].clone()
    bad[9] = -5
    with pytest.raises(ValueError):
        a.step(bad)
    a.close()
    b.close()


def test_numpy_actions_use_the_host_row_and_equal_tensor_actions():
    """SB3 hands VecEnv.step() numpy actions: they go into the host-mapped action row (no H2D copy;
    ABI v11 host memory) and the step equals the device-tensor step, rewards / flags / observations,
    including an out-of-range action raising like env.py's index error would."""
    import hbx
    from hbx.env import HologramVecEnv, OBS_KEYS
    cfg = hbx.mono_config(256)
    B = 5
    g = torch.Generator(device="cuda").manual_seed(41)
    pres = [torch.rand((cfg.channels, 256, 256), generator=g, device="cuda") for _ in range(B)]
    tgts = [torch.rand((cfg.groups, 256, 256), generator=g, device="cuda") for _ in range(B)]
    kw = dict(pre_model_source=lambda i: pres[i], auto_reset=True, max_steps=15, obs_keys=OBS_KEYS)
    a = HologramVecEnv(cfg, B, lambda i: tgts[i], **kw)
    b = HologramVecEnv(cfg, B, lambda i: tgts[i], **kw)
    a.reset()
    b.reset()
    acts = torch.randint(0, cfg.channels * 256 * 256, (40, B), generator=g, device="cuda")
    acts_h = acts.cpu().numpy()
    for k in range(40):
        o1, r1, d1, _ = a.step(acts[k])
        o2, r2, d2, _ = b.step(acts_h[k])
        assert np.array_equal(r1, r2) and np.array_equal(d1, d2), k
        assert np.array_equal(b._act_np, acts_h[k])
        for key in OBS_KEYS:
            assert torch.equal(o1[key], o2[key]), (k, key)
    bad = acts_h[0].copy()
    bad[2] = cfg.channels * 256 * 256
    with pytest.raises(ValueError):
        b.step(bad)
    a.close()
    b.close()


def test_dropin_graph_replay_equals_eager():
    """hbx.env.BinaryHologramEnv(graph=True): the drop-in step replayed from the host-action graph
    returns the eager drop-in env's rewards, flags and observations."""
    import hbx
    from hbx.env import BinaryHologramEnv
    N = 256
    rng = np.random.default_rng(5)
    pre = rng.random((8, N, N), np.float32)
    tgt = rng.random((1, N, N), np.float32)
    envs = [BinaryHologramEnv(lambda t: torch.from_numpy(pre[None]).to(t.device), [(torch.from_numpy(tgt[None]), ["x"])],
                              max_steps=30, config=hbx.mono_config(N), verbose=False, graph=gr) for gr in (False, True)]
    for e in envs:
        e.reset()
    ended = False
    for k, a in enumerate(rng.integers(0, 8 * N * N, 34).tolist()):
        (o1, r1, t1, u1, _), (o2, r2, t2, u2, _) = (e.step(a) for e in envs)
        assert (r1, t1, u1) == (r2, t2, u2), k
        for key in o1:
            assert np.array_equal(o1[key], o2[key]), (k, key)
        ended |= t1 or u1
    assert envs[1]._vec._graph_h is not None and ended
    for e in envs:
        e.close()


@pytest.mark.parametrize("N,G,steps", [(256, 1, 300), (64, 3, 200)])
def test_numpy_obs_host_mirrors_equal_torch_obs(N, G, steps):
    """obs_format="numpy" (VERDICT r05 #4): host mirrors updated by env.py:164-181's rules, only
    recon_image copied device -> host per step.  Against a twin env with obs_format="torch": every
    key equal at every step across rollbacks and auto-resets; an observation the caller holds
    keeps its values through the next step (SB3 adds _last_obs after the following step); the
    per-step D2H is recon alone; terminal observations match; a bare step_device re-syncs the
    mirrors."""
    import hbx
    from hbx.env import HologramVecEnv, OBS_KEYS
    cfg = hbx.mono_config(N) if G == 1 else hbx.OpticsConfig(N, N, 3, 2, hbx.plan.WL_RGB)
    B = 6
    g = torch.Generator(device="cuda").manual_seed(41 + N)
    pres = [torch.rand((cfg.channels, N, N), generator=g, device="cuda") for _ in range(B)]
    tgts = [torch.rand((cfg.groups, N, N), generator=g, device="cuda") for _ in range(B)]
    kw = dict(pre_model_source=lambda i: pres[i], auto_reset=True, max_steps=37, obs_keys=OBS_KEYS)
    ref = HologramVecEnv(cfg, B, lambda i: tgts[i], **kw)
    npy = HologramVecEnv(cfg, B, lambda i: tgts[i], obs_format="numpy", **kw)
    o_ref, o_np = ref.reset(), npy.reset()
    for k in OBS_KEYS:
        assert isinstance(o_np[k], np.ndarray) and np.array_equal(o_np[k], o_ref[k].cpu().numpy()), k
    acts = torch.randint(0, cfg.channels * N * N, (steps, B), generator=g, device="cuda")
    acts_h = acts.cpu().numpy()
    held, held_want = None, None
    n_done = n_rej = 0
    recon_bytes = B * cfg.groups * N * N * 4
    resync = False
    for s in range(steps):
        o1, r1, d1, i1 = ref.step(acts[s])
        o2, r2, d2, i2 = npy.step(acts_h[s])
        assert np.array_equal(r1.astype(np.float32), r2) and np.array_equal(d1, d2), s
        for k in OBS_KEYS:
            assert np.array_equal(o2[k], o1[k].cpu().numpy()), (s, k)
        if held is not None:                      # the obs returned one step ago is unchanged
            for k in OBS_KEYS:
                assert np.array_equal(held[k], held_want[k]), (s, k)
        held, held_want = o2, {k: v.copy() for k, v in o2.items()}
        n_rej += int((~ref.last_step()["accepted"]).sum())
        if d1.any():
            n_done += int(d1.sum())
            for i in np.nonzero(d1)[0]:
                for k in OBS_KEYS:
                    assert np.array_equal(i2[i]["terminal_observation"][k],
                                          i1[i]["terminal_observation"][k].cpu().numpy()), (s, i, k)
        elif not resync:
            assert npy._mirror.d2h_bytes == recon_bytes, s
        resync = s == steps // 2
        if resync:                                # a bare device step: the next step re-copies
            ref.step_device(acts[s])
            npy.step_device(acts[s])
    assert n_done > 0 and n_rej > 0
    ref.close()
    npy.close()


def test_graph_lazy_obs_snapshot_not_recorded():
    """graph=True + obs_format='lazy' + numpy actions.  An observation left unread
    across two more steps still shows its own step's data (the snapshot runs before the capture,
    not inside the graph), and device() hands out a stable copy, not the live buffer."""
    import hbx
    from hbx.env import HologramVecEnv, OBS_KEYS
    cfg = hbx.mono_config(256)
    B = 4
    g = torch.Generator(device="cuda").manual_seed(29)
    pres = [torch.rand((cfg.channels, 256, 256), generator=g, device="cuda") for _ in range(B)]
    tgts = [torch.rand((cfg.groups, 256, 256), generator=g, device="cuda") for _ in range(B)]
    kw = dict(pre_model_source=lambda i: pres[i], auto_reset=False, obs_keys=OBS_KEYS)
    eager = HologramVecEnv(cfg, B, lambda i: tgts[i], **kw)
    lazy = HologramVecEnv(cfg, B, lambda i: tgts[i], obs_format="lazy", graph=True, **kw)
    eager.reset()
    lazy.reset()
    acts = torch.randint(0, cfg.channels * 256 * 256, (12, B), generator=g, device="cuda").cpu().numpy()
    kept = []
    for s in range(12):
        o1, _, _, _ = eager.step(acts[s])
        o2, _, _, _ = lazy.step(acts[s])
        want = {k: o1[k].cpu().numpy().copy() for k in OBS_KEYS}
        dev = o2.device("state") if s % 3 == 0 else None
        kept.append((o2, want, dev))
        if len(kept) > 2:
            old, old_want, old_dev = kept[-3]
            for k in OBS_KEYS:
                assert np.array_equal(old[k], old_want[k]), (s, k)
            if old_dev is not None:
                assert np.array_equal(old_dev.cpu().numpy(), old_want["state"]), s
                assert old_dev.data_ptr() != lazy.state.state_bytes.data_ptr()
    assert lazy._graph_h is not None
    eager.close()
    lazy.close()


@pytest.mark.parametrize("rgb", [False, True])
def test_lazy_obs_undo_and_recon_pingpong_equal_torch_obs(rgb):
    """obs_format="lazy" (r06): on SB3's host-action step an unread state / state_record is kept by
    an undo log and recon_image (one colour group) by the recon ping-pong, no device copy.  Against
    a torch-format twin: every LazyObs read 0, 1, 2 or 5 steps after it was returned shows its own
    step's values, across rollbacks, auto-resets and an out-of-range action; RGB (G = 3) takes the
    recon clone."""
    import hbx
    from hbx.env import HologramVecEnv, OBS_KEYS
    cfg = hbx.OpticsConfig(64, 64, 3, 2, hbx.plan.WL_RGB) if rgb else hbx.mono_config(256)
    N = cfg.height
    B = 4
    g = torch.Generator(device="cuda").manual_seed(61)
    pres = [torch.rand((cfg.channels, N, N), generator=g, device="cuda") for _ in range(B)]
    tgts = [torch.rand((cfg.groups, N, N), generator=g, device="cuda") for _ in range(B)]
    kw = dict(pre_model_source=lambda i: pres[i], auto_reset=True, max_steps=23, obs_keys=OBS_KEYS)
    ref = HologramVecEnv(cfg, B, lambda i: tgts[i], **kw)
    lazy = HologramVecEnv(cfg, B, lambda i: tgts[i], obs_format="lazy", **kw)
    ref.reset()
    lazy.reset()
    acts = torch.randint(0, cfg.channels * N * N, (90, B), generator=g, device="cuda").cpu().numpy()
    held = []                                   # (LazyObs, its step's values, read after k steps)
    swaps = 0
    for s in range(90):
        if s == 45:                             # an out-of-range action: ValueError, other envs step
            bad = acts[s].copy()
            bad[1] = cfg.channels * N * N
            for e in (ref, lazy):
                with pytest.raises(ValueError):
                    e.step(bad)
            continue
        o1, _, d1, _ = ref.step(acts[s])
        live = lazy.state.recon.data_ptr()
        o2, _, d2, _ = lazy.step(acts[s])
        swaps += int(lazy.state.recon.data_ptr() != live)
        assert np.array_equal(d1, d2), s
        held.append((o2, {k: o1[k].cpu().numpy().copy() for k in OBS_KEYS}, s, (0, 1, 2, 5)[s % 4]))
        keep = []
        for lz, want, s0, k in held:
            if s - s0 == k:
                for key in OBS_KEYS:
                    assert np.array_equal(lz[key], want[key]), (s0, s, key)
            else:
                keep.append((lz, want, s0, k))
        held = keep
    assert not rgb and swaps > 0 or rgb and swaps == 0
    ref.close()
    lazy.close()
