"""Plane-cached FFT mode (ABI v9, HologramVecEnv(mode="planes")).

A step of env.py:154-259 flips ONE pixel of one plane; the FFT mode re-propagates all P planes of
the touched colour group, and the P - 1 untouched planes' |U_q|^2 come out bit-identical every
time (deterministic kernels, same inputs).  The plane-cached mode keeps each plane's |U_q|^2,
propagates only the flipped plane's pair (the pair packing of k_rowfwd is kept, so the two planes'
values are the FFT mode's bits too) and sums the planes in the same order.  So the claim tested
here is bit-exactness against the FFT mode, step by step, with rollbacks and resets:
rewards, PSNRs, accept / terminate / truncate flags, masks, records, channel statistics and the
recon_image observation.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _pair(cfg, B, seed, max_steps=10000, obs_keys=None):
    from hbx.env import HologramVecEnv, OBS_KEYS
    g = torch.Generator(device="cuda").manual_seed(seed)
    pres = [torch.rand((cfg.channels, cfg.height, cfg.width), generator=g, device="cuda") for _ in range(B)]
    tgts = [torch.rand((cfg.groups, cfg.height, cfg.width), generator=g, device="cuda") for _ in range(B)]
    kw = dict(pre_model_source=lambda i: pres[i], auto_reset=True, max_steps=max_steps,
              obs_keys=OBS_KEYS if obs_keys is None else obs_keys)
    fft = HologramVecEnv(cfg, B, lambda i: tgts[i], mode="fft", **kw)
    planes = HologramVecEnv(cfg, B, lambda i: tgts[i], mode="planes", **kw)
    return fft, planes, g


def _same_state(a, b, what):
    sa, sb = a.state, b.state
    for k in ("mask", "record", "chan_stats", "prev_psnr", "init_psnr", "steps", "flip_count", "sustained"):
        assert torch.equal(getattr(sa, k), getattr(sb, k)), (what, k)


@pytest.mark.parametrize("N,B,steps,max_steps", [(1024, 4, 120, 10000), (256, 16, 300, 40), (896, 4, 120, 50)])
def test_planes_mode_bit_exact_vs_fft_mode(N, B, steps, max_steps):
    """N = 896 (r06): the 64-pixel centre crop of env_1024_24_128.py:144-149 on the mixed-radix
    28 x 32 passes, whose plane-cached step is built the same way (hbx_passes896.hip)."""
    import hbx
    cfg = hbx.mono_config(256) if N == 256 else hbx.rgb_config(N)
    fft, planes, g = _pair(cfg, B, 5 + N, max_steps=max_steps)
    o1, o2 = fft.reset(), planes.reset()
    assert torch.equal(o1["recon_image"], o2["recon_image"])
    _same_state(fft, planes, "reset")
    acts = torch.randint(0, cfg.channels * N * N, (steps, B), generator=g, device="cuda")
    n_acc = n_rej = n_done = 0
    for k in range(steps):
        o1, r1, d1, _ = fft.step(acts[k])
        o2, r2, d2, _ = planes.step(acts[k])
        assert np.array_equal(r1, r2), k
        assert np.array_equal(d1, d2), k
        l1, l2 = fft.last_step(), planes.last_step()
        assert np.array_equal(l1["psnr"], l2["psnr"]), k
        assert np.array_equal(l1["accepted"], l2["accepted"]), k
        assert torch.equal(o1["recon_image"], o2["recon_image"]), k      # stepped (pre-rollback) group too
        assert torch.equal(o1["state"], o2["state"]), k
        n_acc += int(l1["accepted"].sum())
        n_rej += int((~l1["accepted"]).sum())
        n_done += int(np.sum(d1))
        if k % 30 == 0 or k == steps - 1:
            _same_state(fft, planes, k)
    assert n_acc > 0 and n_rej > 0
    if max_steps < steps:
        assert n_done > 0          # auto resets of subsets of envs went through the fill pass


def test_planes_mode_chunked_launches_equal_fft_mode():
    """More envs than the plan's max_jobs: the step and the reset fill run in launch chunks, the
    pool / slot pointers offset per chunk (hbx_env_step, propagate_full) -- still bit-exact."""
    import hbx
    from hbx.env import HologramVecEnv, OBS_KEYS
    cfg = hbx.mono_config(256)
    B = 7
    g = torch.Generator(device="cuda").manual_seed(41)
    pres = [torch.rand((cfg.channels, 256, 256), generator=g, device="cuda") for _ in range(B)]
    tgts = [torch.rand((cfg.groups, 256, 256), generator=g, device="cuda") for _ in range(B)]
    kw = dict(pre_model_source=lambda i: pres[i], auto_reset=True, max_steps=15, obs_keys=OBS_KEYS, max_jobs=3)
    fft = HologramVecEnv(cfg, B, lambda i: tgts[i], mode="fft", **kw)
    planes = HologramVecEnv(cfg, B, lambda i: tgts[i], mode="planes", **kw)
    fft.reset()
    planes.reset()
    acts = torch.randint(0, cfg.channels * 256 * 256, (50, B), generator=g, device="cuda")
    for k in range(50):
        o1, r1, d1, _ = fft.step(acts[k])
        o2, r2, d2, _ = planes.step(acts[k])
        assert np.array_equal(r1, r2) and np.array_equal(d1, d2), k
        assert torch.equal(o1["recon_image"], o2["recon_image"]), k
    _same_state(fft, planes, "chunked")


def test_planes_cache_holds_current_planes_and_resumes(tmp_path):
    """After random steps every cached plane equals |U_q|^2 of the current mask (hbx_simulate);
    a save() / load() round trip rebuilds the cache and the env continues bit for bit."""
    import hbx
    cfg = hbx.rgb_config(256)
    B = 3
    fft, planes, g = _pair(cfg, B, 11)
    fft.reset()
    planes.reset()
    acts = torch.randint(0, cfg.channels * 256 * 256, (80, B), generator=g, device="cuda")
    for k in range(40):
        fft.step(acts[k])
        planes.step(acts[k])
    st = planes.state
    field, _ = planes.plan.simulate(st.mask)
    inten = field.real ** 2 + field.imag ** 2                             # |U|^2 per plane (f32)
    slots = st.plane_slot.long()
    for b in range(B):
        got = st.plane_inten[b][slots[b, :cfg.channels]]
        assert torch.allclose(got, inten[b], rtol=1e-5, atol=1e-6 * float(inten[b].max()))
    path = str(tmp_path / "planes.npz")
    planes.save(path)
    planes2 = type(planes)(cfg, B, planes.target_source, pre_model_source=planes.pre_model_source,
                           mode="planes", auto_reset=True)
    planes2.reset()
    planes2.load(path)
    for k in range(40, 80):
        o1, r1, d1, _ = fft.step(acts[k])
        o2, r2, d2, _ = planes2.step(acts[k])
        assert np.array_equal(r1, r2), k
        assert torch.equal(o1["recon_image"], o2["recon_image"]), k
    _same_state(fft, planes2, "resumed")


def test_planes_mode_rejects_unbuilt_sizes_and_half_buffers():
    import hbx
    from hbx.env import HologramVecEnv
    cfg = hbx.rgb_config(64)
    with pytest.raises(ValueError):
        HologramVecEnv(cfg, 2, lambda i: torch.rand(3, 64, 64), pre_model_source=lambda i: torch.rand(24, 64, 64),
                       mode="planes")
    cfg = hbx.mono_config(256)
    env = HologramVecEnv(cfg, 2, lambda i: torch.rand(1, 256, 256, device="cuda"),
                         pre_model_source=lambda i: torch.rand(8, 256, 256, device="cuda"), mode="planes")
    env.reset()
    env.state.bufs.plane_slot = None                                     # pool without slot table
    with pytest.raises(RuntimeError):
        env.step_device(torch.zeros(2, dtype=torch.int64, device="cuda"))


def test_planes_896_greedy_walk_equals_host_batches():
    """(r06) the FFT-mode greedy DBS on the plane cache at N = 896 (DBS_1024_24-128.py's crop): the
    device walk (its decision in a launch of its own behind each batch at 896) and the full
    re-propagation per candidate (planes=False) give the same accept sequence and PSNR bits."""
    import hbx
    from hbx import dbs
    cfg = hbx.rgb_config(896)
    g = torch.Generator(device="cuda").manual_seed(3)
    pre = torch.rand((cfg.channels, 896, 896), generator=g, device="cuda")
    tgt = torch.rand((cfg.groups, 896, 896), generator=g, device="cuda")
    mask = hbx.pack_mask(pre, threshold=0.5)
    order = np.random.default_rng(3).permutation(cfg.channels * 896 * 896)[:1500]
    plan = hbx.Plan(cfg, max_jobs=8)
    walk = dbs.greedy(plan, mask.clone(), tgt, order=order, mode="fft", planes=True)
    ref = dbs.greedy(plan, mask.clone(), tgt, order=order, mode="fft", planes=False, k_max=8)
    assert walk.accepted_positions == ref.accepted_positions and len(walk.accepted_positions) > 0
    assert walk.final_psnr == ref.final_psnr
    plan.close()
