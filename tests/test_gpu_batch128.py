"""BASELINE configs[2] as a test: the batched VecEnv step at its benchmarked size,
128 envs x 1024x1024x24 in one launch sequence (the XCD block mapping, the
workspace offsets of all 128 jobs and the per-env finalize all at full scale).

  * 4 sampled envs per step against the float64 oracle on the SAME state
    (O.LinearGreedy, following the GPU's accept decisions): PSNR, reward,
    accept flag wherever the change is clear of the FFT mode's f32 resolution.
  * all 128 envs through identities that need no oracle:
      Parseval   the ASM transfer function has |H| = 1 at these parameters
                 (evanescent cut inactive), so sum_x I_g = popcount(group) / P
      stats      the cached channel sums equal sum I T, sum I^2, sum T^2 of the cached
                 intensity and the target (f64, torch)
      psnr       prev_psnr = PSNR(chan_stats) of every env
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import hbx_oracle as O  # noqa: E402

FFT_TOL_DB = 2e-9    # FFT-mode per-candidate change vs the oracle (tests/test_gpu_dbs_headline.py)


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm GPU")
    import hbx
    hbx.load_library()
    yield


@pytest.mark.timeout(300)
def test_vecenv_step_128x1024x24():
    import hbx
    from hbx.env import HologramVecEnv
    B, N, G, P = 128, 1024, 3, 8
    CH = G * P
    cfg = hbx.rgb_config(N)

    def tsrc(i):
        g = torch.Generator(device="cuda").manual_seed(1_000_003 * i + 1)
        return torch.rand((G, N, N), generator=g, device="cuda")

    def psrc(i):
        g = torch.Generator(device="cuda").manual_seed(1_000_003 * i)
        return torch.rand((CH, N, N), generator=g, device="cuda")

    env = HologramVecEnv(cfg, B, tsrc, pre_model_source=psrc, obs_keys=("recon_image",), auto_reset=False)
    env.reset()
    st = env.state
    sample = [0, 37, 90, 127]
    ocfg = O.rgb_config(N)
    oracles = {}
    for b in sample:
        m = O.unpack_mask(st.mask[b].cpu().numpy().view("<u8"), N).astype(np.float32)
        oracles[b] = O.LinearGreedy(ocfg, m, st.target[b].cpu().numpy())
        assert abs(float(st.init_psnr[b]) - oracles[b].initial_psnr) <= 1e-4
    gen = torch.Generator(device="cuda").manual_seed(2)
    clear = 0
    for k in range(4):
        acts = torch.randint(0, CH * N * N, (B,), generator=gen, device="cuda", dtype=torch.int64)
        r, ps, acc, term, trunc = env.step_device(acts)
        env.state.check_error()
        a_h, r_h, ps_h, acc_h = acts.cpu().numpy(), r.cpu().numpy(), ps.cpu().numpy(), acc.cpu().numpy()
        assert not term.any() and not trunc.any()
        for b in sample:
            lg = oracles[b]
            ev = lg.evaluate(int(a_h[b]))
            change = ev[0] - lg.previous_psnr
            assert abs(ps_h[b] - ev[0]) <= 1e-4
            assert abs(r_h[b] - O.RW * change) <= O.RW * FFT_TOL_DB * 4
            if abs(change) > FFT_TOL_DB:
                clear += 1
                assert bool(acc_h[b]) == (change >= 0), (k, b, change)
            if bool(acc_h[b]):                                   # follow the GPU's decision
                lg.commit(int(a_h[b]), ev)
    assert clear >= 12
    torch.cuda.synchronize()
    # every env's mask is the oracle-followed state for the sampled ones
    for b in sample:
        want = O.pack_mask(oracles[b].state.astype(np.uint8))
        assert np.array_equal(st.mask[b].cpu().numpy().view("<u8"), want)
    # all 128 envs: Parseval, stats-vs-intensity, psnr-vs-stats
    bits = hbx.unpack_bits(st.mask, N).reshape(B, G, P, N, N)
    pop = bits.to(torch.float64).sum(dim=(2, 3, 4)) / P                # [B, G]
    isum = st.intensity.double().sum(dim=(2, 3))                       # [B, G]
    assert torch.allclose(isum, pop, rtol=2e-6, atol=0)
    I, T = st.intensity.double(), st.target.double()
    stats = torch.stack([(I * T).sum(dim=(2, 3)), (I * I).sum(dim=(2, 3)), (T * T).sum(dim=(2, 3))], dim=2)
    assert torch.allclose(st.chan_stats, stats, rtol=2e-6, atol=0)
    assert torch.allclose(env.plan.psnr(st.chan_stats), st.prev_psnr, rtol=0, atol=1e-9)
    assert int(st.steps.sum()) == 4 * B
    env.close()
