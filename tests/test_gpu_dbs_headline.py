"""Greedy-DBS decisions at the reference's full sizes, pinned by float64 fixtures.

DBS_1024_24.py:313-422 keeps a flip iff the PSNR strictly improves (`:355`).
At 1024x1024x24 a single flip moves the PSNR by a median 6.7e-7 dB, so the
accept sequence is only meaningful if every candidate's PSNR change is
resolved far below that.  The fixtures (tests/golden/make_golden.py --large)
hold the float64 oracle's accept sequence and per-candidate PSNR change
(O.LinearGreedy: exact increments by linearity, checked against the
re-propagating oracle in tests/test_oracle.py) over

  dbs_prefix_1024x24.npz        the first 4096 candidates of rng(3).permutation(24 * 1024^2)
                                on the seed-0 synthetic image (amplitude field), plus the
                                change of the first 512 candidates against the initial state
  dbs_prefix_1024x24_phase.npz  4096 candidates, binary-phase field
  dbs_prefix_896x24.npz         2048 candidates at the 896 x 896 x 24 crop size (seed 7)
  env_trace_1024x24.npz         2,000 env steps (rng(2) actions) with env.py's rollback rule
                                (roll back iff change < 0), 1,010 accepts
  dbs_ratio05_256.npz           DBS_ratio_0.5.py's literal run (BASELINE configs[4]):
                                256x256x8 mono until the PSNR has risen 0.5 dB (:366-372)

Measured bounds the tests state (MI355X):
  incremental-field path (device walk, host-decided batches, eval_flips_psf): the flip's
    increments are summed in f64 from an f32 increment per pixel, so a candidate's PSNR
    change is within INCR_TOL_DB of the oracle's; its decisions must equal the oracle's
    everywhere (the fixture's closest call is 3.6e-10 dB).
  FFT mode (the reference's algorithm: the whole touched group re-propagated in f32): a
    candidate's change carries the f32 FFT roundoff of two full-image sums, FFT_TOL_DB;
    a decision may differ from the oracle's only at a candidate whose |change| is within
    that bound, after which the two runs visit different states and the comparison stops.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import hbx_oracle as O  # noqa: E402

INCR_TOL_DB = 1e-11     # incremental path vs f64 oracle, per-candidate PSNR change (measured 9.5e-13)
FFT_TOL_DB = 2e-9       # FFT re-propagation vs f64 oracle, per-candidate PSNR change (measured 1.4e-9)
ENV_FFT_TOL_DB = 4e-9   # FFT-mode env step: the change is this flip's re-propagated PSNR minus the
                        # previous accepted flip's, two independent f32 roundoffs (measured 2.5e-9)
GAIN_TOL_DB = 1e-8      # accumulated PSNR gain of the accepted flips vs the oracle's (measured
                        # 7.5e-11 walk without refresh, 3.7e-9 with exact refreshes every 256
                        # accepts, 7.9e-9 FFT mode)


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm GPU")
    import hbx
    hbx.load_library()
    yield


def _fixture(golden_dir, name):
    d = np.load(os.path.join(golden_dir, name), allow_pickle=False)
    n, g, p = int(d["size"]), int(d["groups"]), int(d["planes"])
    wl = O.WL_RGB if g == 3 else O.WL_MONO
    ocfg = O.OpticsConfig(n, n, g, p, wl, field_kind=int(d["field_kind"]))
    pre, tgt = O.synthetic_inputs(ocfg, int(d["seed"]))
    order = np.random.default_rng(int(d["order_seed"])).permutation(ocfg.channels * n * n)
    return d, ocfg, pre, tgt, order


def _dev(ocfg, pre, tgt, precision=0, max_jobs=256):
    import hbx
    cfg = hbx.OpticsConfig(ocfg.height, ocfg.width, ocfg.groups, ocfg.planes, tuple(ocfg.wavelengths),
                           field_kind=ocfg.field_kind)
    plan = hbx.Plan(cfg, max_jobs=max_jobs, precision=precision)
    mask = hbx.pack_bits(torch.from_numpy(pre).cuda() >= 0.5)
    target = torch.from_numpy(tgt).cuda()
    return plan, mask, target


def _first_difference(positions, accepted):
    got = np.zeros(len(accepted), bool)
    pos = np.asarray(positions, np.int64)
    pos = pos[pos < len(accepted)]
    got[pos] = True
    diff = np.nonzero(got != accepted)[0]
    return int(diff[0]) if len(diff) else None


def _abs_psnr_resolution(plan, ocfg, tgt, n_states):
    """Max |device PSNR - oracle PSNR| of one propagation over n_states seeded random
    masks at the plan's size: the f32 resolution of an absolute PSNR."""
    import hbx
    prop = O.Propagator(ocfg)
    worst = 0.0
    for s in range(n_states):
        m = (np.random.default_rng(1000 + s).random((ocfg.channels, ocfg.height, ocfg.width)) >= 0.5)
        inten = prop.all_intensity(m.astype(np.uint8))
        want = prop.psnr(np.stack([O.chan_stats(inten[g], tgt[g]) for g in range(ocfg.groups)]))
        bits = hbx.pack_bits(torch.from_numpy(m).cuda())
        _, _, ps = plan.propagate(bits[None], torch.from_numpy(tgt).cuda()[None], want_intensity=False)
        worst = max(worst, abs(float(ps[0]) - want))
    return worst


def _gain_error(res, d, upto):
    acc_idx = np.nonzero(d["accepted"][:upto])[0]
    pos = np.asarray(res.accepted_positions, np.int64)
    k = int(np.searchsorted(pos, upto))
    n = min(k, len(acc_idx))
    if n == 0:
        return 0.0
    got = np.asarray(res.accepted_psnr[:n]) - res.initial_psnr
    want = d["psnr"][acc_idx[:n]] - float(d["initial_psnr"])
    return float(np.max(np.abs(got - want)))


@pytest.mark.parametrize("name", ["dbs_prefix_1024x24.npz", "dbs_prefix_1024x24_phase.npz", "dbs_prefix_896x24.npz"])
@pytest.mark.parametrize("mode,refresh", [("psf", 4096), ("psf", 256), ("psf_host", 4096)])
def test_incremental_greedy_1024x24_equals_oracle(golden_dir, name, mode, refresh):
    """Device walk and host-decided batches: the oracle's accept sequence,
    every decision, at the headline size (with and without exact refreshes)."""
    from hbx import dbs
    d, ocfg, pre, tgt, order = _fixture(golden_dir, name)
    n = int(d["n"])
    plan, mask, target = _dev(ocfg, pre, tgt)
    res = dbs.greedy(plan, mask, target, order[:n], mode=mode, refresh_every=refresh)
    first = _first_difference(res.accepted_positions, d["accepted"])
    assert first is None, (first, float(d["delta"][first]))
    assert res.steps == n
    gerr = _gain_error(res, d, n)
    print(f"{name} {mode} refresh={refresh}: {len(res.accepted_positions)} accepts, gain error {gerr:.2e} dB")
    assert gerr <= GAIN_TOL_DB
    assert abs(res.initial_psnr - float(d["initial_psnr"])) <= 1e-4
    # the mask is the oracle's initial mask with exactly the accepted flips toggled
    want = (pre >= 0.5).astype(np.uint8)
    c, r, col = O.decode_action(order[:n][d["accepted"]], ocfg.height, ocfg.width)
    np.bitwise_xor.at(want, (c, r, col), 1)
    assert np.array_equal(mask.cpu().numpy().view("<u8"), O.pack_mask(want))
    plan.close()


@pytest.mark.parametrize("persist", ["0", "1"])
@pytest.mark.parametrize("refresh", [4096, 256])
def test_incremental_greedy_1024x24_16k_equals_oracle(golden_dir, refresh, persist, monkeypatch):
    """The device walk over a 16,384-candidate prefix of the 1024x24 sweep (the float64
    oracle's run, dbs_prefix_1024x24_16k.npz): every decision the oracle's, with and
    without exact refreshes, with one launch per batch and with the persistent walk
    (HBX_WALK_PERSIST=1: one cooperative launch per call, a grid barrier per batch)."""
    from hbx import dbs
    monkeypatch.setenv("HBX_WALK_PERSIST", persist)   # read at plan creation
    d, ocfg, pre, tgt, order = _fixture(golden_dir, "dbs_prefix_1024x24_16k.npz")
    n = int(d["n"])
    plan, mask, target = _dev(ocfg, pre, tgt)
    res = dbs.greedy(plan, mask, target, order[:n], mode="psf", refresh_every=refresh)
    first = _first_difference(res.accepted_positions, d["accepted"])
    assert first is None, (first, float(d["delta"][first]))
    assert res.steps == n
    gerr = _gain_error(res, d, n)
    print(f"16k prefix refresh={refresh}: {len(res.accepted_positions)} accepts, gain error {gerr:.2e} dB")
    assert gerr <= GAIN_TOL_DB
    want = (pre >= 0.5).astype(np.uint8)
    c, r, col = O.decode_action(order[:n][d["accepted"]], ocfg.height, ocfg.width)
    np.bitwise_xor.at(want, (c, r, col), 1)
    assert np.array_equal(mask.cpu().numpy().view("<u8"), O.pack_mask(want))
    plan.close()


@pytest.mark.parametrize("name", ["dbs_prefix_1024x24.npz", "dbs_prefix_1024x24_16k.npz", "dbs_prefix_896x24.npz"])
def test_fft_greedy_1024x24_vs_oracle(golden_dir, name):
    """FFT mode (every candidate a full f32 re-propagation of its group): the
    oracle's accept sequence up to the first candidate whose change lies within
    the f32 FFT resolution FFT_TOL_DB."""
    from hbx import dbs
    d, ocfg, pre, tgt, order = _fixture(golden_dir, name)
    n = int(d["n"])
    plan, mask, target = _dev(ocfg, pre, tgt)
    res = dbs.greedy(plan, mask, target, order[:n], mode="fft")
    first = _first_difference(res.accepted_positions, d["accepted"])
    upto = n if first is None else first
    if first is not None:
        assert abs(float(d["delta"][first])) <= FFT_TOL_DB, (first, float(d["delta"][first]))
    assert upto >= 1024
    gerr = _gain_error(res, d, upto)
    print(f"fft mode: first difference {first}, gain error {gerr:.2e} dB")
    assert gerr <= 50 * FFT_TOL_DB
    plan.close()


@pytest.mark.parametrize("name,stop", [("dbs_prefix_1024x24_16k.npz", None), ("dbs_ratio05_256.npz", 0.5),
                                       ("dbs_prefix_1024x24_phase.npz", None)])
def test_fft_greedy_plane_cache_equals_full_repropagation(golden_dir, name, stop):
    """the FFT-mode greedy with the base state's plane cache (hbx_eval_flips_planes,
    only the flipped plane's pair propagated per candidate) makes the full re-propagation's
    decisions with the full re-propagation's PSNR BITS -- every accepted PSNR equal, the same
    candidates visited, the same final mask."""
    from hbx import dbs
    d, ocfg, pre, tgt, order = _fixture(golden_dir, name)
    n = int(d["n"])
    runs = {}
    for planes, walk in ((False, False), (True, False), (True, True)):
        plan, mask, target = _dev(ocfg, pre, tgt)
        res = dbs.greedy(plan, mask, target, order[:n], stop_diff=stop, mode="fft", planes=planes,
                         device_walk=walk)
        runs[(planes, walk)] = (res, mask.cpu().numpy())
        plan.close()
    full, m_full = runs[(False, False)]
    for key in ((True, False), (True, True)):    # host-decided and device-decided batches
        cached, m_cached = runs[key]
        print(f"{name} planes / device walk {key}: {cached.steps} candidates, "
              f"{len(cached.accepted_positions)} accepts, {cached.launches} batches")
        assert cached.accepted_positions == full.accepted_positions, key
        assert cached.accepted_psnr == full.accepted_psnr, key            # bit for bit
        assert cached.initial_psnr == full.initial_psnr and cached.final_psnr == full.final_psnr, key
        assert cached.steps == full.steps and cached.stopped_early == full.stopped_early, key
        assert np.array_equal(m_full, m_cached), key
    assert len(full.accepted_positions) > 100


@pytest.mark.parametrize("k", [2, 4, 7])
def test_fft_walk_retention_equals_fresh_batches(golden_dir, monkeypatch, k):
    """(r06) the device walk keeps the candidates a batch propagated but did not visit (their job
    slot, B and -- untouched colour group -- partials) for the next batch.  The walk with that on
    and with it off (HBX_WALK_NO_RETAIN, every batch propagated from scratch) makes the same
    decisions with the same PSNR bits and leaves the same mask, at fixed speculation depths."""
    from hbx import dbs
    d, ocfg, pre, tgt, order = _fixture(golden_dir, "dbs_prefix_1024x24_16k.npz")
    runs = {}
    for retain in (True, False):
        if retain:
            monkeypatch.delenv("HBX_WALK_NO_RETAIN", raising=False)
        else:
            monkeypatch.setenv("HBX_WALK_NO_RETAIN", "1")
        plan, mask, target = _dev(ocfg, pre, tgt)
        res = dbs.greedy(plan, mask, target, order[:3000], mode="fft", k_min=k, k_max=k)
        runs[retain] = (res, mask.cpu().numpy())
        plan.close()
    (a, ma), (b, mb) = runs[True], runs[False]
    assert a.accepted_positions == b.accepted_positions
    assert a.accepted_psnr == b.accepted_psnr                       # bit for bit
    assert a.final_psnr == b.final_psnr and a.steps == b.steps and a.launches == b.launches
    assert np.array_equal(ma, mb)
    assert len(a.accepted_positions) > 100


def test_fft_walk_edge_orders(golden_dir):
    """The device-decided FFT-mode walk (hbx_dbs_walk_planes) on the orders that stress its batch
    logic, each against the host-decided full re-propagation (planes=False): an empty order, one
    candidate, fewer candidates than K, every position repeated (an accepted pixel comes back in
    the same batch: its group is touched, the batch must end there), runs of one colour group
    (at most one accept per batch), k_max 1 and 7, and an early stop.  Same accepts,
    same PSNR bits, same final mask."""
    from hbx import dbs
    d, ocfg, pre, tgt, order = _fixture(golden_dir, "dbs_prefix_1024x24_16k.npz")
    hw = 1024 * 1024
    base = [int(v) for v in order[:600]]
    same_group = [int(v) for v in order[:4000] if int(v) // (8 * hw) == 1][:200]
    cases = {
        "empty": ([], {}),
        "one": (base[:1], {}),
        "short": (base[:3], {"k_max": 8}),
        "repeated": ([v for v in base[:150] for _ in range(2)], {}),
        "one_group": (same_group, {}),
        "kmax1": (base[:300], {"k_max": 1}),
        "kmax7": (base[:300], {"k_max": 7}),
        "stop": (base, {"stop_diff": 1e-4}),
    }
    for name, (o, kw) in cases.items():
        o = np.asarray(o, np.int64)
        runs = []
        for planes, walk in ((False, False), (True, True)):
            plan, mask, target = _dev(ocfg, pre, tgt)
            res = dbs.greedy(plan, mask, target, o, mode="fft", planes=planes, device_walk=walk, **kw)
            runs.append((res, mask.cpu().numpy()))
            plan.close()
        (full, m_full), (walk, m_walk) = runs
        assert walk.accepted_positions == full.accepted_positions, name
        assert walk.accepted_psnr == full.accepted_psnr, name
        assert walk.steps == full.steps and walk.stopped_early == full.stopped_early, name
        assert np.array_equal(m_full, m_walk), name
        if name == "repeated":
            assert len(walk.accepted_positions) > 10
        if name == "stop":
            assert walk.stopped_early and walk.steps < len(o)


def test_fft_greedy_many_equals_single_walks(golden_dir):
    """dbs.greedy_many(mode="fft"): several images' FFT-mode walks side by side (one plan and
    stream each) give every image exactly its greedy(mode="fft") result -- accepts, PSNR bits,
    final mask -- including an empty order and an early stop."""
    from hbx import dbs
    d, ocfg, pre, tgt, order = _fixture(golden_dir, "dbs_prefix_1024x24_16k.npz")
    rng = np.random.default_rng(5)
    imgs = [(pre, tgt, order[:2500])]
    for i in range(2):
        imgs.append((rng.random(pre.shape).astype(pre.dtype), rng.random(tgt.shape).astype(tgt.dtype),
                     rng.permutation(order)[:2000 + 300 * i]))
    imgs.append((pre, tgt, order[:0]))
    for stop in (None, 2e-4):
        single = []
        for p_, t_, o_ in imgs:
            plan, mask, target = _dev(ocfg, p_, t_, max_jobs=16)
            single.append((dbs.greedy(plan, mask, target, o_, mode="fft", stop_diff=stop), mask.cpu().numpy()))
            plan.close()
        devs = [_dev(ocfg, p_, t_, max_jobs=16) for p_, t_, _ in imgs]
        many = dbs.greedy_many([x[0] for x in devs], [x[1] for x in devs], [x[2] for x in devs],
                               [o_ for _, _, o_ in imgs], stop_diff=stop, mode="fft")
        for (want, wm), got, (plan, gm, _) in zip(single, many, devs):
            assert got.accepted_positions == want.accepted_positions, stop
            assert got.accepted_psnr == want.accepted_psnr, stop
            assert got.steps == want.steps and got.stopped_early == want.stopped_early, stop
            assert np.array_equal(gm.cpu().numpy(), wm), stop
            plan.close()
        assert sum(len(r.accepted_positions) for r in many) > 100


def test_candidate_change_precision_1024x24(golden_dir):
    """Each candidate's PSNR change against the initial state, accepted or not
    (probe sweep / speculative batches): incremental path within INCR_TOL_DB,
    FFT path within FFT_TOL_DB, the all-flip map within 1e-10 dB."""
    d, ocfg, pre, tgt, order = _fixture(golden_dir, "dbs_prefix_1024x24.npz")
    want = d["probe_delta"]
    k = len(want)
    plan, mask, target = _dev(ocfg, pre, tgt)
    flips = torch.from_numpy(order[:k]).cuda()
    _, stats, p0 = plan.propagate(mask.unsqueeze(0), target.unsqueeze(0), want_intensity=False)
    base_stats = stats[0].contiguous()
    fc, it = plan.simulate(mask.unsqueeze(0), want_intensity=True)
    field = torch.view_as_real(fc[0]).contiguous()
    ps_psf, _ = plan.eval_flips_psf(mask, target, base_stats, field, it[0].contiguous(), flips)
    ps_fft, _ = plan.eval_flips(mask, target, base_stats, flips)
    dmap, base = plan.flip_map(mask, target)
    base0 = float(p0.item())
    e_psf = np.abs(ps_psf.cpu().numpy() - base0 - want)
    e_fft = np.abs(ps_fft.cpu().numpy() - base0 - want)
    e_map = np.abs(dmap.reshape(-1)[flips].double().cpu().numpy() - want)
    print(f"per-candidate |change - oracle| max: incremental {e_psf.max():.2e}, fft {e_fft.max():.2e}, "
          f"map {e_map.max():.2e} dB (median |change| {np.median(np.abs(want)):.2e})")
    assert e_psf.max() <= INCR_TOL_DB
    assert e_fft.max() <= FFT_TOL_DB
    assert e_map.max() <= 1e-10
    # decisions against the fixed base: signs equal wherever the change is resolved
    assert np.array_equal(ps_psf.cpu().numpy() > base0, want > 0)
    plan.close()


@pytest.mark.parametrize("mode", ["psf", "fft"])
def test_dbs_ratio05_256_literal_run(golden_dir, mode):
    """BASELINE configs[4] / DBS_ratio_0.5.py: 256x256x8 mono greedy DBS until
    the PSNR has risen 0.5 dB (:366-372).  Same accept sequence, same stopping
    candidate, same final PSNR as the float64 oracle."""
    from hbx import dbs
    d, ocfg, pre, tgt, order = _fixture(golden_dir, "dbs_ratio05_256.npz")
    n = int(d["n"])
    plan, mask, target = _dev(ocfg, pre, tgt)
    res = dbs.greedy(plan, mask, target, order, stop_diff=0.5, mode=mode)
    first = _first_difference(res.accepted_positions, d["accepted"])
    if mode == "psf":
        assert first is None, (first, float(d["delta"][first]))
        assert res.steps == n and res.stopped_early
    elif first is not None:
        assert abs(float(d["delta"][first])) <= FFT_TOL_DB, (first, float(d["delta"][first]))
    if first is None:
        assert res.steps == n and res.stopped_early
        # Gain error bound, derived.  The gain is final - initial PSNR, each
        # an ABSOLUTE PSNR of a state: the initial one from an f32 propagation, the final one
        # (FFT mode) from the last accepted candidate's f32 re-propagation, or (walk) from the
        # last exact f32 refresh plus the f64-summed increments of the accepts since.  So
        #   |gain error| <= 2 E_abs  (+ accepts since the last refresh x INCR_TOL_DB, walk)
        # with E_abs the f32 resolution of an absolute 256x256x8 PSNR, measured here on 16
        # random states against the float64 oracle (max error x 1.5).
        e_abs = 1.5 * _abs_psnr_resolution(plan, ocfg, tgt, 16)
        n_acc = len(res.accepted_positions)
        since = n_acc % 4096 if mode == "psf" else 0      # greedy's refresh_every default
        bound = 2.0 * e_abs + since * INCR_TOL_DB
        gerr = abs((res.final_psnr - res.initial_psnr) - (float(d["final_psnr"]) - float(d["initial_psnr"])))
        print(f"ratio05 {mode}: {res.steps} candidates, {n_acc} accepts, gain error {gerr:.2e} dB, "
              f"E_abs {e_abs:.2e} dB, derived bound {bound:.2e} dB")
        assert gerr <= bound
    assert abs(res.final_psnr - float(d["final_psnr"])) <= 1e-4
    plan.close()


def test_bf16_intermediates_deviation_256(golden_dir):
    """hbx_plan_set_precision (SURVEY 8d cfg 5, fp32 vs bf16 sweep): the
    bf16-rounded intermediates change the PSNR by far more than the f32
    product path does (DESIGN 4g measured 1.1e-4 dB at the +0.5 dB stop); the
    f32 plan is untouched by the option."""
    import hbx
    from hbx import dbs
    d, ocfg, pre, tgt, order = _fixture(golden_dir, "dbs_ratio05_256.npz")
    plan, mask, target = _dev(ocfg, pre, tgt, precision=hbx.PRECISION_BF16_STORE)
    assert plan.precision == hbx.PRECISION_BF16_STORE
    _, _, p_bf = plan.propagate(mask.unsqueeze(0), target.unsqueeze(0), want_intensity=False)
    plan.precision = hbx.PRECISION_F32
    _, _, p_32 = plan.propagate(mask.unsqueeze(0), target.unsqueeze(0), want_intensity=False)
    e32 = abs(float(p_32.item()) - float(d["initial_psnr"]))
    ebf = abs(float(p_bf.item()) - float(d["initial_psnr"]))
    print(f"initial PSNR error: f32 {e32:.2e} dB, bf16 intermediates {ebf:.2e} dB")
    assert e32 <= 1e-6 and ebf > e32 and ebf <= 5e-2
    plan.precision = hbx.PRECISION_BF16_STORE
    res = dbs.greedy(plan, mask, target, order, stop_diff=0.5, mode="fft")
    assert res.stopped_early
    dev_final = abs(res.final_psnr - float(d["final_psnr"]))
    print(f"bf16 run: {res.steps} candidates to +0.5 dB (oracle {int(d['n'])}), final PSNR error {dev_final:.2e} dB")
    assert dev_final <= 5e-2
    plan.close()


def test_split_walk_batches_equal_oracle(golden_dir, monkeypatch):
    """The ABI v5 three-launch batches (HBX_WALK_SPLIT=1 at plan creation) still give the
    oracle's accept sequence -- the fused one-launch step is the default."""
    from hbx import dbs
    monkeypatch.setenv("HBX_WALK_SPLIT", "1")
    d, ocfg, pre, tgt, order = _fixture(golden_dir, "dbs_prefix_1024x24.npz")
    n = 2048
    plan, mask, target = _dev(ocfg, pre, tgt)
    res = dbs.greedy(plan, mask, target, order[:n], mode="psf")
    assert _first_difference(res.accepted_positions, d["accepted"][:n]) is None
    assert _gain_error(res, d, n) <= GAIN_TOL_DB
    plan.close()


@pytest.mark.parametrize("refresh", [4096, 256])
def test_walk_mixed_k_fused_and_split_equal_oracle(golden_dir, monkeypatch, refresh):
    """The speculation depth changes between chunks (walk_k follows the acceptance
    rate): fused one-launch steps (K <= 4, commits applied by the NEXT launch) and
    split three-launch batches (K > 4, commit inside the batch) interleave in one walk.
    Cycling K through both kinds every chunk still gives the oracle's accept
    sequence and mask -- no pending commit lost or applied twice at a switch."""
    from hbx import dbs
    ks = [3, 8, 1, 32, 2, 4, 5, 2]
    it = iter(range(10 ** 6))
    monkeypatch.setattr(dbs, "walk_k", lambda *a, **k: ks[next(it) % len(ks)])
    d, ocfg, pre, tgt, order = _fixture(golden_dir, "dbs_prefix_1024x24.npz")
    n = 4096
    plan, mask, target = _dev(ocfg, pre, tgt)
    res = dbs.greedy(plan, mask, target, order[:n], mode="psf", refresh_every=refresh)
    first = _first_difference(res.accepted_positions, d["accepted"][:n])
    assert first is None, (first, float(d["delta"][first]))
    assert res.steps == n
    assert _gain_error(res, d, n) <= GAIN_TOL_DB
    want = (pre >= 0.5).astype(np.uint8)
    c, r, col = O.decode_action(order[:n][d["accepted"][:n]], ocfg.height, ocfg.width)
    np.bitwise_xor.at(want, (c, r, col), 1)
    assert np.array_equal(mask.cpu().numpy().view("<u8"), O.pack_mask(want))
    plan.close()


@pytest.mark.parametrize("mode", ["psf", "fft"])
def test_env_step_1024x24_trace_vs_oracle(golden_dir, mode):
    """BASELINE configs[2]'s env step at the headline size over 2,000 seeded random actions
    (env_trace_1024x24.npz: the float64 oracle with the env's rule -- roll back iff the PSNR
    change is negative, reward 800 * change either way, env.py:184-214).  The incremental
    mode makes every decision the oracle's and resolves each change within INCR_TOL_DB; the
    FFT mode (the reference's algorithm) within ENV_FFT_TOL_DB, its decisions the oracle's
    until the first step whose change lies inside that bound (measured: all 2,000 steps and
    1,010 accepts equal in both modes, max change error 1.4e-12 / 2.5e-9 dB)."""
    import hbx
    from hbx.env import HologramVecEnv
    d = np.load(os.path.join(golden_dir, "env_trace_1024x24.npz"), allow_pickle=False)
    n_px = int(d["size"])
    ocfg = O.OpticsConfig(n_px, n_px, int(d["groups"]), int(d["planes"]), O.WL_RGB, field_kind=int(d["field_kind"]))
    pre, tgt = O.synthetic_inputs(ocfg, int(d["seed"]))
    cfg = hbx.OpticsConfig(n_px, n_px, ocfg.groups, ocfg.planes, tuple(ocfg.wavelengths), field_kind=ocfg.field_kind)
    pre_t, tgt_t = torch.from_numpy(pre).cuda(), torch.from_numpy(tgt).cuda()
    env = HologramVecEnv(cfg, 1, lambda i: tgt_t, pre_model_source=lambda i: pre_t, obs_keys=(),
                         auto_reset=False, mode=mode)
    env.reset()
    init = float(env.state.init_psnr[0])
    assert abs(init - float(d["initial_psnr"])) <= 1e-4
    acts = torch.from_numpy(d["actions"]).cuda()
    rs, pss, accs = [], [], []
    for i in range(len(acts)):
        r, ps, acc, term, trunc = env.step_device(acts[i:i + 1])
        rs.append(r.clone()); pss.append(ps.clone()); accs.append(acc.clone())
    r = torch.cat(rs).cpu().numpy()
    ps = torch.cat(pss).cpu().numpy()
    acc = torch.cat(accs).cpu().numpy().astype(bool)
    want_acc, want_ps, want_delta = d["accepted"], d["psnr"], d["delta"]
    diff = np.nonzero(acc != want_acc)[0]
    upto = len(acc) if len(diff) == 0 else int(diff[0])
    tol = INCR_TOL_DB if mode == "psf" else ENV_FFT_TOL_DB
    if mode == "psf":
        assert upto == len(acc), (upto, float(want_delta[upto]))
    elif upto < len(acc):
        assert abs(float(want_delta[upto])) <= tol, (upto, float(want_delta[upto]))
    # the change of every step against the previous accepted state, up to the first divergence
    prev, change = init, np.empty(upto)
    for i in range(upto):
        change[i] = ps[i] - prev
        if acc[i]:
            prev = ps[i]
    err = np.abs(change - want_delta[:upto])
    print(f"env trace {mode}: {int(acc[:upto].sum())} accepts in {upto} steps, max |change - oracle| "
          f"{err.max():.2e} dB, max |psnr - oracle| {np.abs(ps[:upto] - want_ps[:upto]).max():.2e} dB")
    assert err.max() <= tol
    assert np.abs(r[:upto] - O.RW * want_delta[:upto]).max() <= O.RW * tol
    assert np.abs(ps[:upto] - want_ps[:upto]).max() <= 1e-4
    assert upto >= 1000
    env.close()
