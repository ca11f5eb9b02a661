"""Host-side logic without a GPU: bit packing, spaces, DBS speculation
bookkeeping, pre-model binning -- each checked against the oracle."""
import os
import numpy as np
import pytest
import torch

from oracle import hbx_oracle as O


def test_pack_bits_torch_matches_oracle():
    from hbx.plan import pack_bits, unpack_bits
    m = (np.random.default_rng(0).random((2, 3, 128)) > 0.5).astype(np.uint8)
    got = pack_bits(torch.from_numpy(m)).numpy().view("<u8")
    assert np.array_equal(got, O.pack_mask(m))
    assert np.array_equal(unpack_bits(torch.from_numpy(got.view(np.int64)), 128).numpy(), m)


def test_pack_bits_bit63():
    from hbx.plan import pack_bits
    m = torch.zeros(1, 64, dtype=torch.uint8)
    m[0, 63] = 1
    assert pack_bits(m).numpy().view("<u8")[0] == np.uint64(1 << 63)


def test_pack_bits_rejects_ragged_width():
    from hbx.plan import pack_bits
    with pytest.raises(ValueError):
        pack_bits(torch.zeros(4, 100))


def test_spaces_surface():
    from hbx import spaces
    d = spaces.Discrete(8 * 256 * 256)
    assert d.n == 524288 and d.contains(524287) and not d.contains(524288)
    b = spaces.Box(0, 1, (1, 8, 4, 4), np.int8)
    assert b.sample().shape == (1, 8, 4, 4)
    md = spaces.MultiDiscrete([8, 256, 256])
    s = md.sample()
    assert md.contains(s)


def test_first_improving_is_strict():
    from hbx.dbs import first_improving
    assert first_improving(np.array([1.0, 2.0, 2.5]), 2.0) == 2
    assert first_improving(np.array([1.0, 2.0]), 2.0) is None
    assert first_improving(np.array([3.0]), 2.0) == 0


def test_speculative_walk_equals_serial():
    """The speculative batching rule reproduces the serial accept sequence on any
    deterministic evaluator (here a toy 'psnr' = running sum of per-index gains)."""
    from hbx.dbs import KController, first_improving
    rng = np.random.default_rng(1)
    gains = rng.normal(size=2000)
    # serial
    prev, acc_serial = 0.0, []
    for i, g in enumerate(gains):
        if prev + g > prev:
            prev += g
            acc_serial.append(i)
    # speculative, evaluating candidates against the base
    prev, acc, pos, ctl = 0.0, [], 0, KController(k_min=2, k_max=64, k0=8)
    while pos < len(gains):
        k = min(ctl.k, len(gains) - pos)
        ps = prev + gains[pos:pos + k]
        i = first_improving(ps, prev)
        ctl.update(i)
        if i is None:
            pos += k
            continue
        prev = ps[i]
        acc.append(pos + i)
        pos += i + 1
    assert acc == acc_serial


def test_premodel_bins_match_oracle():
    from hbx.dbs import premodel_bins
    vals = np.concatenate([np.linspace(-0.1, 1.1, 241), np.round(np.linspace(0, 1, 11), 10)])
    got = premodel_bins(vals)
    want = np.array([O.premodel_bin(float(v)) for v in vals])
    assert np.array_equal(got, want)


def test_shard_range_covers_everything():
    from hbx.dist import shard_range
    for total in (0, 1, 7, 128, 1024, 1025):
        for world in (1, 2, 3, 8):
            parts = [shard_range(total, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def test_optics_config_to_c():
    from hbx.plan import rgb_config
    c = rgb_config(1024).to_c()
    assert (c.height, c.groups, c.planes) == (1024, 3, 8)
    assert abs(c.wavelength[2] - 450e-9) < 1e-18 and c.z == 2e-3
    with pytest.raises(ValueError):
        from hbx.plan import OpticsConfig
        OpticsConfig(64, 64, 2, 2, (515e-9,)).to_c()


def test_plan_requires_gpu():
    import hbx
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        hbx.Plan(hbx.mono_config(64))


def test_greedy_report_formats():
    """hbx.dbs.greedy_report prints the DBS_1024_24.py console lines that the
    log_py parsers (DBS_psnr_log.py step blocks, com.py range lines) read."""
    import re
    from hbx.dbs import GreedyResult, greedy_report
    H = W = 8
    rng = np.random.default_rng(0)
    pre = rng.random((2, H, W)).astype(np.float32)
    order = rng.permutation(2 * H * W)
    res = GreedyResult(initial_psnr=10.0, final_psnr=10.35, steps=40,
                       accepted_positions=[2, 9, 17, 30], accepted_psnr=[10.05, 10.12, 10.25, 10.35],
                       launches=7, accept_times=[0.1, 0.2, 0.3, 0.4], last_psnr=10.3, seconds=0.5)
    txt = greedy_report(res, order, pre, H, W, file_name="0801")
    step_re = re.compile(r"Step: (\d+)\s+PSNR Before: [\d.]+\s+\|\s+PSNR After: [\d.]+\s+\|\s+Change: "
                         r"[\d.e+-]+\s+\|\s+Diff: ([\d.e+-]+)\s+Success Ratio: ([\d.e+-]+)\s+\|\s+"
                         r"Flip Count: (\d+).*?Time taken for this data: ([\d.]+) seconds", re.DOTALL)
    steps = [(int(m.group(1)), float(m.group(2)), int(m.group(4))) for m in step_re.finditer(txt)]
    # thresholds +0.1 (crossed at the 10.12 accept) and +0.2 / +0.3 (10.25 / 10.35)
    assert steps == [(10, 0.12, 2), (18, 0.25, 3), (31, 0.35, 4)]
    range_re = re.compile(r"Range (\d\.\d-\d\.\d): Total Pixels = (\d+), Improved Pixels = (\d+), "
                          r"Improvement Ratio \(in range\) = ([\d\.]+), Improvement Ratio \(to total "
                          r"improved\) = ([\d\.]+), Total PSNR Improvement = ([\d\.]+), Average PSNR "
                          r"Improvement = ([\d\.]+)")
    final = txt.split("Pre-model output range statistics:")[1]
    rows = range_re.findall(final)
    assert len(rows) == 10
    base = np.histogram(pre, bins=np.linspace(0, 1, 11))[0]
    assert sum(int(r[2]) for r in rows) == 4                       # every accept binned once
    assert sum(int(r[1]) for r in rows) == int(base.sum()) + 4     # whole pre-model + accepts
    assert abs(sum(float(r[5]) for r in rows) - 0.35) < 1e-5
    assert "0801.png Optimization completed. Final PSNR improvement: 0.300000" in txt


def test_binarynet_reference_layout_and_checkpoint(tmp_path):
    """BinaryNet keeps the reference's module names (checkpoint compatibility,
    DBS_1024_24.py:48-164) and loads a state_dict with weights_only=True."""
    import torch
    from hbx.premodel import BinaryNet, load_premodel, reference_premodel
    m = reference_premodel(num_hologram=24, in_planes=3)
    names = {k.rsplit(".", 2)[0] for k in m.state_dict()}
    want = {f"enc{l}_{i}" for l in range(1, 6) for i in (1, 2)} | {f"pool{l}" for l in range(1, 5)} \
        | {f"dec{l}_{i}" for l in range(1, 5) for i in (1, 2)} | {f"deconv{l}" for l in range(1, 5)} | {"classifier"}
    assert names == want
    assert all(k.endswith((".0.weight", ".0.bias")) for k in m.state_dict())   # conv only, no act / BN
    full = BinaryNet(num_hologram=8, in_planes=1)
    assert "enc1_1.2.running_mean" in full.state_dict() and "deconv1.1.weight" in full.state_dict()
    x = torch.rand(1, 3, 32, 32)
    y = m(x)
    assert y.shape == (1, 24, 32, 32) and float(y.min()) >= 0 and float(y.max()) <= 1
    p = tmp_path / "pre.pth"
    torch.save({"model": m.state_dict()}, p)
    m2 = load_premodel(str(p), num_hologram=24)
    assert torch.equal(m2(x), y)


def test_target_folder(tmp_path):
    from PIL import Image
    from hbx.premodel import TargetFolder
    rng = np.random.default_rng(0)
    for name, (h, w) in (("b.png", (40, 60)), ("a.png", (24, 30))):
        Image.fromarray((rng.random((h, w, 3)) * 255).astype(np.uint8)).save(tmp_path / name)
    ds = TargetFolder(str(tmp_path), ips=32, train=False, padding=2)
    assert [os.path.basename(p) for p in ds.target_list] == ["a.png", "b.png"]
    t, path = ds[1]
    assert t.shape == (1, 3, 36, 36) and path.endswith("b.png")
    src = np.asarray(Image.open(tmp_path / "b.png"), np.float32) / 255.0
    assert np.allclose(t[0, :, 2:-2, 2:-2].numpy(), np.transpose(src[4:36, 14:46], (2, 0, 1)))
    t2, _ = ds[0]                                   # 24x30 -> shorter side resized to 32
    assert t2.shape == (1, 3, 36, 36)
    tr = TargetFolder(str(tmp_path), ips=32, train=True, seed=3)
    assert tr[1][0].shape == (1, 3, 32, 32)
    a, imgname = next(iter(ds))                      # DataLoader(batch_size=1) shape of a batch
    assert a.shape == (1, 3, 36, 36) and isinstance(imgname, list) and imgname[0].endswith("a.png")


def test_crop_bits_matches_oracle_crop():
    """Packed 64-pixel crop (env_1024_24_128.py:144-149) == crop then pack."""
    from hbx.plan import crop, crop_bits, pack_bits
    m = (np.random.default_rng(4).random((2, 256, 256)) > 0.5).astype(np.uint8)
    got = crop_bits(pack_bits(torch.from_numpy(m)), 64).numpy().view("<u8")
    assert np.array_equal(got, O.pack_mask(O.crop(m, 64)))
    assert np.array_equal(crop(torch.from_numpy(m), 64).numpy(), O.crop(m, 64))
    with pytest.raises(ValueError):
        crop_bits(pack_bits(torch.from_numpy(m)), 32)


def test_crop_config():
    import hbx
    c = hbx.crop_config(hbx.rgb_config(1024), 64)
    assert (c.height, c.width, c.groups, c.planes) == (896, 896, 3, 8)


def test_walk_k_choice():
    """Device-walk speculation depth: short batches at high acceptance and
    large sides, long ones when acceptance is rare or candidates are cheap."""
    from hbx.dbs import walk_k
    assert walk_k(0.5, 1024) <= 4
    assert walk_k(0.01, 1024) > walk_k(0.5, 1024)
    assert walk_k(0.5, 64) > walk_k(0.5, 1024)
    assert walk_k(1e-9, 1024, 1, 256, fused=False) == 256
    assert walk_k(1e-9, 1024, 1, 256) == 256           # rare accepts: long split batches
    assert 1 <= walk_k(1.0, 1024) <= 2
    from hbx import _lib
    for q in (0.9, 0.5, 0.3):                          # frequent accepts: one-launch two-accept steps
        assert walk_k(q, 1024) in _lib.WALK_FUSED_K


def test_vecenv_mode_validation_before_any_device_work():
    """mode='planes' is built for N = 256 / 1024 only and graph replay applies to the FFT-type
    modes: both are decided from the arguments before a plan (or the GPU) is touched."""
    import pytest
    import hbx
    from hbx.env import HologramVecEnv
    src = lambda i: None  # noqa: E731  (never called: construction fails first)
    with pytest.raises(ValueError, match="planes"):
        HologramVecEnv(hbx.rgb_config(64), 2, src, pre_model_source=src, mode="planes")
    with pytest.raises(ValueError, match="mode must be"):
        HologramVecEnv(hbx.mono_config(256), 2, src, pre_model_source=src, mode="cached")


def test_env_buffers_struct_matches_header():
    """ctypes mirror of hbx_env_buffers_t (include/hbx.h, ABI v9): field order and offsets."""
    import ctypes as C
    import re
    from hbx import _lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "include", "hbx.h")).read()
    body = hdr[hdr.index("typedef struct hbx_env_buffers {"):hdr.index("} hbx_env_buffers_t;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = re.findall(r"\b(\w+);", body)
    assert [f[0] for f in _lib.EnvBuffers._fields_] == names
    assert C.sizeof(_lib.EnvBuffers) == 8 * (len(names) - 2) + 4 * 2   # two int32 fields


def test_walk_state_fault_plumbing():
    """A persistent walk whose grid barrier timed out leaves fault = done = 1 in the walk state
    (k_walk_abort_fold, after the grid has drained): the host reader raises on it and passes a
    clean state through unchanged (hbx.dbs.walk_state)."""
    import ctypes as C
    import pytest
    from hbx import _lib
    from hbx.dbs import walk_state
    w = _lib.DbsWalk()
    w.pos, w.accepted, w.done = 17, 5, 0
    st = walk_state(bytes(w))
    assert (st.pos, st.accepted, st.fault, st.done) == (17, 5, 0, 0)
    w.fault, w.done = 1, 1
    with pytest.raises(RuntimeError, match="barrier timed out"):
        walk_state(bytes(w))
    assert C.sizeof(_lib.DbsWalk) == len(bytes(w))


def test_dropin_env_rejects_unsupported_modes_before_device_work():
    """BinaryHologramEnv returns the stepped recon_image (env.py:179): the incremental mode
    (which has none) and a caller-chosen obs_keys are refused from the arguments alone."""
    import pytest
    from hbx.env import BinaryHologramEnv
    with pytest.raises(ValueError, match="recon_image"):
        BinaryHologramEnv(lambda t: t, [], mode="psf")
    with pytest.raises(ValueError, match="five observation keys"):
        BinaryHologramEnv(lambda t: t, [], obs_keys=("state",))
