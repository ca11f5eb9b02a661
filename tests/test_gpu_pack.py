"""hbx_pack_mask / hbx_rel_stats (ABI v14) on the GPU against the oracle.

The mask -> bits conversion the reference does per call (env.py:120 `pre_model >= 0.5`;
env.py:123,170-171 and DBS_1024_24.py:326-327 feed tt.simulate a float / int8 mask) is one HIP
launch here; these tests pin its bits to O.pack_mask (bit-exact, every input kind, word counts
that are not a multiple of the kernel's 4-word group, the threshold edge 0.5 and NaN), its
asynchronous binary check (the error word), and the fused tt.relativeLoss(.., tm.get_PSNR)
reduction against the oracle's float64 statistics.  The shim's error behaviour: a non-binary
mask raises ValueError in the relativeLoss that consumes it, at the next tt.simulate, at
check_binary(), or at once with strict=True."""
import numpy as np
import pytest
import torch

from oracle import hbx_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")


def _err_row():
    from hbx import _lib
    from hbx.env import HostRow
    row = HostRow(_lib.load(), 64)
    return row, row.array[:4].view(np.int32)


def _words(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view("<u8")


@pytest.mark.parametrize("dtype", [torch.bool, torch.int8, torch.uint8, torch.float32, torch.float64])
@pytest.mark.parametrize("shape", [(1, 64), (3, 5, 64), (2, 7, 192), (2, 24, 256, 256)])
def test_pack_binary_matches_oracle(dtype, shape):
    import hbx
    rng = np.random.default_rng(sum(shape))
    m = (rng.random(shape) < 0.5).astype(np.uint8)
    t = torch.from_numpy(m).to("cuda", dtype)
    row, err = _err_row()
    got = hbx.pack_mask(t, error_ptr=row.device)
    torch.cuda.synchronize()
    assert got.shape == (*shape[:-1], shape[-1] // 64) and got.dtype == torch.int64
    assert np.array_equal(_words(got), O.pack_mask(m))
    assert err[0] == 0
    assert np.array_equal(_words(hbx.pack_bits(t)), O.pack_mask(m))   # pack_bits routes here on the GPU
    row.close()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_pack_threshold_matches_numpy(dtype):
    """env.py:120 `state = (pre_model >= 0.5)`: exact 0.5 is on, NaN is off (torch's >=)."""
    import hbx
    rng = np.random.default_rng(7)
    pre = rng.random((24, 128, 128)).astype(np.float64 if dtype == torch.float64 else np.float32)
    pre.reshape(-1)[::97] = 0.5
    pre.reshape(-1)[5::131] = np.nextafter(pre.dtype.type(0.5), pre.dtype.type(0))
    pre.reshape(-1)[11::211] = np.nan
    got = hbx.pack_mask(torch.from_numpy(pre).cuda(), threshold=0.5)
    assert np.array_equal(_words(got), O.pack_mask((pre >= 0.5).astype(np.uint8)))


def test_pack_into_env_slice_and_misaligned_view():
    """out= an env's mask row (what reset does); a view whose start is not 16-byte aligned
    is copied first, with the same bits."""
    import hbx
    rng = np.random.default_rng(3)
    pre = rng.random((2, 8, 64, 64)).astype(np.float32)
    dev = torch.from_numpy(pre).cuda()
    out = torch.zeros((2, 8, 64, 1), dtype=torch.int64, device="cuda")
    hbx.pack_mask(dev[1], threshold=0.5, out=out[1])
    want = O.pack_mask((pre >= 0.5).astype(np.uint8))
    assert np.array_equal(_words(out[1]), want[1]) and not out[0].any()
    flat = torch.from_numpy(np.concatenate([[0.0], pre.reshape(-1)]).astype(np.float32)).cuda()
    view = flat[1:].reshape(pre.shape)                  # 4 bytes off the allocation's alignment
    assert view.data_ptr() % 16 != 0
    assert np.array_equal(_words(hbx.pack_mask(view, threshold=0.5)), want)
    with pytest.raises(ValueError):
        hbx.pack_mask(torch.zeros((4, 100), device="cuda"))


@pytest.mark.parametrize("dtype,bad", [(torch.float32, 0.5), (torch.float32, float("nan")), (torch.float32, 2.0),
                                       (torch.float64, -1.0), (torch.int8, -1), (torch.uint8, 2)])
def test_pack_error_word(dtype, bad):
    """A value other than 0 / 1 anywhere (here the last word of a ragged 15-word input) sets the
    word; -0.0 is a valid 0."""
    import hbx
    row, err = _err_row()
    m = np.zeros((3, 5, 64), np.float64)
    m[0, 0, 3] = 1.0
    m[1, 2, 7] = -0.0
    t = torch.from_numpy(m).to("cuda", dtype)
    hbx.pack_mask(t, error_ptr=row.device)
    torch.cuda.synchronize()
    assert err[0] == 0
    t[2, 4, 63] = bad
    got = hbx.pack_mask(t, error_ptr=row.device)
    torch.cuda.synchronize()
    assert err[0] == 1
    assert _words(got)[0, 0, 0] == 1 << 3
    row.close()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("shape", [(1, 1, 256, 256), (1, 3, 1024, 1024), (1, 1, 3, 5)])
def test_rel_stats_matches_oracle(dtype, shape):
    """tt.relativeLoss(x, y, tm.get_PSNR) as one f64 reduction: the statistics to 1e-12
    relative, the PSNR to 1e-9 dB of the oracle's direct form (float64 numpy)."""
    from hbx import _lib
    from hbx.env import HostRow
    rng = np.random.default_rng(11)
    x = (rng.random(shape) * 3).astype(np.float32 if dtype == torch.float32 else np.float64)
    y = rng.random(shape).astype(x.dtype)
    lib = _lib.load()
    row = HostRow(lib, 64)
    out = row.array[:40].view(np.float64)
    work = torch.empty(_lib.REL_WORKSPACE_DOUBLES, dtype=torch.float64, device="cuda")
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    res = []
    for _ in range(2):
        _lib.check(lib.hbx_rel_stats(xd.data_ptr(), yd.data_ptr(), _lib.SRC_F32 if dtype == torch.float32
                                     else _lib.SRC_F64, x.size, _lib.REL_LSQ, 1.0, work.data_ptr(), row.device,
                                     torch.cuda.current_stream().cuda_stream), "hbx_rel_stats")
        torch.cuda.synchronize()
        res.append(out.copy())
    assert np.array_equal(res[0], res[1])                 # fixed-order reduction: same bits
    x64, y64 = x.astype(np.float64), y.astype(np.float64)
    want = np.array([np.sum(x64 * y64), np.sum(x64 * x64), np.sum(y64 * y64)])
    assert np.allclose(res[0][:3], want, rtol=1e-12, atol=0)
    assert res[0][3] == pytest.approx(O.relative_psnr(x, y), abs=1e-9)
    assert res[0][4] == pytest.approx(O.relative_mse(x, y), rel=1e-9)
    row.close()


def test_shim_relative_loss_fast_path_equals_torch_path():
    import torchOptics.metrics as tm
    import torchOptics.optics as tt
    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.random((1, 1, 256, 256)).astype(np.float32)).cuda()
    y = torch.from_numpy(rng.random((1, 1, 256, 256)).astype(np.float32)).cuda()
    fast = tt.relativeLoss(x, y, tm.get_PSNR)
    generic = tt.relativeLoss(x, y, lambda a, b: tm.get_PSNR(a, b))   # not get_PSNR itself: torch ops
    assert isinstance(fast, float) and fast == pytest.approx(generic, abs=1e-9)
    assert fast == pytest.approx(O.relative_psnr(x.cpu().numpy(), y.cpu().numpy()), abs=1e-9)


def test_shim_binary_check_raises_without_a_sync_in_simulate():
    """The DBS.py:259-270 chain with a non-binary mask: ValueError in the relativeLoss that
    consumes it; the next good call runs; strict=True and check_binary() raise at once."""
    import torchOptics.metrics as tm
    import torchOptics.optics as tt
    meta = {"dx": (7.56e-6, 7.56e-6), "wl": 515e-9}
    rng = np.random.default_rng(9)
    good = (rng.random((1, 8, 64, 64)) > 0.5).astype(np.float32)
    bad = good.copy()
    bad[0, 3, 10, 20] = 0.5
    tgt = torch.from_numpy(rng.random((1, 1, 64, 64)).astype(np.float32)).cuda()

    def psnr(m):
        sim = tt.simulate(tt.Tensor(torch.from_numpy(m).cuda(), meta=meta), 2e-3).abs() ** 2
        return tt.relativeLoss(torch.mean(sim, dim=1, keepdim=True), tgt, tm.get_PSNR)

    p0 = psnr(good)
    with pytest.raises(ValueError, match="binary"):
        psnr(bad)
    assert psnr(good) == p0                      # the word was cleared; same bits as before
    tt.simulate(tt.Tensor(torch.from_numpy(bad).cuda(), meta=meta), 2e-3)
    with pytest.raises(ValueError, match="binary"):
        tt.check_binary()
    with pytest.raises(ValueError, match="binary"):
        tt.simulate(tt.Tensor(torch.from_numpy(bad).cuda(), meta=meta), 2e-3, strict=True)
    tt.simulate(tt.Tensor(torch.from_numpy(bad).cuda(), meta=meta), 2e-3)
    torch.cuda.synchronize()
    with pytest.raises(ValueError, match="binary"):   # an earlier call's input, seen at the next call
        tt.simulate(tt.Tensor(torch.from_numpy(good).cuda(), meta=meta), 2e-3)
    tt.check_binary()                            # nothing pending


def test_pack_threshold_full_headline_size():
    """configs[2]'s reset input at full size (24 x 1024 x 1024 f32 per env, 4 envs): pack then
    unpack equals `pre >= 0.5` bit for bit (a size-independent round trip, on the device)."""
    import hbx
    g = torch.Generator(device="cuda").manual_seed(17)
    pre = torch.rand((4, 24, 1024, 1024), generator=g, device="cuda")
    bits = hbx.pack_mask(pre, threshold=0.5)
    assert bits.shape == (4, 24, 1024, 16)
    assert torch.equal(hbx.unpack_bits(bits, 1024), (pre >= 0.5).to(torch.int8))
