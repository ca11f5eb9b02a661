"""torchOptics shim: the reference's `tt` / `tm` call
sites run unchanged.  CPU part: Tensor/meta plumbing and the loss / metric
arithmetic against the oracle.  GPU part: tt.simulate through libhbx.so
against the oracle's propagation, and the env.py reset/step expression
chain end to end."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import hbx_oracle as O


def test_tensor_meta_and_plain_results():
    import torchOptics.optics as tt
    x = tt.Tensor(np.ones((1, 2, 4, 4), np.int8), meta={"dx": (7.56e-6, 7.56e-6), "wl": 515e-9})
    assert x.dtype == torch.float32 and x.meta["wl"] == 515e-9
    y = x.abs() ** 2
    assert type(y) is torch.Tensor                    # ops return plain tensors
    assert torch.mean(y, dim=1, keepdim=True).shape == (1, 1, 4, 4)


def test_relative_loss_and_psnr_match_oracle():
    import torchOptics.metrics as tm
    import torchOptics.optics as tt
    rng = np.random.default_rng(0)
    x = rng.random((1, 3, 16, 16))
    y = rng.random((1, 3, 16, 16)).astype(np.float32)
    psnr = tt.relativeLoss(torch.from_numpy(x).float(), torch.from_numpy(y), tm.get_PSNR)
    assert psnr == pytest.approx(O.relative_psnr(x.astype(np.float32), y), abs=1e-5)
    mse = tt.relativeLoss(torch.from_numpy(x).float(), torch.from_numpy(y), F.mse_loss)
    assert float(mse) == pytest.approx(O.relative_mse(x.astype(np.float32), y), rel=1e-5)


def test_imread_roundtrip(tmp_path):
    from PIL import Image
    import torchOptics.optics as tt
    a = (np.random.default_rng(1).random((8, 8, 3)) * 255).astype(np.uint8)
    Image.fromarray(a).save(tmp_path / "x.png")
    t = tt.imread(str(tmp_path / "x.png"), meta={"wl": 515e-9})
    assert t.shape == (1, 3, 8, 8) and np.allclose(t.numpy()[0], np.transpose(a, (2, 0, 1)) / 255.0)


@pytest.mark.gpu
def test_simulate_matches_oracle():
    import torchOptics.optics as tt
    m = (np.random.default_rng(2).random((1, 8, 64, 64)) > 0.5).astype(np.int8)
    x = tt.Tensor(m, meta={"dx": (7.56e-6, 7.56e-6), "wl": 515e-9})
    u = tt.simulate(x, 2e-3)
    h = O.transfer_function(64, 64, 7.56e-6, 7.56e-6, 515e-9, 2e-3)
    want = O.propagate(m[0].astype(np.float64), h)
    got = u[0].cpu().numpy()
    assert u.dtype == torch.complex64 and u.shape == (1, 8, 64, 64)
    assert np.max(np.abs(got - want)) <= 2e-5 * np.max(np.abs(want))
    # odd plane count is padded internally
    u3 = tt.simulate(tt.Tensor(m[:, :3], meta=x.meta), 2e-3)
    assert np.max(np.abs(u3[0].cpu().numpy() - want[:3])) <= 2e-5 * np.max(np.abs(want))
    with pytest.raises(ValueError):
        tt.simulate(tt.Tensor(np.full((1, 2, 64, 64), 0.5, np.float32), meta=x.meta), 2e-3, strict=True)


@pytest.mark.gpu
def test_env_py_expression_chain_via_shim():
    """The literal env.py:123-132 expressions, evaluated through the shim."""
    import torchOptics.metrics as tm
    import torchOptics.optics as tt
    cfg = O.mono_config(256)
    pre, tgt = O.synthetic_inputs(cfg, 3)
    state = (pre[None] >= 0.5).astype(np.int8)                          # env.py:120
    target_image = torch.from_numpy(tgt[None]).cuda()
    binary = torch.tensor(state, dtype=torch.float32).cuda()            # env.py:123
    binary = tt.Tensor(binary, meta={'dx': (7.56e-6, 7.56e-6), 'wl': 515e-9})
    sim = tt.simulate(binary, 2e-3).abs() ** 2                          # env.py:127
    result = torch.mean(sim, dim=1, keepdim=True)                       # env.py:128
    psnr = tt.relativeLoss(result, target_image, tm.get_PSNR)           # env.py:132
    ref = O.Propagator(cfg)
    inten = ref.group_intensity(state[0], 0)
    assert psnr == pytest.approx(ref.psnr(O.chan_stats(inten, tgt[0])[None]), abs=1e-4)
