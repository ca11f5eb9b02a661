"""torchOptics.optics -- drop-in for the operator API the reference imports as ``tt``.

The reference calls (env.py:124-132,170-174; env_1024_24.py:149-166;
DBS_1024_24.py:244-257,326-352; range.py:225-309):

    x = tt.Tensor(state_or_numpy, meta={'dx': (7.56e-6, 7.56e-6), 'wl': 515e-9})
    sim = tt.simulate(x, z).abs() ** 2            # complex field of every plane
    psnr = tt.relativeLoss(mean_intensity, target, tm.get_PSNR)
    mse = tt.relativeLoss(mean_intensity, target, F.mse_loss)

``simulate`` runs on the MI355X through libhbx.so (hbx_simulate: bit-packed
mask -> three HIP FFT passes with the transfer function fused in).  The
reference only ever propagates binary masks, and so does this shim: a
non-binary field raises ValueError (there is no CPU / float fallback).
The physics follows the assumptions documented in DESIGN.md (the original
torchOptics is absent and unpinned): exact angular spectrum, no padding,
amplitude field.  relativeLoss uses the least-squares scale s = sum(xy)/sum(x^2).
"""
from __future__ import annotations

from typing import Callable, Dict, Optional, Tuple

import numpy as np
import torch

import hbx
from hbx import _lib

__all__ = ["Tensor", "simulate", "relativeLoss", "imread"]


class Tensor(torch.Tensor):
    """A torch tensor with an optics ``meta`` dict ({'dx': (dx, dy), 'wl': wl}).

    Integer / numpy inputs (DBS_1024_24.py:326 passes an int8 numpy slice)
    become float32.  Results of torch ops on it are plain torch tensors."""

    @staticmethod
    def __new__(cls, data, meta: Optional[Dict] = None, **_):
        t = data if isinstance(data, torch.Tensor) else torch.as_tensor(np.asarray(data))
        if not (t.is_floating_point() or t.is_complex()):
            t = t.to(torch.float32)
        obj = t.as_subclass(cls)
        obj.meta = dict(meta or (getattr(data, "meta", None) or {}))
        return obj

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        with torch._C.DisableTorchFunctionSubclass():
            return func(*args, **(kwargs or {}))


_PLANS: Dict[Tuple, "hbx.Plan"] = {}


def _meta_of(x) -> Dict:
    meta = getattr(x, "meta", None)
    if not meta:
        raise ValueError("tt.simulate needs a tt.Tensor with meta={'dx': ..., 'wl': ...}")
    return meta


def _plan_for(h: int, w: int, planes: int, wl: float, dx: float, dy: float, z: float, n: int, dev: int):
    key = (h, w, planes, float(wl), float(dx), float(dy), float(z), dev)
    p = _PLANS.get(key)
    if p is None or p.max_jobs < n:
        cfg = hbx.OpticsConfig(h, w, 1, planes, (float(wl),), float(dx), float(dy), float(z),
                               _lib.TF_ASM, _lib.FIELD_AMPLITUDE, _lib.REL_LSQ, 1.0)
        p = hbx.Plan(cfg, max_jobs=max(n, 1), device=dev)
        _PLANS[key] = p
    return p


def simulate(x, z: float, **_) -> torch.Tensor:
    """Free-space propagation of a binary mask tensor [B, C, H, W] (or [C, H, W])
    by z metres: the complex field of every plane, complex64, on the GPU."""
    meta = _meta_of(x)
    wl = meta["wl"]
    if isinstance(wl, (tuple, list)):
        if len(wl) != 1:
            raise ValueError("simulate: one wavelength per call (the reference splits RGB groups, "
                             "env_1024_24.py:149-155)")
        wl = wl[0]
    dx, dy = meta.get("dx", (hbx.plan.PIXEL_PITCH,) * 2)
    t = x.as_subclass(torch.Tensor) if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))
    squeeze = t.dim() == 3
    if squeeze:
        t = t.unsqueeze(0)
    if t.dim() != 4:
        raise ValueError(f"simulate expects [B, C, H, W], got {tuple(t.shape)}")
    if not torch.cuda.is_available():
        raise RuntimeError("tt.simulate needs a ROCm GPU (libhbx.so)")
    dev = torch.cuda.current_device() if not t.is_cuda else t.device.index
    t = t.to(f"cuda:{dev}")
    if t.is_complex() or not bool(((t == 0) | (t == 1)).all()):
        raise ValueError("tt.simulate (hbx) propagates binary {0,1} masks only, as the reference does")
    b, c, h, w = t.shape
    cp = c + (c % 2)                                # the kernels pack plane pairs
    if cp != c:
        t = torch.cat([t, torch.zeros_like(t[:, :1])], dim=1)
    plan = _plan_for(h, w, cp, wl, dx, dy, z, b, dev)
    field, _ = plan.simulate(hbx.pack_bits(t))
    field = field[:, :c]
    return field[0] if squeeze else field


def relativeLoss(x: torch.Tensor, y, fn: Callable) -> torch.Tensor:
    """fn(s * x, y) with the least-squares scale s = sum(x y) / sum(x^2), all in
    float64: DBS_1024_24.py:355 compares two such PSNRs whose difference is
    ~1e-6 dB at 1024x24, below float32 resolution of the PSNR itself."""
    x = x.as_subclass(torch.Tensor) if isinstance(x, torch.Tensor) else torch.as_tensor(x)
    y = torch.as_tensor(np.asarray(y)) if not isinstance(y, torch.Tensor) else y.as_subclass(torch.Tensor)
    xd, yd = x.double(), y.to(x.device).double()
    s = torch.sum(xd * yd) / torch.sum(xd * xd)
    return fn(s * xd, yd)


def imread(path: str, meta: Optional[Dict] = None, gray: bool = False) -> Tensor:
    """Image file -> tt.Tensor [1, C, H, W] in [0, 1] (Dataset512's loader, DBS_1024_24.py:191)."""
    from PIL import Image
    img = Image.open(path)
    img = img.convert("L" if gray else "RGB")
    a = np.asarray(img, dtype=np.float32) / 255.0
    a = a[None, None] if gray else np.transpose(a, (2, 0, 1))[None]
    return Tensor(torch.from_numpy(np.ascontiguousarray(a)), meta=meta)
