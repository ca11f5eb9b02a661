"""torchOptics.optics -- drop-in for the operator API the reference imports as ``tt``.

The reference calls (env.py:124-132,170-174; env_1024_24.py:149-166;
DBS_1024_24.py:244-257,326-352; range.py:225-309):

    x = tt.Tensor(state_or_numpy, meta={'dx': (7.56e-6, 7.56e-6), 'wl': 515e-9})
    sim = tt.simulate(x, z).abs() ** 2            # complex field of every plane
    psnr = tt.relativeLoss(mean_intensity, target, tm.get_PSNR)
    mse = tt.relativeLoss(mean_intensity, target, F.mse_loss)

``simulate`` runs on the MI355X through libhbx.so: one hbx_pack_mask launch turns the mask
into bits (ABI v14), then hbx_simulate's three HIP FFT passes with the transfer function fused
in.  The reference only ever propagates binary masks, and so does this shim: a non-binary
field raises ValueError (there is no CPU / float fallback).  The binary check is part of the
pack kernel and costs no host sync: the kernel flags a value other than 0 / 1 in host-mapped
memory, and the shim raises at the first point the host has waited for that work -- inside
the tt.relativeLoss(.., tm.get_PSNR) that consumes the result (it waits for its PSNR anyway,
env.py:174 / DBS.py:270 compare it at once), at the next tt.simulate, or at check_binary().
``simulate(x, z, strict=True)`` waits and raises before returning.
The physics follows the assumptions documented in DESIGN.md (the original
torchOptics is absent and unpinned): exact angular spectrum, no padding,
amplitude field.  relativeLoss uses the least-squares scale s = sum(xy)/sum(x^2); with
tm.get_PSNR on GPU tensors it is one fixed-order f64 reduction (hbx_rel_stats) whose PSNR
is read from host-mapped memory.
"""
from __future__ import annotations

from typing import Callable, Dict, Optional, Tuple

import numpy as np
import torch

import hbx
from hbx import _lib

from . import metrics as _metrics

__all__ = ["Tensor", "simulate", "relativeLoss", "imread", "check_binary"]


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


class _Scratch:
    """Per-device shim scratch: a host-mapped row (the pack kernel's binary-check word at
    byte 0, hbx_rel_stats' five doubles at byte 8) and the reduction's device workspace."""

    def __init__(self, dev: int):
        from hbx.env import HostRow
        self.row = HostRow(_lib.load(), 64)
        self.err = self.row.array[0:4].view(np.int32)
        self.out = self.row.array[8:48].view(np.float64)
        self.err_dev = self.row.device
        self.out_dev = self.row.device + 8
        self.work = torch.empty(_lib.REL_WORKSPACE_DOUBLES, dtype=torch.float64, device=f"cuda:{dev}")


_SCRATCH: Dict[int, _Scratch] = {}


def _scratch(dev: int) -> _Scratch:
    sc = _SCRATCH.get(dev)
    if sc is None:
        sc = _SCRATCH[dev] = _Scratch(dev)
    return sc


def _raise_pending(sc: _Scratch):
    if sc.err[0]:
        sc.err[0] = 0
        raise ValueError("tt.simulate (hbx) propagates binary {0,1} masks only, as the reference does: "
                         "a mask passed to tt.simulate held another value")


def check_binary(device: Optional[int] = None):
    """Wait for the device's queued work and raise ValueError if any tt.simulate input
    since the last check held a value other than 0 / 1."""
    dev = torch.cuda.current_device() if device is None else int(device)
    sc = _SCRATCH.get(dev)
    if sc is not None:
        torch.cuda.synchronize(dev)
        _raise_pending(sc)


def simulate(x, z: float, strict: bool = False, **_) -> torch.Tensor:
    """Free-space propagation of a binary mask tensor [B, C, H, W] (or [C, H, W])
    by z metres: the complex field of every plane, complex64, on the GPU.
    strict=True waits for the binary check and raises here (one host sync)."""
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
    if t.is_complex():
        raise ValueError("tt.simulate (hbx) propagates binary {0,1} masks only, as the reference does")
    if not torch.cuda.is_available():
        raise RuntimeError("tt.simulate needs a ROCm GPU (libhbx.so)")
    if t.is_cuda:
        dev = t.device.index
    else:
        dev = torch.cuda.current_device()
        t = t.to(f"cuda:{dev}")
    sc = _scratch(dev)
    _raise_pending(sc)                              # an earlier call's input, already checked
    b, c, h, w = t.shape
    cp = c + (c % 2)                                # the kernels pack plane pairs
    plan = _plan_for(h, w, cp, wl, dx, dy, z, b, dev)
    if cp == c:
        bits = hbx.pack_mask(t, error_ptr=sc.err_dev)
    else:
        bits = torch.zeros((b, cp, h, w // 64), dtype=torch.int64, device=t.device)
        bits[:, :c] = hbx.pack_mask(t, error_ptr=sc.err_dev)
    field, _ = plan.simulate(bits)
    if strict:
        torch.cuda.current_stream(dev).synchronize()
        _raise_pending(sc)
    if cp != c:
        field = field[:, :c]
    return field[0] if squeeze else field


def relativeLoss(x: torch.Tensor, y, fn: Callable) -> torch.Tensor:
    """fn(s * x, y) with the least-squares scale s = sum(x y) / sum(x^2), all in
    float64: DBS_1024_24.py:355 compares two such PSNRs whose difference is
    ~1e-6 dB at 1024x24, below float32 resolution of the PSNR itself.

    fn = tm.get_PSNR on two same-shape GPU tensors (every PSNR call site of the reference):
    one hbx_rel_stats reduction (sum xy, sum x^2, sum y^2 in f64, fixed order) and the PSNR of
    the least-squares-scaled intensity, 10 log10(1 / ((sum y^2 - (sum xy)^2 / sum x^2) / n)),
    read from host-mapped memory after one wait -- the wait get_PSNR's float result needs
    anyway.  Other fns (F.mse_loss at env.py:131) run as torch ops."""
    x = x.as_subclass(torch.Tensor) if isinstance(x, torch.Tensor) else torch.as_tensor(x)
    y = torch.as_tensor(np.asarray(y)) if not isinstance(y, torch.Tensor) else y.as_subclass(torch.Tensor)
    if fn is _metrics.get_PSNR and x.is_cuda and y.is_cuda and x.device == y.device and x.shape == y.shape \
            and x.dtype == y.dtype and x.dtype in (torch.float32, torch.float64) and x.numel() > 0:
        dev = x.device.index
        sc = _scratch(dev)
        xc, yc = x.contiguous(), y.contiguous()
        kind = _lib.SRC_F32 if x.dtype == torch.float32 else _lib.SRC_F64
        st = torch.cuda.current_stream(dev)
        rc = _lib.load().hbx_rel_stats(xc.data_ptr(), yc.data_ptr(), kind, xc.numel(), _lib.REL_LSQ, 1.0,
                                       sc.work.data_ptr(), sc.out_dev, st.cuda_stream)
        if rc != _lib.OK:
            _lib.check(rc, "hbx_rel_stats")
        st.synchronize()
        _raise_pending(sc)                          # the simulate that produced x, if it was not binary
        return float(sc.out[3])
    xd, yd = x.double(), y.to(x.device).double()
    s = torch.sum(xd * yd) / torch.sum(xd * xd)
    out = fn(s * xd, yd)
    if x.is_cuda and x.device.index in _SCRATCH and not isinstance(out, torch.Tensor):
        _raise_pending(_SCRATCH[x.device.index])    # fn waited for the device (a float result)
    return out


def imread(path: str, meta: Optional[Dict] = None, gray: bool = False) -> Tensor:
    """Image file -> tt.Tensor [1, C, H, W] in [0, 1] (Dataset512's loader, DBS_1024_24.py:191)."""
    from PIL import Image
    img = Image.open(path)
    img = img.convert("L" if gray else "RGB")
    a = np.asarray(img, dtype=np.float32) / 255.0
    a = a[None, None] if gray else np.transpose(a, (2, 0, 1))[None]
    return Tensor(torch.from_numpy(np.ascontiguousarray(a)), meta=meta)
