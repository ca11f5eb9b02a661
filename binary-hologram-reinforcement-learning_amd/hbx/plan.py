"""Plan: one propagation configuration on one GPU (wraps hbx_plan_t).

Mirrors what ``tt.simulate(tt.Tensor(x, meta={'dx','wl'}), z)`` +
``tt.relativeLoss(.., tm.get_PSNR)`` compute in the reference
(env.py:123-133,170-174; DBS_1024_24.py:244-257,326-332), but for a whole
batch of bit-packed masks at once, entirely on the device.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional, Sequence

import torch

from . import _lib

PIXEL_PITCH = 7.56e-6          # env.py:124
Z_DEFAULT = 2e-3               # env.py:90
WL_MONO = (515e-9,)            # env.py:124
WL_RGB = (638e-9, 515e-9, 450e-9)   # env_1024_24.py:135-138


@dataclass
class OpticsConfig:
    height: int
    width: int
    groups: int = 1
    planes: int = 8
    wavelengths: Sequence[float] = WL_MONO
    dx: float = PIXEL_PITCH
    dy: float = PIXEL_PITCH
    z: float = Z_DEFAULT
    tf_kind: int = _lib.TF_ASM
    field_kind: int = _lib.FIELD_AMPLITUDE
    rel_scale: int = _lib.REL_LSQ
    peak: float = 1.0

    @property
    def channels(self) -> int:
        return self.groups * self.planes

    @property
    def words(self) -> int:
        return self.width // 64

    def to_c(self) -> _lib.Optics:
        o = _lib.Optics()
        o.height, o.width, o.groups, o.planes = self.height, self.width, self.groups, self.planes
        wl = list(self.wavelengths)
        if len(wl) != self.groups:
            raise ValueError(f"{len(wl)} wavelengths for {self.groups} groups")
        for i, w in enumerate(wl):
            o.wavelength[i] = float(w)
        o.dx, o.dy, o.z = float(self.dx), float(self.dy), float(self.z)
        o.tf_kind, o.field_kind, o.rel_scale = int(self.tf_kind), int(self.field_kind), int(self.rel_scale)
        o.peak = float(self.peak)
        return o


def mono_config(n: int = 256, **kw) -> OpticsConfig:
    """env.py: 1 group x 8 planes at 515 nm (IPS=256, CH=8)."""
    return OpticsConfig(n, n, 1, 8, WL_MONO, **kw)


def rgb_config(n: int = 1024, planes: int = 8, **kw) -> OpticsConfig:
    """env_1024_24.py: 3 groups x 8 planes at 638/515/450 nm (IPS=1024, CH=24)."""
    return OpticsConfig(n, n, 3, planes, WL_RGB, **kw)


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(stream: Optional[torch.cuda.Stream]):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def _need(t: torch.Tensor, name: str, dtype: torch.dtype, shape, device: torch.device):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: dtype {t.dtype} != {dtype}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: shape {tuple(t.shape)} != {tuple(shape)}")
    if t.device != device:
        raise ValueError(f"{name}: device {t.device} != {device}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


_PACK_KIND = {torch.bool: _lib.SRC_U8, torch.int8: _lib.SRC_U8, torch.uint8: _lib.SRC_U8,
              torch.float32: _lib.SRC_F32, torch.float64: _lib.SRC_F64}
_PACK_ALIGN = {_lib.SRC_U8: 4, _lib.SRC_F32: 16, _lib.SRC_F64: 32}


def pack_mask(values: torch.Tensor, threshold: Optional[float] = None, out: Optional[torch.Tensor] = None,
              error_ptr: Optional[int] = None, stream=None) -> torch.Tensor:
    """Device tensor [..., H, W] -> int64 words [..., H, W/64] with ONE HIP launch
    (hbx_pack_mask, ABI v14; bit j of word w = column 64 w + j).

    threshold None: bit = (v != 0), and a value other than 0 / 1 stores 1 at `error_ptr`
    (an address the kernel may write: device or host-mapped memory) -- tt.simulate's binary
    check without a host sync.  threshold t: bit = (v >= t) -- env.py:120's `pre_model >= 0.5`.
    bool / int8 / uint8 / float32 / float64 are read as they are; other dtypes are converted
    to float32 on the device first.  `out`: a contiguous int64 tensor of the result's shape."""
    if not values.is_cuda:
        raise ValueError("pack_mask runs on the GPU (hbx_pack_mask); pack_bits packs host tensors")
    w = values.shape[-1]
    if w % 64:
        raise ValueError("width must be a multiple of 64")
    kind = _PACK_KIND.get(values.dtype)
    if kind is None:
        values, kind = values.to(torch.float32), _lib.SRC_F32
    if not values.is_contiguous() or values.data_ptr() % _PACK_ALIGN[kind]:
        values = values.contiguous() if not values.is_contiguous() else values.clone()
    shape = (*values.shape[:-1], w // 64)
    if out is None:
        out = torch.empty(shape, dtype=torch.int64, device=values.device)
    elif tuple(out.shape) != shape or out.dtype != torch.int64 or not out.is_contiguous() \
            or out.device != values.device:
        raise ValueError(f"pack_mask out: a contiguous int64 {shape} tensor on {values.device}")
    lib = _lib.load()
    mode = _lib.PACK_BINARY if threshold is None else _lib.PACK_THRESHOLD
    s = stream.cuda_stream if stream is not None else torch._C._cuda_getCurrentRawStream(values.device.index)
    rc = lib.hbx_pack_mask(values.data_ptr(), kind, values.numel(), mode,
                           0.0 if threshold is None else float(threshold), out.data_ptr(), error_ptr, s)
    if rc != _lib.OK:
        _lib.check(rc, "hbx_pack_mask")
    return out


def pack_bits(mask: torch.Tensor) -> torch.Tensor:
    """{0,1} tensor [..., H, W] -> int64 words [..., H, W/64] (bit j of word w = col 64w+j).

    GPU tensors: one hbx_pack_mask launch (bit = v != 0).  Host tensors (test fixtures,
    checkpoint tooling) are packed with torch ops on the CPU."""
    w = mask.shape[-1]
    if w % 64:
        raise ValueError("width must be a multiple of 64")
    if mask.is_cuda:
        return pack_mask(mask)
    m = (mask != 0).to(torch.int64).reshape(*mask.shape[:-1], w // 64, 64)
    shifts = torch.arange(64, device=mask.device, dtype=torch.int64)
    return (m << shifts).sum(dim=-1, dtype=torch.int64)   # bit 63 wraps into the sign: same bits


def unpack_bits(words: torch.Tensor, width: int) -> torch.Tensor:
    shifts = torch.arange(64, device=words.device, dtype=torch.int64)
    bits = (words.unsqueeze(-1) >> shifts) & 1
    return bits.reshape(*words.shape[:-1], width).to(torch.int8)


def crop(t: torch.Tensor, margin: int = 64) -> torch.Tensor:
    """Centre crop of ``margin`` pixels per side on the last two axes
    (env_1024_24_128.py:144-149, DBS_1024_24-128.py:210-216); 1024 -> 896."""
    if margin <= 0:
        return t
    return t[..., margin:-margin, margin:-margin].contiguous()


def crop_bits(words: torch.Tensor, margin: int = 64) -> torch.Tensor:
    """The same crop on packed masks [..., H, W/64]: a 64-aligned margin drops
    whole words, so this is a strided copy (no unpacking)."""
    if margin % 64:
        raise ValueError("crop_bits needs a margin that is a multiple of 64")
    k = margin // 64
    return words[..., margin:-margin, k:-k].contiguous()


def crop_config(cfg: "OpticsConfig", margin: int = 64) -> "OpticsConfig":
    """Optics of the cropped mask: same physics, N - 2 * margin pixels."""
    import dataclasses
    return dataclasses.replace(cfg, height=cfg.height - 2 * margin, width=cfg.width - 2 * margin)


class Plan:
    """hbx_plan_t owner.  ``max_jobs`` bounds the group propagations in flight
    (workspace = max_jobs * planes * N^2 * 8 bytes)."""

    def __init__(self, cfg: OpticsConfig, max_jobs: int = 8, device: Optional[int] = None,
                 precision: int = _lib.PRECISION_F32):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise RuntimeError("hbx.Plan needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.cfg = cfg
        self.device_index = torch.cuda.current_device() if device is None else int(device)
        self.device = torch.device("cuda", self.device_index)
        self.max_jobs = int(max_jobs)
        h = C.c_void_p()
        oc = cfg.to_c()
        with torch.cuda.device(self.device_index):
            _lib.check(self.lib.hbx_plan_create(C.byref(h), C.byref(oc), self.max_jobs,
                                                self.device_index), "hbx_plan_create")
        self._h = h
        # bumped by every call that changes what a launch sequence records (timing events,
        # precision variant): a captured HIP graph of this plan's launches is stale after it
        self.generation = 0
        if precision != _lib.PRECISION_F32:
            self.precision = precision

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.hbx_plan_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def workspace_bytes(self) -> int:
        return int(self.lib.hbx_plan_workspace_bytes(self._h))

    # -- device timing of the three passes (hbx_plan_set_timing) --------------------
    def set_timing(self, capacity: int, every: int = 1):
        """Record up to `capacity` launches per pass, every `every`-th launch."""
        _lib.check(self.lib.hbx_plan_set_timing_sampled(self._h, int(capacity), int(every)),
                   "hbx_plan_set_timing_sampled")
        self.generation += 1

    def read_timing(self):
        """{pass: (total_ms, launches, jobs)} for k_rowfwd / k_col / k_rowinv (syncs)."""
        ms = (C.c_double * _lib.NUM_PASSES)()
        n = (C.c_int64 * _lib.NUM_PASSES)()
        jobs = (C.c_int64 * _lib.NUM_PASSES)()
        _lib.check(self.lib.hbx_plan_read_timing(self._h, ms, n, jobs), "hbx_plan_read_timing")
        names = _lib.PIPE_PASS_NAMES[self.pipeline]
        return {name: (ms[i], n[i], jobs[i]) for i, name in enumerate(names)}

    @property
    def precision(self) -> int:
        """hbx_plan_precision: rounding of the pass intermediates (_lib.PRECISION_*)."""
        rc = int(self.lib.hbx_plan_precision(self._h))
        if rc < 0:
            _lib.check(rc, "hbx_plan_precision")
        return rc

    @precision.setter
    def precision(self, kind: int):
        """PRECISION_F32 (the product path) or the bf16 / fp16 intermediate-storage
        numerics of SURVEY 8d cfg 5 (DBS_ratio_0.5.py fp32 vs bf16 sweep)."""
        _lib.check(self.lib.hbx_plan_set_precision(self._h, int(kind)), "hbx_plan_set_precision")
        self.generation += 1

    @property
    def pipeline(self) -> int:
        """hbx_plan_pipeline: _lib.PIPE_THREE_PASS (the only pipeline built since ABI v8)."""
        rc = int(self.lib.hbx_plan_pipeline(self._h))
        if rc < 0:
            _lib.check(rc, "hbx_plan_pipeline")
        return rc

    # -- buffer helpers -------------------------------------------------------
    def mask_shape(self, n_env: int):
        c = self.cfg
        return (n_env, c.channels, c.height, c.words)

    def target_shape(self, n_env: int):
        c = self.cfg
        return (n_env, c.groups, c.height, c.width)

    def _check_mask_target(self, mask, target, n):
        _need(mask, "mask", torch.int64, self.mask_shape(n), self.device)
        _need(target, "target", torch.float32, self.target_shape(n), self.device)

    # -- operators ---------------------------------------------------------------
    def propagate(self, mask: torch.Tensor, target: torch.Tensor, want_intensity: bool = True,
                  stream=None):
        """Full propagation of every group: returns (intensity|None, chan_stats, psnr)."""
        n = mask.shape[0]
        self._check_mask_target(mask, target, n)
        c = self.cfg
        inten = torch.empty((n, c.groups, c.height, c.width), dtype=torch.float32,
                            device=self.device) if want_intensity else None
        stats = torch.empty((n, c.groups, 3), dtype=torch.float64, device=self.device)
        psnr = torch.empty((n,), dtype=torch.float64, device=self.device)
        _lib.check(self.lib.hbx_propagate(self._h, _ptr(mask), _ptr(target), n, _ptr(inten),
                                          _ptr(stats), _ptr(psnr), _stream(stream)), "hbx_propagate")
        return inten, stats, psnr

    def simulate(self, mask: torch.Tensor, want_intensity: bool = False, stream=None):
        """Complex field of every plane (tt.simulate restated): returns
        (field complex64 [B, CH, H, W], intensity [B, G, H, W] | None)."""
        n = mask.shape[0]
        c = self.cfg
        _need(mask, "mask", torch.int64, self.mask_shape(n), self.device)
        field = torch.empty((n, c.channels, c.height, c.width, 2), dtype=torch.float32, device=self.device)
        inten = torch.empty((n, c.groups, c.height, c.width), dtype=torch.float32,
                            device=self.device) if want_intensity else None
        _lib.check(self.lib.hbx_simulate(self._h, _ptr(mask), n, _ptr(field), _ptr(inten), _stream(stream)),
                   "hbx_simulate")
        return torch.view_as_complex(field), inten

    def psnr(self, chan_stats: torch.Tensor, stream=None) -> torch.Tensor:
        n = chan_stats.shape[0]
        _need(chan_stats, "chan_stats", torch.float64, (n, self.cfg.groups, 3), self.device)
        out = torch.empty((n,), dtype=torch.float64, device=self.device)
        _lib.check(self.lib.hbx_psnr(self._h, _ptr(chan_stats), n, _ptr(out), _stream(stream)), "hbx_psnr")
        return out

    def flip_map(self, mask: torch.Tensor, target: torch.Tensor, out: Optional[torch.Tensor] = None,
                 stream=None):
        """PSNR change of every single-pixel flip of ONE env against its
        current state (hbx_flip_map): returns (dpsnr f32 [CH, H, W], base
        psnr f64 [1]).  dpsnr.flatten()[a] is the change for action a."""
        c = self.cfg
        _need(mask, "mask", torch.int64, self.mask_shape(1)[1:], self.device)
        _need(target, "target", torch.float32, self.target_shape(1)[1:], self.device)
        if out is None:
            out = torch.empty((c.channels, c.height, c.width), dtype=torch.float32, device=self.device)
        _need(out, "out", torch.float32, (c.channels, c.height, c.width), self.device)
        base = torch.empty((1,), dtype=torch.float64, device=self.device)
        _lib.check(self.lib.hbx_flip_map(self._h, _ptr(mask), _ptr(target), _ptr(out), _ptr(base),
                                         _stream(stream)), "hbx_flip_map")
        return out, base

    def eval_flips(self, base_mask: torch.Tensor, target: torch.Tensor, base_stats: torch.Tensor,
                   flips: torch.Tensor, psnr_out: Optional[torch.Tensor] = None,
                   group_stats: Optional[torch.Tensor] = None, stream=None):
        """PSNR of K independent single-pixel flips of ONE base env."""
        c = self.cfg
        _need(base_mask, "base_mask", torch.int64, self.mask_shape(1)[1:], self.device)
        _need(target, "target", torch.float32, self.target_shape(1)[1:], self.device)
        _need(base_stats, "base_stats", torch.float64, (c.groups, 3), self.device)
        k = flips.shape[0]
        _need(flips, "flips", torch.int64, (k,), self.device)
        if psnr_out is None:
            psnr_out = torch.empty((k,), dtype=torch.float64, device=self.device)
        if group_stats is None:
            group_stats = torch.empty((k, 3), dtype=torch.float64, device=self.device)
        _lib.check(self.lib.hbx_eval_flips(self._h, _ptr(base_mask), _ptr(target), _ptr(base_stats),
                                           _ptr(flips), k, _ptr(psnr_out), _ptr(group_stats),
                                           _stream(stream)), "hbx_eval_flips")
        return psnr_out, group_stats

    # -- plane-cached candidates (ABI v10): the FFT mode's bits, only the flipped pair propagated
    def plane_pool(self, spare_pairs: int):
        """(plane_inten f32 [CH + 2 S, H, W], plane_slot int32 [CH + 2 S]) for one base env."""
        c = self.cfg
        n = c.channels + 2 * int(spare_pairs)
        return (torch.empty((n, c.height, c.width), dtype=torch.float32, device=self.device),
                torch.empty((n,), dtype=torch.int32, device=self.device))

    def _check_pool(self, plane_inten, plane_slot):
        c = self.cfg
        n = plane_slot.shape[0] if isinstance(plane_slot, torch.Tensor) else -1
        _need(plane_slot, "plane_slot", torch.int32, (n,), self.device)
        _need(plane_inten, "plane_inten", torch.float32, (n, c.height, c.width), self.device)
        if n < c.channels + 2 or (n - c.channels) % 2:
            raise ValueError(f"plane pool of {n} slots: need CH + 2 S with S >= 1")
        return (n - c.channels) // 2

    def planes_fill(self, mask, target, plane_inten, plane_slot, stream=None):
        """Full propagation of ONE base env into its plane pool (hbx_planes_fill):
        returns (chan_stats f64 [G, 3], psnr f64 [1])."""
        c = self.cfg
        _need(mask, "mask", torch.int64, self.mask_shape(1)[1:], self.device)
        _need(target, "target", torch.float32, self.target_shape(1)[1:], self.device)
        s = self._check_pool(plane_inten, plane_slot)
        stats = torch.empty((c.groups, 3), dtype=torch.float64, device=self.device)
        psnr = torch.empty((1,), dtype=torch.float64, device=self.device)
        _lib.check(self.lib.hbx_planes_fill(self._h, _ptr(mask), _ptr(target), _ptr(plane_inten), _ptr(plane_slot),
                                            s, _ptr(stats), _ptr(psnr), _stream(stream)), "hbx_planes_fill")
        return stats, psnr

    def eval_flips_planes(self, base_mask, target, base_stats, plane_inten, plane_slot, flips,
                          psnr_out=None, group_stats=None, stream=None):
        """eval_flips with the base env's plane pool: the same PSNRs bit for bit."""
        c = self.cfg
        _need(base_mask, "base_mask", torch.int64, self.mask_shape(1)[1:], self.device)
        _need(target, "target", torch.float32, self.target_shape(1)[1:], self.device)
        _need(base_stats, "base_stats", torch.float64, (c.groups, 3), self.device)
        s = self._check_pool(plane_inten, plane_slot)
        k = flips.shape[0]
        _need(flips, "flips", torch.int64, (k,), self.device)
        if psnr_out is None:
            psnr_out = torch.empty((k,), dtype=torch.float64, device=self.device)
        if group_stats is None:
            group_stats = torch.empty((k, 3), dtype=torch.float64, device=self.device)
        _lib.check(self.lib.hbx_eval_flips_planes(self._h, _ptr(base_mask), _ptr(target), _ptr(base_stats),
                                                  _ptr(plane_inten), _ptr(plane_slot), s, _ptr(flips), k,
                                                  _ptr(psnr_out), _ptr(group_stats), _stream(stream)),
                   "hbx_eval_flips_planes")
        return psnr_out, group_stats

    def commit_flip_planes(self, base_mask, base_stats, prev_psnr, plane_inten, plane_slot, flips, psnr_out,
                           group_stats, k_dev: torch.Tensor, stream=None):
        """Commit candidate k_dev of an eval_flips_planes batch (its fresh pair swaps in)."""
        k = self._check_commit(base_mask, base_stats, prev_psnr, flips, psnr_out, group_stats, k_dev)
        s = self._check_pool(plane_inten, plane_slot)
        _lib.check(self.lib.hbx_commit_flip_planes(self._h, _ptr(base_mask), _ptr(base_stats), _ptr(prev_psnr),
                                                   _ptr(plane_slot), s, _ptr(flips), _ptr(psnr_out),
                                                   _ptr(group_stats), _ptr(k_dev), k, _stream(stream)),
                   "hbx_commit_flip_planes")

    def dbs_walk_planes(self, base_mask, target, base_stats, plane_inten, plane_slot, order: torch.Tensor,
                        walk: torch.Tensor, accept_pos: torch.Tensor, accept_psnr: torch.Tensor, K: int,
                        batches: int, stream=None, fill=None):
        """hbx_dbs_walk_planes: enqueue `batches` device-decided batches of K candidates of the
        FFT-mode greedy on the base state's plane pool (no host round trip).  fill = (counts, target,
        tol): the on-pixel ratio constraint (hbx_dbs_walk_planes_fill, an extension; counts [G] int64
        on the device, updated by the walk)."""
        c = self.cfg
        _need(base_mask, "base_mask", torch.int64, self.mask_shape(1)[1:], self.device)
        _need(target, "target", torch.float32, self.target_shape(1)[1:], self.device)
        _need(base_stats, "base_stats", torch.float64, (c.groups, 3), self.device)
        s = self._check_pool(plane_inten, plane_slot)
        _need(order, "order", torch.int64, (order.shape[0],), self.device)
        _need(walk, "walk", torch.uint8, (C.sizeof(_lib.DbsWalk),), self.device)
        cap = accept_pos.shape[0]
        _need(accept_pos, "accept_pos", torch.int64, (cap,), self.device)
        _need(accept_psnr, "accept_psnr", torch.float64, (cap,), self.device)
        if fill is None:
            _lib.check(self.lib.hbx_dbs_walk_planes(self._h, _ptr(base_mask), _ptr(target), _ptr(base_stats),
                                                    _ptr(plane_inten), _ptr(plane_slot), s, _ptr(order),
                                                    int(order.shape[0]), _ptr(walk), _ptr(accept_pos),
                                                    _ptr(accept_psnr), cap, int(K), int(batches), _stream(stream)),
                       "hbx_dbs_walk_planes")
            return
        counts, f_target, f_tol = fill
        _need(counts, "fill counts", torch.int64, (c.groups,), self.device)
        _lib.check(self.lib.hbx_dbs_walk_planes_fill(self._h, _ptr(base_mask), _ptr(target), _ptr(base_stats),
                                                     _ptr(plane_inten), _ptr(plane_slot), s, _ptr(order),
                                                     int(order.shape[0]), _ptr(walk), _ptr(accept_pos),
                                                     _ptr(accept_psnr), cap, int(K), int(batches), _ptr(counts),
                                                     int(f_target), int(f_tol), _stream(stream)),
                   "hbx_dbs_walk_planes_fill")

    def eval_flips_psf(self, base_mask, target, base_stats, field, intensity, flips,
                       psnr_out=None, group_stats=None, stream=None):
        """eval_flips on the incremental-field path: field [CH, H, W, 2] f32 and
        intensity [G, H, W] f32 of the base state (from simulate)."""
        c = self.cfg
        _need(base_mask, "base_mask", torch.int64, self.mask_shape(1)[1:], self.device)
        _need(target, "target", torch.float32, self.target_shape(1)[1:], self.device)
        _need(base_stats, "base_stats", torch.float64, (c.groups, 3), self.device)
        _need(field, "field", torch.float32, (c.channels, c.height, c.width, 2), self.device)
        _need(intensity, "intensity", torch.float32, (c.groups, c.height, c.width), self.device)
        k = flips.shape[0]
        _need(flips, "flips", torch.int64, (k,), self.device)
        if psnr_out is None:
            psnr_out = torch.empty((k,), dtype=torch.float64, device=self.device)
        if group_stats is None:
            group_stats = torch.empty((k, 3), dtype=torch.float64, device=self.device)
        _lib.check(self.lib.hbx_eval_flips_psf(self._h, _ptr(base_mask), _ptr(target), _ptr(base_stats),
                                               _ptr(field), _ptr(intensity), _ptr(flips), k, _ptr(psnr_out),
                                               _ptr(group_stats), _stream(stream)), "hbx_eval_flips_psf")
        return psnr_out, group_stats

    def _check_commit(self, base_mask, base_stats, prev_psnr, flips, psnr_out, group_stats, k_dev):
        c = self.cfg
        _need(base_mask, "base_mask", torch.int64, self.mask_shape(1)[1:], self.device)
        _need(base_stats, "base_stats", torch.float64, (c.groups, 3), self.device)
        _need(prev_psnr, "prev_psnr", torch.float64, (1,), self.device)
        k = flips.shape[0]
        _need(flips, "flips", torch.int64, (k,), self.device)
        if psnr_out.shape[0] < k or group_stats.shape[0] < k:
            raise ValueError(f"psnr_out / group_stats hold fewer than the {k} candidates of flips")
        _need(psnr_out, "psnr_out", torch.float64, (psnr_out.shape[0],), self.device)
        _need(group_stats, "group_stats", torch.float64, (group_stats.shape[0], 3), self.device)
        _need(k_dev, "k", torch.int32, (1,), self.device)
        return k

    def commit_flip_psf(self, base_mask, base_stats, prev_psnr, field, intensity, flips, psnr_out,
                        group_stats, k_dev: torch.Tensor, stream=None):
        """Commit candidate k_dev of an eval_flips_psf batch (a k outside the
        batch commits nothing)."""
        c = self.cfg
        k = self._check_commit(base_mask, base_stats, prev_psnr, flips, psnr_out, group_stats, k_dev)
        _need(field, "field", torch.float32, (c.channels, c.height, c.width, 2), self.device)
        _need(intensity, "intensity", torch.float32, (c.groups, c.height, c.width), self.device)
        _lib.check(self.lib.hbx_commit_flip_psf(self._h, _ptr(base_mask), _ptr(base_stats), _ptr(prev_psnr),
                                                _ptr(field), _ptr(intensity), _ptr(flips), _ptr(psnr_out),
                                                _ptr(group_stats), _ptr(k_dev), k, _stream(stream)),
                   "hbx_commit_flip_psf")

    def dbs_walk_psf(self, base_mask, target, base_stats, field, intensity, order: torch.Tensor,
                     walk: torch.Tensor, accept_pos: torch.Tensor, accept_psnr: torch.Tensor, K: int,
                     batches: int, stream=None):
        """hbx_dbs_walk_psf: enqueue `batches` speculative batches of K candidates of the
        device-resident greedy walk.  walk: uint8 [sizeof(hbx_dbs_walk_t)] on the device."""
        c = self.cfg
        _need(field, "field", torch.float32, (c.channels, c.height, c.width, 2), self.device)
        _need(intensity, "intensity", torch.float32, (c.groups, c.height, c.width), self.device)
        _need(base_mask, "base_mask", torch.int64, self.mask_shape(1)[1:], self.device)
        _need(target, "target", torch.float32, self.target_shape(1)[1:], self.device)
        _need(base_stats, "base_stats", torch.float64, (c.groups, 3), self.device)
        _need(order, "order", torch.int64, (order.shape[0],), self.device)
        _need(walk, "walk", torch.uint8, (C.sizeof(_lib.DbsWalk),), self.device)
        cap = accept_pos.shape[0]
        _need(accept_pos, "accept_pos", torch.int64, (cap,), self.device)
        _need(accept_psnr, "accept_psnr", torch.float64, (cap,), self.device)
        _lib.check(self.lib.hbx_dbs_walk_psf(self._h, _ptr(base_mask), _ptr(target), _ptr(base_stats),
                                             _ptr(field), _ptr(intensity), _ptr(order), int(order.shape[0]),
                                             _ptr(walk),
                                             _ptr(accept_pos), _ptr(accept_psnr), cap, int(K), int(batches),
                                             _stream(stream)), "hbx_dbs_walk_psf")

    def commit_flip(self, base_mask, base_stats, prev_psnr, flips, psnr_out, group_stats,
                    k_dev: torch.Tensor, stream=None):
        """Commit candidate k_dev of an eval_flips batch (a k outside the batch
        commits nothing)."""
        k = self._check_commit(base_mask, base_stats, prev_psnr, flips, psnr_out, group_stats, k_dev)
        _lib.check(self.lib.hbx_commit_flip(self._h, _ptr(base_mask), _ptr(base_stats), _ptr(prev_psnr),
                                            _ptr(flips), _ptr(psnr_out), _ptr(group_stats), _ptr(k_dev), k,
                                            _stream(stream)), "hbx_commit_flip")

    def step(self, mask, actions, target, chan_stats, prev_psnr, accept_rule=_lib.ACCEPT_DBS,
             stream=None):
        """DBS primitive (include/hbx.h hbx_step): returns (psnr, accepted)."""
        n = mask.shape[0]
        self._check_mask_target(mask, target, n)
        _need(actions, "actions", torch.int64, (n,), self.device)
        psnr = torch.empty((n,), dtype=torch.float64, device=self.device)
        acc = torch.empty((n,), dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.hbx_step(self._h, _ptr(mask), _ptr(actions), n, _ptr(target), _ptr(chan_stats),
                                     _ptr(prev_psnr), _ptr(psnr), _ptr(acc), int(accept_rule),
                                     _stream(stream)), "hbx_step")
        return psnr, acc

    # env-level entry points are used by hbx.env (EnvState owns the buffers)
    def env_reset(self, bufs: _lib.EnvBuffers, n_env: int, env_ids: Optional[torch.Tensor] = None,
                  stream=None):
        n_ids = 0 if env_ids is None else int(env_ids.shape[0])
        _lib.check(self.lib.hbx_env_reset(self._h, C.byref(bufs), n_env, _ptr(env_ids), n_ids,
                                          _stream(stream)), "hbx_env_reset")

    def env_obs_sync(self, bufs: _lib.EnvBuffers, n_env: int, what: int = _lib.OBS_STATE | _lib.OBS_RECON,
                     env_ids: Optional[torch.Tensor] = None, stream=None):
        """Rebuild the observation mirrors (state_bytes from the mask, recon from the
        intensity cache) of the listed envs -- hbx_env_obs_sync."""
        n_ids = 0 if env_ids is None else int(env_ids.shape[0])
        _lib.check(self.lib.hbx_env_obs_sync(self._h, C.byref(bufs), n_env, _ptr(env_ids), n_ids, int(what),
                                             _stream(stream)), "hbx_env_obs_sync")

    def env_step_psf(self, bufs, params, n_env, actions, reward, psnr, accepted, terminated, truncated,
                     stream=None):
        _lib.check(self.lib.hbx_env_step_psf(self._h, C.byref(bufs), C.byref(params), n_env, _ptr(actions),
                                             _ptr(reward), _ptr(psnr), _ptr(accepted), _ptr(terminated),
                                             _ptr(truncated), _stream(stream)), "hbx_env_step_psf")

    def field_refresh(self, bufs, n_env, env_ids: Optional[torch.Tensor] = None, stream=None):
        n_ids = 0 if env_ids is None else int(env_ids.shape[0])
        _lib.check(self.lib.hbx_field_refresh(self._h, C.byref(bufs), n_env, _ptr(env_ids), n_ids,
                                              _stream(stream)), "hbx_field_refresh")

    def env_step(self, bufs, params, n_env, actions, reward, psnr, accepted, terminated, truncated,
                 group_intensity=None, stream=None):
        _lib.check(self.lib.hbx_env_step(self._h, C.byref(bufs), C.byref(params), n_env, _ptr(actions),
                                         _ptr(reward), _ptr(psnr), _ptr(accepted), _ptr(terminated),
                                         _ptr(truncated), _ptr(group_intensity), _stream(stream)),
                   "hbx_env_step")
