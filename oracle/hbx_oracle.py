"""CPU oracle for the binary-hologram hot path -- TEST INFRASTRUCTURE ONLY.

This module is a float64 numpy restatement of the reference's per-flip
evaluation path (mask -> 2-D FFT propagation -> |.|^2 plane mean -> relative
PSNR -> reward / rollback).  Only ``tests/``, ``__graft_entry__.smoke()`` and
the ``cpu_baseline`` leg of ``bench.py`` may import it, and only as the
checker / the timed CPU baseline.  The shipped path (``hbx``) never imports
it and fails loudly when its HIP library is missing.

Parity status
-------------
* Integer work (action decode, flip indexing, bit packing, counters, reward
  cubic, accept/rollback/termination rules) follows the reference code
  line-for-line and is pinned by the known answers the reference itself
  states (``env.py:228-229``: "1 = +300, 1/2 = +100, 1/4 = -100, 1/8 = -300").
* The physics (``tt.simulate``, ``tt.relativeLoss``, ``tm.get_PSNR``) lives
  in the third-party package ``torchOptics`` which is absent from
  /root/reference, unpinned (not in requirements.txt, ``.gitignore:3``) and
  not installable offline.  Its behaviour is RESTATED from the published
  angular-spectrum / PSNR definitions below and every assumption is a
  switch.  -> **parity unpinned** for the floating-point physics: it is pinned
  only by analytic properties (Parseval energy conservation, plane-wave
  invariance, ASM->Fresnel agreement at small angles, symmetry) in
  tests/test_oracle.py, never by reference-produced vectors (none exist).

Reference call sites restated here (all under /root/reference):
  action decode ........ env.py:157-161, DBS_1024_24.py:314-317
  flip / record ........ env.py:164-167
  mask -> field ........ env.py:170-171 (real {0,1} amplitude)
  propagate ............ env.py:172 (tt.simulate(field, z=2e-3))
  plane mean ........... env.py:173, DBS_1024_24.py:329
  RGB groups / metas ... env_1024_24.py:135-147 (wl 638/515/450 nm, 8 planes each)
  relative PSNR ........ env.py:174, DBS_1024_24.py:332
  reward / rollback .... env.py:184-259
  greedy DBS ........... DBS.py:247-294, DBS_1024_24.py:313-422 (strict >)
  early stop ........... DBS_01.py / DBS_ratio_0.5.py:370 (psnr_diff >= thr)
  probe sweep .......... DBS_1024_24-128.py:310-373, range.py:294-335
  pre-model histogram .. DBS_1024_24.py:289-300,398-416
  crop ................. env_1024_24_128.py:144-149
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

# ---------------------------------------------------------------------------
# Constants of the reference (env.py:27-29, env.py:124, env_1024_24.py:135-138)
# ---------------------------------------------------------------------------
RW = 800.0                          # env.py:29 reward weight
PIXEL_PITCH = 7.56e-6               # env.py:124 'dx'
Z_DEFAULT = 2e-3                    # env.py:90,154 z
WL_MONO = (515e-9,)                 # env.py:124 'wl'
WL_RGB = (638e-9, 515e-9, 450e-9)   # env_1024_24.py:135-138
PLANES_PER_GROUP = 8                # env_1024_24.py:140-147 (24 // 3)

TF_ASM, TF_FRESNEL = 0, 1
FIELD_AMPLITUDE, FIELD_PHASE = 0, 1
REL_NONE, REL_LSQ = 0, 1


# ---------------------------------------------------------------------------
# Integer work: action decode, bit packing
# ---------------------------------------------------------------------------
def decode_action(action, height: int, width: int):
    """env.py:157-161 / DBS_1024_24.py:314-317.

    channel = a // (H*W); k = a % (H*W); row = k // W; col = k % W.
    Works elementwise on int64 arrays (bit-exact integer arithmetic)."""
    a = np.asarray(action, dtype=np.int64)
    hw = np.int64(height) * np.int64(width)
    channel = a // hw
    k = a % hw
    return channel, k // width, k % width


def encode_action(channel, row, col, height: int, width: int):
    return (np.asarray(channel, np.int64) * height + np.asarray(row, np.int64)) * width \
        + np.asarray(col, np.int64)


def pack_mask(mask: np.ndarray) -> np.ndarray:
    """{0,1} uint8 [..., H, W] -> uint64 words [..., H, W/64].

    Bit j of word w is pixel column 64*w + j (little-endian bit order), which is
    the layout the C-ABI (include/hbx.h) declares."""
    mask = np.ascontiguousarray(mask, dtype=np.uint8)
    w = mask.shape[-1]
    if w % 64:
        raise ValueError("width must be a multiple of 64")
    packed = np.packbits(mask, axis=-1, bitorder="little")
    return np.ascontiguousarray(packed).view("<u8").reshape(mask.shape[:-1] + (w // 64,))


def unpack_mask(bits: np.ndarray, width: int) -> np.ndarray:
    bits = np.ascontiguousarray(bits, dtype="<u8")
    as_bytes = bits.view(np.uint8).reshape(bits.shape[:-1] + (width // 8,))
    return np.unpackbits(as_bytes, axis=-1, bitorder="little")[..., :width]


# ---------------------------------------------------------------------------
# Physics restatement (torchOptics is absent: assumptions are switches)
# ---------------------------------------------------------------------------
def freq_grid(n: int, d: float) -> np.ndarray:
    """FFT-order spatial frequencies k/(n*d) (numpy.fft.fftfreq)."""
    return np.fft.fftfreq(n, d=d)


def transfer_function(height: int, width: int, dx: float, dy: float, wl: float, z: float,
                      tf_kind: int = TF_ASM) -> np.ndarray:
    """Free-space transfer function H(fy, fx) in FFT order, complex128.

    ASM (default): H = exp(i 2 pi z sqrt(1/wl^2 - fx^2 - fy^2)),
    evanescent components (negative radicand) set to 0 -- inactive at the
    reference parameters.  Fresnel: H = exp(i 2 pi z / wl) exp(-i pi wl z (fx^2+fy^2)).
    """
    fx = freq_grid(width, dx)[None, :]
    fy = freq_grid(height, dy)[:, None]
    f2 = fx * fx + fy * fy
    if tf_kind == TF_ASM:
        arg = 1.0 / (wl * wl) - f2
        prop = arg > 0
        h = np.zeros(f2.shape, np.complex128)
        h[prop] = np.exp(2j * np.pi * z * np.sqrt(arg[prop]))
        return h
    if tf_kind == TF_FRESNEL:
        return np.exp(2j * np.pi * z / wl) * np.exp(-1j * np.pi * wl * z * f2)
    raise ValueError(f"unknown tf_kind {tf_kind}")


def mask_to_field(mask: np.ndarray, field_kind: int = FIELD_AMPLITUDE) -> np.ndarray:
    """env.py:170-171: the int8 {0,1} mask becomes a real float field.

    amplitude (literal reference): u = m;  phase: u = exp(i pi m) = 1 - 2m."""
    m = np.asarray(mask, dtype=np.float64)
    if field_kind == FIELD_AMPLITUDE:
        return m
    if field_kind == FIELD_PHASE:
        return 1.0 - 2.0 * m
    raise ValueError(f"unknown field_kind {field_kind}")


def propagate(field_planes: np.ndarray, h: np.ndarray) -> np.ndarray:
    """tt.simulate(field, z) restated: U = IFFT2(FFT2(u) * H) per plane (no padding)."""
    return np.fft.ifft2(np.fft.fft2(field_planes, axes=(-2, -1)) * h, axes=(-2, -1))


def group_intensity(mask_group: np.ndarray, h: np.ndarray,
                    field_kind: int = FIELD_AMPLITUDE) -> np.ndarray:
    """env.py:172-173 / DBS_1024_24.py:328-329: mean over the P planes of |U_p|^2.

    mask_group: [P, H, W] {0,1}; returns float64 [H, W]."""
    u = propagate(mask_to_field(mask_group, field_kind), h)
    return np.mean(u.real * u.real + u.imag * u.imag, axis=0)


def chan_stats(intensity: np.ndarray, target: np.ndarray) -> np.ndarray:
    """Per-channel sufficient statistics (sum I*T, sum I^2, sum T^2), float64."""
    i = np.asarray(intensity, np.float64)
    t = np.asarray(target, np.float64)
    return np.array([np.sum(i * t), np.sum(i * i), np.sum(t * t)], np.float64)


def psnr_from_stats(stats: np.ndarray, count: int, rel_scale: int = REL_LSQ,
                    peak: float = 1.0) -> float:
    """tt.relativeLoss(x, y, tm.get_PSNR) restated from summed statistics.

    lsq: s = sum(x y)/sum(x^2); mse = mean((s x - y)^2)
                          = (sum y^2 - sum(x y)^2 / sum x^2) / count
    none:            mse = (sum x^2 - 2 sum x y + sum y^2) / count
    psnr = 10 log10(peak^2 / mse).  ``stats`` is (sum xy, sum x^2, sum y^2)
    summed over every channel the reference passes (all of rgb)."""
    sxy, sxx, syy = (float(v) for v in np.asarray(stats, np.float64).reshape(-1, 3).sum(axis=0))
    if rel_scale == REL_LSQ:
        mse = (syy - sxy * sxy / sxx) / count if sxx > 0 else syy / count
    elif rel_scale == REL_NONE:
        mse = (sxx - 2.0 * sxy + syy) / count
    else:
        raise ValueError(f"unknown rel_scale {rel_scale}")
    if mse <= 0:
        return float("inf")
    return 10.0 * math.log10(peak * peak / mse)


def relative_psnr(x: np.ndarray, y: np.ndarray, rel_scale: int = REL_LSQ,
                  peak: float = 1.0) -> float:
    """Direct form of the same metric (used to cross-check psnr_from_stats)."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    if rel_scale == REL_LSQ:
        s = np.sum(x * y) / np.sum(x * x)
        x = s * x
    mse = np.mean((x - y) ** 2)
    return 10.0 * math.log10(peak * peak / mse)


def relative_mse(x: np.ndarray, y: np.ndarray, rel_scale: int = REL_LSQ) -> float:
    """tt.relativeLoss(x, y, F.mse_loss) restated (env.py:131)."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    if rel_scale == REL_LSQ:
        x = (np.sum(x * y) / np.sum(x * x)) * x
    return float(np.mean((x - y) ** 2))


# ---------------------------------------------------------------------------
# Reward (env.py:184-259)
# ---------------------------------------------------------------------------
def success_cubic(s: float) -> float:
    """env.py:230-235 goal-reaching bonus (constant -595.2)."""
    return 1828.57 * (s ** 3) - 3733.33 * (s ** 2) + 2800 * s - 595.2


def max_steps_cubic(s: float) -> float:
    """env.py:249-254 end-of-episode bonus (constant -595.24)."""
    return 1828.57 * (s ** 3) - 3733.33 * (s ** 2) + 2800 * s - 595.24


@dataclass
class OpticsConfig:
    height: int
    width: int
    groups: int = 1
    planes: int = PLANES_PER_GROUP
    wavelengths: Sequence[float] = WL_MONO
    dx: float = PIXEL_PITCH
    dy: float = PIXEL_PITCH
    z: float = Z_DEFAULT
    tf_kind: int = TF_ASM
    field_kind: int = FIELD_AMPLITUDE
    rel_scale: int = REL_LSQ
    peak: float = 1.0

    @property
    def channels(self) -> int:
        return self.groups * self.planes

    def transfer(self, g: int) -> np.ndarray:
        return transfer_function(self.height, self.width, self.dx, self.dy,
                                 self.wavelengths[g], self.z, self.tf_kind)


def mono_config(n: int = 256, **kw) -> OpticsConfig:
    return OpticsConfig(n, n, 1, PLANES_PER_GROUP, WL_MONO, **kw)


def rgb_config(n: int = 1024, planes: int = PLANES_PER_GROUP, **kw) -> OpticsConfig:
    return OpticsConfig(n, n, 3, planes, WL_RGB, **kw)


class Propagator:
    """Caches H per group; evaluates group intensities and PSNR (float64)."""

    def __init__(self, cfg: OpticsConfig):
        self.cfg = cfg
        self.h = [cfg.transfer(g) for g in range(cfg.groups)]

    def group_intensity(self, mask: np.ndarray, g: int) -> np.ndarray:
        p = self.cfg.planes
        return group_intensity(mask[g * p:(g + 1) * p], self.h[g], self.cfg.field_kind)

    def all_intensity(self, mask: np.ndarray) -> np.ndarray:
        return np.stack([self.group_intensity(mask, g) for g in range(self.cfg.groups)])

    def psnr(self, stats: np.ndarray) -> float:
        c = self.cfg
        return psnr_from_stats(stats, c.groups * c.height * c.width, c.rel_scale, c.peak)


# ---------------------------------------------------------------------------
# Environment semantics (env.py:90-259; RGB per-flip intent DBS_1024_24.py:313-422)
# ---------------------------------------------------------------------------
@dataclass
class StepResult:
    action: int
    psnr: float
    reward: float
    accepted: bool
    terminated: bool
    truncated: bool


@dataclass
class OracleEnv:
    """Single-environment restatement of BinaryHologramEnv.

    G=1 follows env.py exactly; G=3 follows the working per-flip semantics of
    DBS_1024_24.py (only the touched colour group is re-propagated, the other
    two group means are cached -- SURVEY F8)."""
    cfg: OpticsConfig
    max_steps: int = 10000
    T_PSNR: float = 30.0
    T_steps: int = 1
    T_PSNR_DIFF: float = 0.1
    accept_rule: int = 0          # 0: env (rollback iff delta < 0); 1: DBS (accept iff delta > 0)
    prop: Propagator = field(init=False)

    def __post_init__(self):
        self.prop = Propagator(self.cfg)

    def reset(self, pre_model: np.ndarray, target: np.ndarray):
        """env.py:90-152 minus data loading / pre-model inference (injected)."""
        c = self.cfg
        self.pre_model = np.asarray(pre_model, np.float32)
        self.state = (self.pre_model >= 0.5).astype(np.int8)          # env.py:120
        self.state_record = np.zeros_like(self.state)                  # env.py:121
        self.target = np.asarray(target, np.float32).reshape(c.groups, c.height, c.width)
        self.intensity = self.prop.all_intensity(self.state)
        self.stats = np.stack([chan_stats(self.intensity[g], self.target[g])
                               for g in range(c.groups)])
        self.initial_psnr = self.prop.psnr(self.stats)                 # env.py:132
        self.previous_psnr = self.initial_psnr
        self.steps = 0
        self.flip_count = 0
        self.psnr_sustained_steps = 0
        self.max_psnr_diff = float("-inf")
        return self.initial_psnr

    def evaluate_flip(self, action: int):
        """psnr after flipping `action` (state left unchanged) + new group data."""
        c = self.cfg
        ch, r, col = (int(v) for v in decode_action(action, c.height, c.width))
        g = ch // c.planes
        self.state[ch, r, col] ^= 1
        ig = self.prop.group_intensity(self.state, g)
        self.state[ch, r, col] ^= 1
        st = self.stats.copy()
        st[g] = chan_stats(ig, self.target[g])
        return self.prop.psnr(st), g, ig, st

    def step(self, action: int, accept: Optional[bool] = None) -> StepResult:
        """env.py:154-259.  ``accept`` (tests only) overrides the rollback decision -- to
        follow the device's decision at a change below f32 resolution, where an f32 and an
        f64 propagation can order a near-tie differently; the caller asserts the rule's own
        decision wherever the change is clear of that resolution.  ``last_change`` and
        ``last_group_intensity`` keep the change and the stepped group's intensity."""
        c = self.cfg
        self.steps += 1                                                # env.py:155
        ch, r, col = (int(v) for v in decode_action(action, c.height, c.width))
        self.state_record[ch, r, col] += 1                             # env.py:165
        self.flip_count += 1                                           # env.py:167
        psnr_after, g, ig, st = self.evaluate_flip(action)
        psnr_change = psnr_after - self.previous_psnr                  # env.py:184
        psnr_diff = psnr_after - self.initial_psnr                     # env.py:185
        self.last_change, self.last_group_intensity = psnr_change, (g, ig)
        reward = psnr_change * RW                                      # env.py:188
        reject = (psnr_change < 0) if self.accept_rule == 0 else not (psnr_change > 0)
        if accept is not None:
            reject = not accept
        if reject:                                                     # env.py:191-196
            self.flip_count -= 1
            return StepResult(action, psnr_after, reward, False, False, False)
        self.state[ch, r, col] ^= 1
        self.intensity[g] = ig
        self.stats = st
        self.max_psnr_diff = max(self.max_psnr_diff, psnr_diff)        # env.py:198
        success_ratio = self.flip_count / self.steps if self.steps > 0 else 0   # env.py:200
        self.previous_psnr = psnr_after                                # env.py:214
        if psnr_diff >= self.T_PSNR_DIFF or (psnr_after >= self.T_PSNR and psnr_diff < 0.1):
            self.psnr_sustained_steps += 1                             # env.py:225
            if self.psnr_sustained_steps >= self.T_steps and psnr_diff >= self.T_PSNR_DIFF:
                reward += success_cubic(success_ratio)                 # env.py:230-235
        if self.steps >= self.max_steps:
            reward += max_steps_cubic(success_ratio)                   # env.py:249-254
        terminated = self.steps >= self.max_steps or self.psnr_sustained_steps >= self.T_steps
        truncated = self.steps >= self.max_steps                       # env.py:257-258
        return StepResult(action, psnr_after, reward, True, bool(terminated), bool(truncated))


def importance_sample(num_pixels: int, k: int, seed: int, env_index: int = 0, reset_index: int = 0):
    """The K random flips of an importance reset.  env_group.py:96 draws them
    with the global np.random.randint; the build seeds them per env and reset
    (hbx/env.py::_importance_reset uses the same rule)."""
    return np.random.default_rng([seed, env_index, reset_index]).integers(0, num_pixels, k)


def group_linear_bonus(steps: int) -> float:
    """env_group.py:297-298 / 313-314: 100 + m (steps - 1000), m = -200/1500."""
    return 100 + (-200.0 / 1500.0) * (steps - 1000)


class OracleEnvGroup(OracleEnv):
    """env_group.py:37-320: importance-rank rewards, dynamic T_PSNR_DIFF."""

    def reset_group(self, pre_model, target, sample_actions):
        base = self.reset(pre_model, target)
        ps = probe_sweep(self, sample_actions)                         # env_group.py:90-120
        self.psnr_change_list = ps - base
        self.importance_ranks, self.T_PSNR_DIFF = importance_ranks(self.psnr_change_list)  # :121-143,198
        return base

    def step(self, action: int) -> StepResult:
        c = self.cfg
        self.steps += 1                                                # env_group.py:221
        ch, r, col = (int(v) for v in decode_action(action, c.height, c.width))
        self.state_record[ch, r, col] += 1                             # env_group.py:231
        self.flip_count += 1
        psnr_after, g, ig, st = self.evaluate_flip(action)
        psnr_change = psnr_after - self.previous_psnr                  # env_group.py:250
        psnr_diff = psnr_after - self.initial_psnr
        closest = int(np.argmin(np.abs(np.asarray(self.psnr_change_list) - psnr_change)))
        reward = float(self.importance_ranks[closest])                 # env_group.py:254-255
        reject = (psnr_change < 0) if self.accept_rule == 0 else not (psnr_change > 0)
        if reject:                                                     # env_group.py:258-263
            self.flip_count -= 1
            return StepResult(action, psnr_after, reward, False, False, False)
        self.state[ch, r, col] ^= 1
        self.intensity[g] = ig
        self.stats = st
        self.max_psnr_diff = max(self.max_psnr_diff, psnr_diff)
        self.previous_psnr = psnr_after                                # env_group.py:281
        if psnr_diff >= self.T_PSNR_DIFF or (psnr_after >= self.T_PSNR and psnr_diff < 0.1):
            self.psnr_sustained_steps += 1                             # env_group.py:292
            if self.psnr_sustained_steps >= self.T_steps and psnr_diff >= self.T_PSNR_DIFF:
                reward += group_linear_bonus(self.steps)               # env_group.py:294-299
        if self.steps >= self.max_steps:
            reward += group_linear_bonus(self.steps)                   # env_group.py:301-315
        terminated = self.steps >= self.max_steps or self.psnr_sustained_steps >= self.T_steps
        truncated = self.steps >= self.max_steps
        return StepResult(action, psnr_after, reward, True, bool(terminated), bool(truncated))


# ---------------------------------------------------------------------------
# DBS drivers
# ---------------------------------------------------------------------------
OUTPUT_BINS = np.round(np.linspace(0, 1.0, 11), decimals=10)   # DBS_1024_24.py:209


def premodel_bin(value: float) -> int:
    """Bin index of a pre-model value: [0,.1),[.1,.2),...,[.9,1.0] (last closed).

    DBS_1024_24.py:289-300,402-416.  Values outside [0,1] map to -1."""
    for i in range(len(OUTPUT_BINS) - 1):
        lo, hi = OUTPUT_BINS[i], OUTPUT_BINS[i + 1]
        if i == len(OUTPUT_BINS) - 2:
            if lo <= value <= hi:
                return i
        elif lo <= value < hi:
            return i
    return -1


def fill_admissible(count: int, target: int, tol: int, bit: int) -> bool:
    """EXTENSION (no reference counterpart -- SURVEY F7; BASELINE configs[4] names a "50 % on-pixel
    constraint"): flipping a pixel whose bit is `bit` moves its colour group's on-pixel count by
    -1 / +1; admissible iff the count ends within `tol` of `target` or closer to it than before."""
    d = -1 if bit else 1
    after = abs(count + d - target)
    return after <= tol or after < abs(count - target)


def group_fill_counts(state: np.ndarray, groups: int) -> np.ndarray:
    """On-pixel count per colour group of an unpacked mask [CH][H][W]."""
    return np.asarray(state, np.int64).reshape(groups, -1).sum(axis=1)


def dbs_greedy(env: OracleEnv, order: Sequence[int], stop_diff: Optional[float] = None, fill=None):
    """Sequential greedy DBS (DBS.py:247-294, DBS_1024_24.py:313-422).

    Accept iff psnr_after > previous_psnr (strict).  Optional early stop once
    psnr - initial >= stop_diff (DBS_ratio_0.5.py:366-372, checked after every
    candidate).  fill = (target count, tol): the on-pixel ratio constraint (extension,
    fill_admissible; an inadmissible candidate is rejected unevaluated, psnr NaN).
    Returns (accepted flags, psnr per candidate, final psnr)."""
    accepted, psnrs = [], []
    counts = None if fill is None else group_fill_counts(env.state, env.cfg.groups)
    for a in order:
        if counts is not None:
            ch, r, col = (int(v) for v in decode_action(a, env.cfg.height, env.cfg.width))
            g = ch // env.cfg.planes
            if not fill_admissible(int(counts[g]), fill[0], fill[1], int(env.state[ch, r, col])):
                accepted.append(False)
                psnrs.append(np.nan)
                continue
        psnr_after, g, ig, st = env.evaluate_flip(int(a))
        ok = psnr_after > env.previous_psnr
        if ok:
            ch, r, col = (int(v) for v in decode_action(a, env.cfg.height, env.cfg.width))
            if counts is not None:
                counts[g] += -1 if env.state[ch, r, col] else 1
            env.state[ch, r, col] ^= 1
            env.intensity[g] = ig
            env.stats = st
            env.previous_psnr = psnr_after
        accepted.append(ok)
        psnrs.append(psnr_after)
        if stop_diff is not None and psnr_after - env.initial_psnr >= stop_diff:
            break
    return np.array(accepted, bool), np.array(psnrs, np.float64), env.previous_psnr


def single_pixel_field(cfg: OpticsConfig, g: int) -> np.ndarray:
    """Field of one unit pixel at (0, 0) after tt.simulate: IFFT2(H_g) (complex128).

    tt.simulate is linear in the field, so flipping pixel (c, r, col)
    of group g adds delta * roll(h_g, (r, col)) to plane c's field, with
    delta = +-1 (amplitude {0,1}) or -+2 (phase {+1,-1}) (env.py:170-172)."""
    return np.fft.ifft2(cfg.transfer(g))


class LinearGreedy:
    """Greedy DBS (DBS_1024_24.py:313-422, accept iff psnr > previous, strict
    :355) evaluated in float64 by linearity instead of re-propagating the
    touched group per candidate: the per-plane fields U_c (complex128) are kept,
    a candidate's field change is delta * h_g shifted to the pixel, and its
    channel sums change by

        d(sum I T)   = sum dI T,        d(sum I^2) = sum (2 I + dI) dI,
        dI = (|U_c + delta h|^2 - |U_c|^2) / P = delta (2 Re(U_c conj h) + delta |h|^2) / P,

    all exact in float64 (tests/test_oracle.py checks it against the
    re-propagating OracleEnv.evaluate_flip).  This makes a 1024x1024x24 greedy
    prefix of thousands of candidates tractable on the CPU (~25 ms per
    candidate instead of two 8-plane 1024^2 FFT sets), which pins the GPU
    accept sequence at the headline size (tests/golden/dbs_prefix_1024x24.npz)."""

    def __init__(self, cfg: OpticsConfig, pre_model: np.ndarray, target: np.ndarray):
        self.cfg = c = cfg
        self.state = (np.asarray(pre_model, np.float32) >= 0.5).astype(np.int8)   # env.py:120
        self.target = np.asarray(target, np.float64).reshape(c.groups, c.height, c.width)
        self.vb = 1.0 if c.field_kind == FIELD_AMPLITUDE else -2.0
        self.h = []
        self.fields = np.empty((c.channels, c.height, c.width), np.complex128)
        self.intensity = np.empty((c.groups, c.height, c.width), np.float64)
        for g in range(c.groups):
            tf = c.transfer(g)
            self.h.append(np.fft.ifft2(tf))
            sl = slice(g * c.planes, (g + 1) * c.planes)
            u = propagate(mask_to_field(self.state[sl], c.field_kind), tf)
            self.fields[sl] = u
            self.intensity[g] = np.mean(u.real * u.real + u.imag * u.imag, axis=0)
        self.stats = np.stack([chan_stats(self.intensity[g], self.target[g]) for g in range(c.groups)])
        self.count = c.groups * c.height * c.width
        self.initial_psnr = self.previous_psnr = self.psnr(self.stats)

    def psnr(self, stats) -> float:
        c = self.cfg
        return psnr_from_stats(stats, self.count, c.rel_scale, c.peak)

    def evaluate(self, action: int):
        """(psnr after the flip, g, ch, delta, shifted h, dI, new stats); state unchanged."""
        c = self.cfg
        ch, r, col = (int(v) for v in decode_action(action, c.height, c.width))
        g = ch // c.planes
        delta = self.vb * (1.0 - 2.0 * float(self.state[ch, r, col]))
        hs = np.roll(self.h[g], (r, col), axis=(0, 1))
        u = self.fields[ch]
        re = u.real * hs.real + u.imag * hs.imag
        di = delta * (2.0 * re + delta * (hs.real * hs.real + hs.imag * hs.imag)) / c.planes
        st = self.stats.copy()
        st[g, 0] += float(np.dot(di.ravel(), self.target[g].ravel()))
        st[g, 1] += float(np.dot((2.0 * self.intensity[g] + di).ravel(), di.ravel()))
        return self.psnr(st), g, ch, delta, hs, di, st

    def commit(self, action: int, ev) -> None:
        c = self.cfg
        _, g, ch, delta, hs, di, st = ev
        _, r, col = (int(v) for v in decode_action(action, c.height, c.width))
        self.state[ch, r, col] ^= 1                                       # DBS_1024_24.py:320
        self.fields[ch] += delta * hs
        self.intensity[g] += di
        self.stats = st                                                   # :358-363
        self.previous_psnr = ev[0]

    def run(self, order: Sequence[int], stop_diff: Optional[float] = None, fill=None):
        """Returns (accepted flags, psnr per candidate, psnr change per candidate
        = psnr - previous psnr at that candidate) over ``order``.  fill = (target count, tol):
        the on-pixel ratio constraint (extension, as dbs_greedy; rejected candidates: NaN)."""
        accepted, psnrs, deltas = [], [], []
        c = self.cfg
        self.fill_counts = None if fill is None else group_fill_counts(self.state, c.groups)
        for a in order:
            if fill is not None:
                ch, r, col = (int(v) for v in decode_action(a, c.height, c.width))
                g = ch // c.planes
                bit = int(self.state[ch, r, col])
                if not fill_admissible(int(self.fill_counts[g]), fill[0], fill[1], bit):
                    accepted.append(False)
                    psnrs.append(np.nan)
                    deltas.append(np.nan)
                    continue
            ev = self.evaluate(int(a))
            ps = ev[0]
            ok = ps > self.previous_psnr                                   # :355 (strict)
            deltas.append(ps - self.previous_psnr)
            if ok:
                if fill is not None:
                    self.fill_counts[g] += -1 if bit else 1
                self.commit(int(a), ev)
            accepted.append(ok)
            psnrs.append(ps)
            if stop_diff is not None and ps - self.initial_psnr >= stop_diff:   # DBS_ratio_0.5.py:366-372
                break
        return np.array(accepted, bool), np.array(psnrs, np.float64), np.array(deltas, np.float64)

    def run_env(self, actions: Sequence[int]):
        """The env step's accept / rollback rule over ``actions`` (env.py:184-214: a flip is
        rolled back iff the PSNR change is negative; the reward 800 * change is returned
        either way, :188).  Returns (accepted flags, psnr after each flip, change against
        the previous accepted state).  No termination within the trace (the caller keeps it
        short of T_PSNR_DIFF)."""
        accepted, psnrs, deltas = [], [], []
        for a in actions:
            ev = self.evaluate(int(a))
            change = ev[0] - self.previous_psnr                            # env.py:184
            ok = not (change < 0)                                          # env.py:191
            if ok:
                self.commit(int(a), ev)
            accepted.append(ok)
            psnrs.append(ev[0])
            deltas.append(change)
        return np.array(accepted, bool), np.array(psnrs, np.float64), np.array(deltas, np.float64)


def probe_sweep(env: OracleEnv, flips: Sequence[int]):
    """Independent flip-evaluate-undo trials against the fixed base
    (DBS_1024_24-128.py:310-373, range.py:294-335, env_group.py:96-120).
    Returns psnr per trial (float64)."""
    return np.array([env.evaluate_flip(int(a))[0] for a in flips], np.float64)


def premodel_histogram(pre_model: np.ndarray, flips: Sequence[int], improved: Sequence[bool],
                       deltas: Sequence[float], height: int, width: int):
    """10-bin attempted / improved / sum-delta histogram (range.py:315-333)."""
    attempted = np.zeros(10, np.int64)
    imp = np.zeros(10, np.int64)
    dsum = np.zeros(10, np.float64)
    ch, r, col = decode_action(np.asarray(flips, np.int64), height, width)
    for k in range(len(flips)):
        b = premodel_bin(float(pre_model[ch[k], r[k], col[k]]))
        if b < 0:
            continue
        attempted[b] += 1
        if improved[k]:
            imp[b] += 1
            dsum[b] += deltas[k]
    return attempted, imp, dsum


def importance_ranks(psnr_changes: np.ndarray):
    """env_group.py:122-143: rank-mapped degree-5 polynomial reward + T_PSNR_DIFF."""
    step_poly = np.array([10000, 9000, 8000, 5000, 2500, 1])
    rewards_poly = np.array([-0.5, -0.48, -0.45, -0.35, 0, 1])
    poly = np.poly1d(np.polyfit(step_poly, rewards_poly, len(step_poly) - 1))
    n = len(psnr_changes)
    order = np.argsort(psnr_changes, kind="stable")
    ranks = np.zeros(n)
    for rank, idx in enumerate(order):
        x_val = 10000 - (10000 - 1) * (rank / (n - 1))
        ranks[idx] = poly(x_val)
    positive_sum = float(np.sum(np.asarray(psnr_changes)[np.asarray(psnr_changes) > 0]))
    return ranks, positive_sum / 4


# ---------------------------------------------------------------------------
# Seeded synthetic inputs
# ---------------------------------------------------------------------------
def synthetic_inputs(cfg: OpticsConfig, seed: int = 0):
    """pre_model ~ U[0,1) (seed), target ~ U[0,1) (seed+1), float32."""
    pre = np.random.default_rng(seed).random((cfg.channels, cfg.height, cfg.width), np.float32)
    tgt = np.random.default_rng(seed + 1).random((cfg.groups, cfg.height, cfg.width), np.float32)
    return pre, tgt


def crop(arr: np.ndarray, margin: int) -> np.ndarray:
    """env_1024_24_128.py:144-149 centre crop of `margin` pixels per side."""
    return arr[..., margin:-margin, margin:-margin]
