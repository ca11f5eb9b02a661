"""Direct binary search drivers on the device.

greedy()  -- DBS.py:247-294 / DBS_1024_24.py:313-422: visit pixels in a
             shuffled order, keep a flip iff PSNR strictly improves.  Run as
             SPECULATIVE batches: the next K candidates are evaluated against
             the current base in one launch; the first improving one (in
             visiting order) is committed on the device and the walk resumes
             right after it.  Every candidate before it was evaluated against
             exactly the state the serial loop would have had, so the accept
             sequence is the serial one.  mode="psf" runs the whole walk on the
             device (hbx_dbs_walk_psf: a one-block kernel makes the
             decision, no host round trip per batch); mode="psf_host" and
             mode="fft" return to the host after every batch.
probe()   -- DBS_1024_24-128.py:310-373 / range.py:294-335: every flip
             evaluated against the FIXED base and undone; embarrassingly
             parallel, one launch per max_jobs candidates.
"""
from __future__ import annotations

import ctypes as C
import io
import math
import os
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .env import PLANE_SIZES
from .plan import Plan

OUTPUT_BINS = np.round(np.linspace(0, 1.0, 11), decimals=10)   # DBS_1024_24.py:209


@dataclass
class GreedyResult:
    initial_psnr: float
    final_psnr: float
    steps: int                       # candidates visited (serial-loop `steps`)
    accepted_positions: List[int]    # positions in `order` that were accepted
    accepted_psnr: List[float]
    launches: int
    stopped_early: bool = False
    accept_times: List[float] = field(default_factory=list)   # seconds since start, per accept
    last_psnr: Optional[float] = None    # psnr of the last visited candidate (accepted or not)
    seconds: float = 0.0
    fill_counts: Optional[List[int]] = None   # on-pixel count per colour group at the end (fill_ratio runs)


class KController:
    """Adaptive speculation depth: short batches while flips are often
    accepted, long ones once acceptance becomes rare."""

    def __init__(self, k_min: int = 4, k_max: int = 256, k0: int = 16):
        self.k_min, self.k_max, self.k = k_min, k_max, k0

    def update(self, found_at: Optional[int]):
        if found_at is None:
            self.k = min(self.k_max, self.k * 2)
        else:
            self.k = int(min(self.k_max, max(self.k_min, 2 * (found_at + 1))))
        return self.k


def fill_admissible(count: int, target: int, tol: int, bit: int) -> bool:
    """The on-pixel ratio constraint (an EXTENSION: BASELINE configs[4] names a "50 % on-pixel
    constraint", the reference has none -- SURVEY F7): flipping a pixel whose bit is `bit` moves
    its colour group's on-pixel count by d = -1 / +1; admissible iff |count + d - target| <= tol or
    the flip brings the count closer to the target (hbx_walk_planes.hpp fill_admissible)."""
    d = -1 if bit else 1
    after = abs(count + d - target)
    return after <= tol or after < abs(count - target)


def fill_counts(mask: torch.Tensor, groups: int, planes: int) -> np.ndarray:
    """On-pixel count of each colour group of a packed mask [CH][H][W/64] int64 (host)."""
    b = mask.detach().cpu().contiguous().numpy().view(np.uint8).reshape(groups, -1)
    return np.unpackbits(b, axis=1).sum(axis=1).astype(np.int64)


def fill_target(fill_ratio: float, planes: int, height: int, width: int) -> int:
    """Target on-pixel count of one colour group (P planes of H x W)."""
    return int(round(float(fill_ratio) * planes * height * width))


def first_improving(psnr: np.ndarray, prev: float) -> Optional[int]:
    """Index of the first candidate with psnr > prev (strict, DBS_1024_24.py:355)."""
    idx = np.nonzero(psnr > prev)[0]
    return int(idx[0]) if idx.size else None


def greedy_dataset(n_images: int, load, order_for, plan_factory, per_gpu: int = 4,
                   stop_diff: Optional[float] = None, refresh_every: int = 4096,
                   max_candidates: Optional[int] = None, save_dir: Optional[str] = None):
    """DBS_1024_24.py's loop over a folder of images (`:208-211`, one greedy sweep per
    image) over the ranks of the default process group (a single image's
    walk does not split -- images are the replicas): image i runs on rank i % world,
    each rank runs its images `per_gpu` side by side (greedy_many, one plan each from
    `plan_factory()`), and the per-image summary is gathered to rank 0 with one
    dist.gather (RCCL over xGMI; gloo on CPU).

    load(i) -> (mask bits [CH][H][W/64] int64 on this rank's device, target [G][H][W]);
    order_for(i) -> the candidate order.  save_dir: each rank writes image i's accepted
    positions and PSNRs to save_dir/dbs_image{i}_accepted.npz.  Returns on rank 0 the
    list of per-image dicts in image order (image, initial_psnr, final_psnr, candidates,
    accepted, seconds, stopped_early, rank); None on the other ranks."""
    import torch.distributed as tdist
    from . import dist as hd
    rank, world = 0, 1
    if tdist.is_available() and tdist.is_initialized():
        rank, world = tdist.get_rank(), tdist.get_world_size()
    mine = list(range(rank, n_images, world))
    per_gpu = max(1, int(per_gpu))
    plans = [plan_factory() for _ in range(min(per_gpu, max(1, len(mine))))]
    rows = []
    for c0 in range(0, len(mine), per_gpu):
        chunk = mine[c0:c0 + per_gpu]
        data = [load(i) for i in chunk]
        res = greedy_many(plans[:len(chunk)], [d[0] for d in data], [d[1] for d in data],
                          [order_for(i) for i in chunk], stop_diff=stop_diff, refresh_every=refresh_every,
                          max_candidates=max_candidates, concurrency=per_gpu)
        for i, r in zip(chunk, res):
            rows.append([i, r.initial_psnr, r.final_psnr, r.steps, len(r.accepted_positions), r.seconds,
                         float(r.stopped_early), rank])
            if save_dir is not None:
                os.makedirs(save_dir, exist_ok=True)
                np.savez(os.path.join(save_dir, f"dbs_image{i}_accepted.npz"),
                         positions=np.asarray(r.accepted_positions, np.int64),
                         psnr=np.asarray(r.accepted_psnr, np.float64))
    for pl in plans:
        close = getattr(pl, "close", None)
        if close is not None:
            close()
    # equal shapes for the gather: every rank sends ceil(n / world) rows, padded with image -1
    per_rank = -(-n_images // world)
    buf = torch.full((per_rank, 8), -1.0, dtype=torch.float64)
    if rows:
        buf[:len(rows)] = torch.tensor(rows, dtype=torch.float64)
    got = hd.gather_to_rank0(buf)        # RCCL / gloo whenever a group exists (any world size)
    if got is None:
        return None
    keys = ("image", "initial_psnr", "final_psnr", "candidates", "accepted", "seconds", "stopped_early", "rank")
    out = []
    for row in got.cpu().tolist():
        if row[0] < 0:
            continue
        d = dict(zip(keys, row))
        for k in ("image", "candidates", "accepted", "rank"):
            d[k] = int(d[k])
        d["stopped_early"] = bool(d["stopped_early"])
        out.append(d)
    out.sort(key=lambda d: d["image"])
    return out


def rgb_artifact_paths(file_name: str, dbs_folder: str = "DBS"):
    """The reconstructed-RGB files DBS_1024_24.py writes per image, names verbatim
    (`:283` has 'png' before '_rgb_before', `:447` does not): (before, after)."""
    return (os.path.join(dbs_folder, f"episode_{file_name}png_rgb_before.npy"),
            os.path.join(dbs_folder, f"episode_{file_name}_rgb_after.npy"))


def save_rgb(plan: Plan, mask: torch.Tensor, target: torch.Tensor, path: str, stream=None) -> np.ndarray:
    """np.save of the reconstructed RGB the reference saves before and after its greedy loop
    (DBS_1024_24.py:252-257 + :280-286 / :444-451): per colour group the plane mean of
    |tt.simulate|^2, float32 [1, G, H, W], from one exact propagation of ``mask``.  Prints the
    reference's 'RGB data saved to ...' line; returns the array."""
    inten, _, _ = plan.propagate(mask.unsqueeze(0), target.unsqueeze(0), want_intensity=True, stream=stream)
    if stream is not None:
        stream.synchronize()
    rgb = inten.float().cpu().numpy()                      # [1, G, H, W]
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    np.save(path, rgb)
    print(f"RGB data saved to {path}")
    return rgb


def walk_k(q: float, n: int, k_min: int = 1, k_max: int = 256, fused: bool = True) -> int:
    """Speculation depth of the device walk for acceptance rate q at side n: the K
    minimising (per-batch overhead + K * per-candidate stream time + accepts *
    commit time) / expected candidates visited per batch.

    fused (ABI v7): K in _lib.WALK_FUSED_K is one launch per batch, and for K = 2..4 the
    batch runs to the SECOND accept (visited = sum_{k<=K} P(fewer than 2 accepts in
    the first k-1)), otherwise to the first (sum_{k<=K} (1-q)^(k-1)).  Split (v5):
    three launches, first accept only."""
    c = 16.0 * n * n / 3.7e6          # us: one candidate's 16 B/px (~3.7 TB/s effective, measured)
    cm = 24.0 * n * n / 5.5e6         # us: committing an accepted flip (24 B/px)
    q = min(max(q, 1e-6), 1.0)
    p = 1.0 - q
    best, bk = math.inf, k_min
    for k in range(max(1, k_min), max(k_min, k_max) + 1):
        one_launch = fused and k in _lib.WALK_FUSED_K      # larger K: the split three-launch batch
        two = one_launch and k >= 2
        if two:
            vis = sum(p ** (i - 1) + (i - 1) * q * p ** max(i - 2, 0) for i in range(1, k + 1))
            acc = (1.0 - p ** k) + (1.0 - p ** k - k * q * p ** (k - 1))     # min(2, accepts)
        else:
            vis = (1.0 - p ** k) / q
            acc = 1.0 - p ** k
        # us per batch besides the streaming: launch boundary + arrival + decision tail (one
        # launch, measured 8.5 at 1024 x 24) / three launches
        o = 8.5 if one_launch else 14.0
        cost = (o + k * c + acc * cm) / vis
        if cost < best:
            best, bk = cost, k
    return bk


class _Walk:
    """Host side of one device-resident greedy walk (hbx_dbs_walk_psf).

    Two chunks of `chunk` batches stay in flight: chunk n+1 is enqueued before
    chunk n's state (copied to pinned memory behind it) is read, so the device
    never idles on the host; batches enqueued after the walk is done or halted
    return at once.  Several walks, each on its own stream, can be advanced in
    turn (greedy_many): their latency-bound launches then overlap on the GPU."""

    def __init__(self, plan: Plan, mask, target, order_t, total, stop_diff, k_min, k_max, stream,
                 refresh_every, chunk: int = 64, progress=None, graphs: bool = False):
        self.plan, self.mask, self.target, self.order_t = plan, mask, target, order_t
        self.chunk, self.progress = chunk, progress
        self.use_graphs, self.graphs = graphs, {}
        dev = plan.device
        self.s = s = stream if stream is not None else torch.cuda.current_stream()
        s.wait_stream(torch.cuda.current_stream())    # inputs written on the caller's stream
        with torch.cuda.stream(s):                     # buffers and reads ordered on the walk's stream
            self._setup(plan, mask, target, total, stop_diff, k_min, k_max, refresh_every, dev, s)
        self.issue()
        self.issue()

    def _setup(self, plan, mask, target, total, stop_diff, k_min, k_max, refresh_every, dev, s):
        _, stats, psnr0 = plan.propagate(mask.unsqueeze(0), target.unsqueeze(0), want_intensity=False, stream=s)
        self.base_stats = stats[0].contiguous()
        fc, it = plan.simulate(mask.unsqueeze(0), want_intensity=True, stream=s)
        self.field = torch.view_as_real(fc[0]).contiguous()
        self.inten = it[0].contiguous()
        self.init = float(psnr0.item())
        w = _lib.DbsWalk()
        w.total = total
        w.prev_psnr = w.init_psnr = self.init
        w.last_psnr = math.nan
        w.stop_enabled = 1 if stop_diff is not None else 0
        w.stop_diff = float(stop_diff) if stop_diff is not None else 0.0
        w.refresh_every = int(refresh_every or 0)
        w.commit_ch = -1
        w.commit2_ch1 = 0
        self.st = w
        nbytes = C.sizeof(_lib.DbsWalk)
        self.wbuf = torch.frombuffer(bytearray(bytes(w)), dtype=torch.uint8).to(dev)
        self.cap = max(1, total)
        self.log_pos = torch.empty(self.cap, dtype=torch.int64, device=dev)
        self.log_psnr = torch.empty(self.cap, dtype=torch.float64, device=dev)
        self.pinned = [torch.empty(nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        self.events = [torch.cuda.Event(), torch.cuda.Event()]
        self.k_lo, self.k_hi = max(1, k_min), min(k_max, _lib.WALK_MAX_K)
        self.q, self.pos_prev, self.acc_prev = 0.5, 0, 0
        self.fused = os.environ.get("HBX_WALK_SPLIT", "0") in ("", "0")
        self.k = walk_k(self.q, plan.cfg.height, self.k_lo, self.k_hi, self.fused)
        self.marks = []               # (accepts so far, seconds) per processed chunk
        self.exact = {}               # accept index -> exact PSNR after a refresh
        self.issued = self.done_n = 0
        self.finished = False
        self.t0 = time.perf_counter()

    def _chunk(self, stream):
        self._chunk_n(stream, self.chunk)

    def _chunk_n(self, stream, batches):
        self.plan.dbs_walk_psf(self.mask, self.target, self.base_stats, self.field, self.inten, self.order_t,
                               self.wbuf, self.log_pos, self.log_psnr, self.k, batches, stream=stream)

    def issue(self):
        slot = self.issued % 2
        if not self.use_graphs:
            self._chunk(self.s)
        else:
            # one captured chunk per speculation depth K (the walk buffers never move), replayed
            g = self.graphs.get(self.k)
            if g is None:
                self._chunk(self.s)                        # this chunk runs eagerly
                g = torch.cuda.CUDAGraph()
                if not hasattr(self, "cap_stream"):
                    self.cap_stream = torch.cuda.Stream(device=self.plan.device)   # capture needs a side stream
                with torch.cuda.graph(g, stream=self.cap_stream):
                    self._chunk(None)                      # recorded, not run; replayed on self.s
                self.graphs[self.k] = g
            else:
                with torch.cuda.stream(self.s):
                    g.replay()
        with torch.cuda.stream(self.s):
            self.pinned[slot].copy_(self.wbuf, non_blocking=True)
        self.events[slot].record(self.s)
        self.issued += 1

    def take(self):
        slot = self.done_n % 2
        self.events[slot].synchronize()
        self.done_n += 1
        return walk_state(self.pinned[slot].numpy().tobytes())

    def advance(self):
        """Wait for the oldest chunk in flight, act on its state, refill."""
        if self.finished:
            return
        st = self.st = self.take()
        self.marks.append((int(st.accepted), time.perf_counter() - self.t0))
        if self.progress is not None:
            self.progress(int(st.pos), int(st.accepted), float(st.prev_psnr), self.marks[-1][1])
        dpos, dacc = st.pos - self.pos_prev, st.accepted - self.acc_prev
        if dpos > 0:
            self.q = 0.5 * self.q + 0.5 * (dacc / dpos)
            self.k = walk_k(self.q, self.plan.cfg.height, self.k_lo, self.k_hi, self.fused)
        self.pos_prev, self.acc_prev = st.pos, st.accepted
        if st.halt:
            while self.done_n < self.issued:   # the chunk behind it saw halt: no-ops
                st = self.st = self.take()
            # exact re-propagation bounds the fp32 drift of the incremental updates
            plan, s = self.plan, self.s
            with torch.cuda.stream(s):
                _, stats, ps_exact = plan.propagate(self.mask.unsqueeze(0), self.target.unsqueeze(0),
                                                    want_intensity=False, stream=s)
                self.base_stats.copy_(stats[0])
                fc, it = plan.simulate(self.mask.unsqueeze(0), want_intensity=True, stream=s)
                self.field.copy_(torch.view_as_real(fc[0]))
                self.inten.copy_(it[0])
                st.prev_psnr = float(ps_exact.item())
                st.halt = 0
                st.commit_ch, st.commit2_ch1 = -1, 0     # the mask holds them: the refresh applied them
                self.exact[int(st.accepted) - 1] = st.prev_psnr
                self.wbuf.copy_(torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8))
            if st.done:
                self._finish()
                return
            self.issue()
            self.issue()
            return
        if st.done:
            while self.done_n < self.issued:
                self.take()
            self._finish()
            return
        self.issue()

    def _finish(self):
        # the fused walk step applies a batch's accepted flips in the NEXT launch: one more
        # (commit-only) launch brings field / intensity up to the final mask
        self.k = 1
        self._chunk_n(self.s, 1)
        self.s.synchronize()
        self.finished = True
        self.seconds = time.perf_counter() - self.t0

    def result(self) -> GreedyResult:
        st = self.st
        n_acc = min(int(st.accepted), self.cap)
        self.s.synchronize()
        acc_pos = self.log_pos[:n_acc].cpu().tolist()
        acc_psnr = self.log_psnr[:n_acc].cpu().tolist()
        for i, v in self.exact.items():
            if i < n_acc:
                acc_psnr[i] = v
        acc_t, m = [], 0
        marks = self.marks
        for i in range(n_acc):                # time of the chunk that logged accept i
            while m < len(marks) - 1 and marks[m][0] <= i:
                m += 1
            acc_t.append(marks[m][1] if marks else self.seconds)
        final = acc_psnr[-1] if acc_psnr else self.init
        last = None if math.isnan(st.last_psnr) else float(st.last_psnr)
        return GreedyResult(self.init, final, int(st.pos), acc_pos, acc_psnr, int(st.batches),
                            bool(st.stopped_early), acc_t, last, self.seconds)


def planes_visited(q: float, k: int, groups: int) -> float:
    """Expected candidates a device-decided FFT-mode batch of k visits (hbx_dbs_walk_planes): the
    batch runs until the first candidate of a colour group an accept of this batch has touched
    (each candidate's group uniform over `groups`, accepted with probability q)."""
    dist = [1.0] + [0.0] * groups              # P(m groups touched, batch still running)
    vis = 0.0
    for _ in range(k):
        nxt = [0.0] * (groups + 1)
        for m, pm in enumerate(dist):
            if pm:
                cont = pm * (1.0 - m / groups)
                vis += cont
                nxt[m] += cont * (1.0 - q)
                if m < groups:
                    nxt[m + 1] += cont * q
        dist = nxt
    return vis


# device-walk batch time (us) per speculation depth K at 1024 x 24, decision fused into the last
# pass (r05, tools/dbs_walk_bench.py --k, profiles/r05/dbs_walk_k_r05o.txt; K = 1, 7 interpolated)
_PLANES_BATCH_US = {1: 45.0, 2: 56.4, 3: 72.2, 4: 81.7, 5: 110.0, 6: 121.5, 7: 133.2, 8: 144.9}


def walk_k_planes(q: float, groups: int = 3, k_min: int = 1, k_max: int = 64, table=None,
                  slope: float = 11.7) -> int:
    """Speculation depth of the FFT-mode plane-cached walk for acceptance rate q: K minimising
    the batch time / expected candidates visited (planes_visited).  Batch times from the measured
    table (beyond it, `slope` us per candidate more); the step past K = 4 is the passes' workgroups
    of K candidates no longer fitting the chip at once.  At q = 0.5 it picks K = 4 (34.0k
    candidates/s against 33.3k at K = 3 on the r05 sweep)."""
    tab = _PLANES_BATCH_US if table is None else table
    kmax_t = max(tab)
    q = min(max(q, 1e-6), 1.0)
    # one pass of planes_visited's recursion gives the visited count of every k (the host runs
    # this once per 64-batch chunk: the per-k recomputation, O(k_max^2), took ~12 ms at k_max =
    # 256 and starved the GPU, 260 vs 78 us per batch, profiles/archive/r04/walk_kmax_r04i.txt)
    best, bk = math.inf, k_min
    dist = [1.0] + [0.0] * groups
    vis = 0.0
    for k in range(1, max(k_min, k_max) + 1):
        nxt = [0.0] * (groups + 1)
        for m, pm in enumerate(dist):
            if pm:
                cont = pm * (1.0 - m / groups)
                vis += cont
                nxt[m] += cont * (1.0 - q)
                if m < groups:
                    nxt[m + 1] += cont * q
        dist = nxt
        if k >= max(1, k_min):
            t = tab[k] if k in tab else tab[kmax_t] + slope * (k - kmax_t)
            cost = t / vis
            if cost < best:
                best, bk = cost, k
    return bk


class _PlanesWalk(_Walk):
    """Host side of the device-decided FFT-mode walk (hbx_dbs_walk_planes): the same two
    chunks in flight as _Walk, no refreshes (the FFT mode is exact), K from walk_k_planes.
    fill = (fill_ratio, fill_tol): the on-pixel ratio constraint (hbx_dbs_walk_planes_fill)."""

    def __init__(self, *args, fill=None, **kw):
        self.fill = fill
        super().__init__(*args, **kw)

    def _setup(self, plan, mask, target, total, stop_diff, k_min, k_max, refresh_every, dev, s):
        self.fill_arg = None
        if self.fill is not None:
            c = plan.cfg
            counts = torch.as_tensor(fill_counts(mask, c.groups, c.planes)).to(dev)
            self.fill_arg = (counts, fill_target(self.fill[0], c.planes, c.height, c.width), int(self.fill[1]))
        self.k_hi = max(1, min(k_max, plan.max_jobs, 256))
        self.pool = plan.plane_pool(self.k_hi)
        stats, psnr0 = plan.planes_fill(mask, target, *self.pool, stream=s)
        self.base_stats = stats.contiguous()
        self.init = float(psnr0.item())
        w = _lib.DbsWalk()
        w.total = total
        w.prev_psnr = w.init_psnr = self.init
        w.last_psnr = math.nan
        w.stop_enabled = 1 if stop_diff is not None else 0
        w.stop_diff = float(stop_diff) if stop_diff is not None else 0.0
        w.commit_ch = -1
        self.st = w
        nbytes = C.sizeof(_lib.DbsWalk)
        self.wbuf = torch.frombuffer(bytearray(bytes(w)), dtype=torch.uint8).to(dev)
        self.cap = max(1, total)
        self.log_pos = torch.empty(self.cap, dtype=torch.int64, device=dev)
        self.log_psnr = torch.empty(self.cap, dtype=torch.float64, device=dev)
        self.pinned = [torch.empty(nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        self.events = [torch.cuda.Event(), torch.cuda.Event()]
        self.k_lo = max(1, k_min)
        self.q, self.pos_prev, self.acc_prev = 0.5, 0, 0
        self.fused = False
        self.k = walk_k_planes(self.q, plan.cfg.groups, self.k_lo, self.k_hi)
        self.marks, self.exact = [], {}
        self.issued = self.done_n = 0
        self.finished = False
        self.t0 = time.perf_counter()

    def _chunk_n(self, stream, batches):
        self.plan.dbs_walk_planes(self.mask, self.target, self.base_stats, *self.pool, self.order_t, self.wbuf,
                                  self.log_pos, self.log_psnr, self.k, batches, stream=stream, fill=self.fill_arg)

    def result(self) -> GreedyResult:
        r = super().result()
        if self.fill_arg is not None:
            r.fill_counts = [int(v) for v in self.fill_arg[0].cpu().tolist()]
        return r

    def advance(self):
        if self.finished:
            return
        st = self.st = self.take()
        self.marks.append((int(st.accepted), time.perf_counter() - self.t0))
        if self.progress is not None:
            self.progress(int(st.pos), int(st.accepted), float(st.prev_psnr), self.marks[-1][1])
        dpos, dacc = st.pos - self.pos_prev, st.accepted - self.acc_prev
        if dpos > 0:
            self.q = 0.5 * self.q + 0.5 * (dacc / dpos)
            self.k = walk_k_planes(self.q, self.plan.cfg.groups, self.k_lo, self.k_hi)
        self.pos_prev, self.acc_prev = st.pos, st.accepted
        if st.done:
            while self.done_n < self.issued:
                self.take()
            self.s.synchronize()
            self.finished = True
            self.seconds = time.perf_counter() - self.t0
            return
        self.issue()


def _greedy_walk(plan: Plan, mask, target, order_t, total, stop_diff, k_min, k_max, stream,
                 refresh_every, chunk: int = 64, progress=None, graphs: bool = False) -> GreedyResult:
    """greedy(mode="psf") on the device-resident walk (hbx_dbs_walk_psf)."""
    w = _Walk(plan, mask, target, order_t, total, stop_diff, k_min, k_max, stream, refresh_every, chunk,
              progress, graphs)
    while not w.finished:
        w.advance()
    return w.result()


_STREAMS = {}


def walk_state(raw: bytes) -> "_lib.DbsWalk":
    """The hbx_dbs_walk_t a walk chunk left (read back through pinned memory); raises when
    the state is faulted -- a persistent launch's grid barrier timed out (hbx.h: fault; the
    abort word is folded into the state once the grid has drained, k_walk_abort_fold)."""
    st = _lib.DbsWalk.from_buffer_copy(raw)
    if st.fault:
        raise RuntimeError("hbx_dbs_walk_psf: persistent walk barrier timed out; walk state unreliable "
                           "(rerun with HBX_WALK_PERSIST=0)")
    return st


def _walk_stream(device, i: int):
    """The stream of side-by-side walk i.  Default: a fresh torch stream per walk per call
    (measured at 1024x24, 32,768 candidates per image: 2 walks 95k, 3 walks 178k, 4 walks
    190k candidates/s aggregate).  HBX_WALK_STREAMS=n: walk i on stream i % n of a per-device
    pool created in one go (2 walks 154k, 3 walks 180k, 4 walks 148k) -- better for two
    images, worse for the default four (profiles/archive/r02_walk/walk_streams.txt)."""
    dev = torch.device(device)
    n = os.environ.get("HBX_WALK_STREAMS", "")
    if not n.isdigit() or int(n) < 1:
        return torch.cuda.Stream(device=dev)
    pool = _STREAMS.get(dev)
    if pool is None or len(pool) != int(n):
        pool = _STREAMS[dev] = [torch.cuda.Stream(device=dev) for _ in range(int(n))]
    return pool[i % len(pool)]


def greedy_many(plans: Sequence[Plan], masks: Sequence[torch.Tensor], targets: Sequence[torch.Tensor], orders,
                stop_diff: Optional[float] = None, k_max: Optional[int] = None,
                max_candidates: Optional[int] = None, refresh_every: int = 4096,
                concurrency: int = 4, mode: str = "psf", fill_ratio: Optional[float] = None,
                fill_tol: int = 1) -> List[GreedyResult]:
    """DBS_1024_24.py's loop over several images (`:208-211`), up to `concurrency`
    images' greedy walks side by side: walk i on plans[i] (one plan per image:
    its own workspace, tables and walk buffers) and its own HIP stream, the host
    advancing the walks in turn, so their latency-bound launches overlap on the
    GPU (1024x24: 188k candidates/s over 4 walks against 97k for one, r02; 8
    walks 191k).  mode "psf": the incremental-field walks (each result exactly
    greedy(mode="psf") on that image alone); "fft": the FFT-mode walks on the plane cache
    (hbx_dbs_walk_planes; each result exactly greedy(mode="fft") on that image alone).
    fill_ratio / fill_tol (mode="fft" only): the on-pixel ratio constraint of greedy() (an
    extension, hbx_dbs_walk_planes_fill).  Masks are modified in place."""
    if mode not in ("psf", "fft"):
        raise ValueError(f"greedy_many: mode must be 'psf' or 'fft', got {mode!r}")
    if fill_ratio is not None and mode != "fft":
        raise ValueError("fill_ratio: the on-pixel constraint is built for mode='fft' only")
    if not (len(plans) == len(masks) == len(targets) == len(orders)):
        raise ValueError("one plan, mask, target and order per image")
    step = max(1, int(concurrency))
    for g0 in range(0, len(plans), step):
        # each walk writes its plan's walk partials and job workspace from its own stream
        if len({id(p) for p in plans[g0:g0 + step]}) < len(plans[g0:g0 + step]):
            raise ValueError("greedy_many: walks running side by side need distinct Plan objects")
    results: List[GreedyResult] = []
    for g0 in range(0, len(plans), step):
        walks = []
        for plan, mask, target, order in zip(plans[g0:g0 + step], masks[g0:g0 + step], targets[g0:g0 + step],
                                             orders[g0:g0 + step]):
            order_t = torch.as_tensor(np.asarray(order, np.int64)).to(plan.device)
            total = int(order_t.shape[0]) if max_candidates is None else min(int(order_t.shape[0]), max_candidates)
            if total == 0:                     # nothing to visit (the device walks take a non-empty order)
                walks.append(greedy(plan, mask, target, [], mode="fft" if mode == "fft" else "psf",
                                    fill_ratio=fill_ratio, fill_tol=fill_tol))
            elif mode == "fft":
                km = min(k_max or plan.max_jobs, plan.max_jobs)
                walks.append(_PlanesWalk(plan, mask, target, order_t, total, stop_diff, 1, km,
                                         _walk_stream(plan.device, len(walks)), 0,
                                         fill=None if fill_ratio is None else (fill_ratio, fill_tol)))
            else:
                walks.append(_Walk(plan, mask, target, order_t, total, stop_diff, 1, k_max or _lib.WALK_MAX_K,
                                   _walk_stream(plan.device, len(walks)), refresh_every))
        live = [w for w in walks if not isinstance(w, GreedyResult)]
        while not all(w.finished for w in live):
            for w in live:
                w.advance()
        torch.cuda.synchronize()
        results.extend(w if isinstance(w, GreedyResult) else w.result() for w in walks)
    return results


def greedy(plan: Plan, mask: torch.Tensor, target: torch.Tensor, order, stop_diff: Optional[float] = None,
           k_min: Optional[int] = None, k_max: Optional[int] = None, max_candidates: Optional[int] = None,
           stream=None, mode: str = "fft", refresh_every: int = 4096, progress=None,
           graphs: bool = False, planes: Optional[bool] = None, device_walk: Optional[bool] = None,
           fill_ratio: Optional[float] = None, fill_tol: int = 1) -> GreedyResult:
    """mask [CH][H][W/64] int64 (modified in place), target [G][H][W] f32.

    mode="fft": every candidate is the FFT-mode propagation of its colour group
    (DBS_1024_24.py:326-332).  planes (default: on at N = 1024 / 256) keeps the base
    state's per-plane |U_p|^2 (hbx_eval_flips_planes, ABI v10): a candidate propagates
    only its flipped plane's pair and sums the cached planes in the same order, so its
    PSNR -- and the accept sequence -- is the full re-propagation's bit for bit;
    planes=False re-propagates all P planes of the group per candidate.  device_walk (default:
    on with planes) decides each batch on the device (hbx_dbs_walk_planes: no host round trip
    per batch, the host reads the walk state every 64 batches); False decides on the host.
    mode="psf": candidates are evaluated on the incremental-field path, the
    whole walk device-resident (hbx_dbs_walk_psf); the base fields are
    re-propagated exactly every ``refresh_every`` accepted flips.
    mode="psf_host": the same candidates through hbx_eval_flips_psf /
    hbx_commit_flip_psf with a host decision per batch.
    progress(pos, accepted, prev_psnr, seconds): optional callback per chunk of
    the device walk (mode="psf").
    k_min / k_max bound the speculation depth K (candidates per batch): the device walks pick K
    from the running acceptance rate within [k_min (default 1), k_max]; host-decided batches
    (device_walk=False, mode="psf_host") grow K from k_min (default 4).  graphs=True replays the
    incremental walk's chunks from HIP graphs (mode="psf"); the FFT-mode device walk has no
    graph variant and refuses it.
    fill_ratio (EXTENSION, mode="fft" only; BASELINE configs[4]'s "50 % on-pixel constraint", which
    the reference does not have -- SURVEY F7): a candidate whose flip would move its colour group's
    on-pixel count away from round(fill_ratio * P * H * W) by more than fill_tol pixels is visited
    and rejected without a propagation (fill_admissible); the result's fill_counts are the final
    per-group counts.  Device walk: hbx_dbs_walk_planes_fill; host-decided batches: the same rule
    on the host, so both give the same accept sequence."""
    if mode not in ("fft", "psf", "psf_host"):
        raise ValueError(f"mode must be 'fft', 'psf' or 'psf_host', got {mode!r}")
    if fill_ratio is not None:
        if mode != "fft":
            raise ValueError("fill_ratio: the on-pixel constraint is built for mode='fft' only")
        if not (0.0 <= float(fill_ratio) <= 1.0) or int(fill_tol) < 0:
            raise ValueError("fill_ratio must be in [0, 1] and fill_tol >= 0")
    dev = plan.device
    if len(order) == 0 or max_candidates == 0:
        # nothing to visit: the serial loop's result over zero candidates (the device walks take
        # a non-empty order)
        _, _, p0 = plan.propagate(mask.unsqueeze(0), target.unsqueeze(0), want_intensity=False, stream=stream)
        init = float(p0.item())
        fc = None if fill_ratio is None else [int(v) for v in fill_counts(mask, plan.cfg.groups, plan.cfg.planes)]
        return GreedyResult(init, init, 0, [], [], 0, fill_counts=fc)
    if mode == "psf":
        order_t = torch.as_tensor(np.asarray(order, np.int64)).to(dev)
        total = int(order_t.shape[0]) if max_candidates is None else min(int(order_t.shape[0]), max_candidates)
        return _greedy_walk(plan, mask, target, order_t, total, stop_diff, k_min or 1, k_max or _lib.WALK_MAX_K,
                            stream, refresh_every, progress=progress, graphs=graphs)
    mode = "psf" if mode == "psf_host" else mode
    k_max = min(k_max or plan.max_jobs, plan.max_jobs)
    order_t = torch.as_tensor(np.asarray(order, np.int64)).to(dev)
    total = int(order_t.shape[0]) if max_candidates is None else min(int(order_t.shape[0]), max_candidates)
    if planes is None:
        planes = mode == "fft" and plan.cfg.height in PLANE_SIZES
    if planes and (mode != "fft" or plan.cfg.height not in PLANE_SIZES):
        raise ValueError("planes=True is the FFT mode's plane cache at N = 1024 / 896 / 256")
    if device_walk is None:
        device_walk = planes
    if device_walk:
        if not planes:
            raise ValueError("device_walk=True runs on the plane cache (planes=True)")
        if graphs:
            raise ValueError("graphs=True: the FFT-mode device walk has no graph variant (device_walk=False "
                             "for host-decided batches, or mode='psf')")
        w = _PlanesWalk(plan, mask, target, order_t, total, stop_diff, k_min or 1, k_max, stream, 0,
                        progress=progress, fill=None if fill_ratio is None else (fill_ratio, fill_tol))
        while not w.finished:
            w.advance()
        return w.result()
    pool = None
    if planes:
        pool = plan.plane_pool(k_max)
        stats, psnr0 = plan.planes_fill(mask, target, *pool, stream=stream)
        stats = stats.unsqueeze(0)
    else:
        _, stats, psnr0 = plan.propagate(mask.unsqueeze(0), target.unsqueeze(0), want_intensity=False,
                                         stream=stream)
    base_stats = stats[0].contiguous()
    prev_dev = psnr0.clone()
    field = inten = None
    if mode == "psf":
        fc, it = plan.simulate(mask.unsqueeze(0), want_intensity=True, stream=stream)
        field = torch.view_as_real(fc[0]).contiguous()
        inten = it[0].contiguous()
    init = float(psnr0.item())
    prev = init
    psnr_buf = torch.empty(k_max, dtype=torch.float64, device=dev)
    gst_buf = torch.empty((k_max, 3), dtype=torch.float64, device=dev)
    kdev = torch.empty(1, dtype=torch.int32, device=dev)
    ctl = KController(k_min=4 if k_min is None else k_min, k_max=k_max, k0=min(16, k_max))
    pos, launches = 0, 0
    acc_pos, acc_psnr, acc_t = [], [], []
    stopped = False
    last = None
    fill = None
    if fill_ratio is not None:           # host mirror of the bits and the per-group counts
        c = plan.cfg
        bits = np.unpackbits(mask.detach().cpu().contiguous().numpy().view(np.uint8),
                             bitorder="little").reshape(c.channels, c.height, c.width)
        fill = (bits, fill_counts(mask, c.groups, c.planes),
                fill_target(fill_ratio, c.planes, c.height, c.width), int(fill_tol))
        order_np = np.asarray(order, np.int64)
    t0 = time.perf_counter()
    while pos < total:
        k = min(ctl.k, total - pos)
        flips = order_t[pos:pos + k]
        if mode == "psf":
            plan.eval_flips_psf(mask, target, base_stats, field, inten, flips, psnr_buf[:k], gst_buf[:k],
                                stream=stream)
        elif pool is not None:
            plan.eval_flips_planes(mask, target, base_stats, *pool, flips, psnr_buf[:k], gst_buf[:k],
                                   stream=stream)
        else:
            plan.eval_flips(mask, target, base_stats, flips, psnr_buf[:k], gst_buf[:k], stream=stream)
        launches += 1
        ps = psnr_buf[:k].cpu().numpy()
        if fill is not None:                 # inadmissible candidates: visited, rejected, no PSNR
            bits, counts, f_t, f_tol = fill
            c = plan.cfg
            ps = ps.copy()
            for j in range(k):
                a = int(order_np[pos + j])
                ch, rem = divmod(a, c.height * c.width)
                r, col = divmod(rem, c.width)
                if not fill_admissible(int(counts[ch // c.planes]), f_t, f_tol, int(bits[ch, r, col])):
                    ps[j] = np.nan
        i = first_improving(ps, prev)
        ctl.update(i)
        if i is None:
            last = None if math.isnan(ps[k - 1]) else float(ps[k - 1])
            pos += k
            continue
        last = float(ps[i])
        if fill is not None:
            a = int(order_np[pos + i])
            ch, rem = divmod(a, c.height * c.width)
            r, col = divmod(rem, c.width)
            fill[1][ch // c.planes] += -1 if bits[ch, r, col] else 1
            bits[ch, r, col] ^= 1
        kdev.fill_(i)
        if mode == "psf":
            plan.commit_flip_psf(mask, base_stats, prev_dev, field, inten, flips, psnr_buf, gst_buf, kdev,
                                 stream=stream)
        elif pool is not None:
            plan.commit_flip_planes(mask, base_stats, prev_dev, *pool, flips, psnr_buf[:k], gst_buf[:k], kdev,
                                    stream=stream)
        else:
            plan.commit_flip(mask, base_stats, prev_dev, flips, psnr_buf, gst_buf, kdev, stream=stream)
        prev = float(ps[i])
        if mode == "psf" and refresh_every and (len(acc_pos) + 1) % refresh_every == 0:
            # exact re-propagation bounds the fp32 drift of the incremental updates
            _, stats, ps_exact = plan.propagate(mask.unsqueeze(0), target.unsqueeze(0), want_intensity=False,
                                                stream=stream)
            base_stats.copy_(stats[0])
            prev_dev.copy_(ps_exact)
            fc, it = plan.simulate(mask.unsqueeze(0), want_intensity=True, stream=stream)
            field.copy_(torch.view_as_real(fc[0]))
            inten.copy_(it[0])
            prev = float(ps_exact.item())
        acc_pos.append(pos + i)
        acc_psnr.append(prev)
        acc_t.append(time.perf_counter() - t0)
        pos += i + 1
        if stop_diff is not None and prev - init >= stop_diff:      # DBS_ratio_0.5.py:366-372
            stopped = True
            break
    return GreedyResult(init, prev, pos, acc_pos, acc_psnr, launches, stopped, acc_t, last,
                        time.perf_counter() - t0,
                        fill_counts=None if fill is None else [int(v) for v in fill[1]])


def greedy_report(res: GreedyResult, order, pre_model: np.ndarray, height: int, width: int,
                  file_name: str = "image", print_every: float = 0.1) -> str:
    """The console report of DBS_1024_24.py:302-470 for a greedy run, in the
    exact line formats log_py/DBS_psnr_log.py and log_py/com.py parse: a Step
    block each time the PSNR crosses initial + k * print_every (with the
    pre-model range statistics accumulated so far), then the final block.
    Range statistics follow the reference's bookkeeping: the per-bin pixel
    counts of the whole pre-model, incremented again for every accepted flip."""
    out = io.StringIO()
    pm = np.asarray(pre_model, np.float64)
    order = np.asarray(order, np.int64)
    bins = np.zeros(10, np.int64)
    for i in range(10):
        lo, hi = OUTPUT_BINS[i], OUTPUT_BINS[i + 1]
        bins[i] = np.logical_and(pm >= lo, pm <= hi if i == 9 else pm < hi).sum()
    improved = np.zeros(10, np.int64)
    gains = [[] for _ in range(10)]
    thresholds = [res.initial_psnr + i * print_every for i in range(1, 101)]
    hw = height * width

    def coords(a):
        c = int(a) // hw
        k = int(a) % hw
        return c, k // width, k % width

    def range_lines():
        tot_imp = int(improved.sum())
        for i in range(10):
            tc, ic = int(bins[i]), int(improved[i])
            r_in = ic / tc if tc > 0 else 0
            r_tot = ic / tot_imp if tot_imp > 0 else 0
            s_g = sum(gains[i]) if ic > 0 else 0
            avg = s_g / ic if ic > 0 else 0
            print(f"Range {OUTPUT_BINS[i]:.1f}-{OUTPUT_BINS[i + 1]:.1f}: "
                  f"Total Pixels = {tc}, Improved Pixels = {ic}, "
                  f"Improvement Ratio (in range) = {r_in:.6f}, "
                  f"Improvement Ratio (to total improved) = {r_tot:.6f}, "
                  f"Total PSNR Improvement = {s_g:.6f}, "
                  f"Average PSNR Improvement = {avg:.8f}", file=out)

    print(f"Starting pixel flip optimization for file {file_name}.png with initial PSNR: "
          f"{res.initial_psnr:.6f}", file=out)
    prev = res.initial_psnr
    for n, (p, ps) in enumerate(zip(res.accepted_positions, res.accepted_psnr)):
        steps, flips = p + 1, n + 1
        c, r, col = coords(order[p])
        t = res.accept_times[n] if n < len(res.accept_times) else res.seconds
        while thresholds and ps >= thresholds[0]:                  # DBS_1024_24.py:366-396
            thresholds.pop(0)
            print(f"Step: {steps}"
                  f"\nPSNR Before: {prev:.6f} | PSNR After: {ps:.6f} | Change: {ps - prev:.6f} | "
                  f"Diff: {ps - res.initial_psnr:.6f}"
                  f"\nSuccess Ratio: {flips / steps:.6f} | Flip Count: {flips}"
                  f"\nFlip Pixel: Channel={c}, Row={r}, Col={col}"
                  f"\nTime taken for this data: {t:.2f} seconds", file=out)
            range_lines()
            print("\n", file=out)
        v = pm[c, r, col]                                          # DBS_1024_24.py:399-416
        for i in range(10):
            lo, hi = OUTPUT_BINS[i], OUTPUT_BINS[i + 1]
            if (lo <= v <= hi) if i == 9 else (lo <= v < hi):
                bins[i] += 1
                improved[i] += 1
                gains[i].append(ps - prev)
                break
        prev = ps
    steps = max(res.steps, 1)
    last = res.last_psnr if res.last_psnr is not None else res.final_psnr
    diff = last - res.initial_psnr
    c, r, col = coords(order[res.steps - 1]) if res.steps > 0 else (0, 0, 0)
    print(f"Step: {res.steps}"                                      # DBS_1024_24.py:425-470
          f"\nPSNR Before: {prev:.6f} | PSNR After: {last:.6f} | Change: {diff:.6f}"
          f"\nSuccess Ratio: {len(res.accepted_positions) / steps:.6f} | "
          f"Flip Count: {len(res.accepted_positions)}"
          f"\nFlip Pixel: Channel={c}, Row={r}, Col={col}"
          f"\nTime taken for this data: {res.seconds:.2f} seconds", file=out)
    print(f"{file_name}.png Optimization completed. Final PSNR improvement: {diff:.6f}", file=out)
    print(f"Time taken for this data: {res.seconds:.2f} seconds\n", file=out)
    print("Pre-model output range statistics:", file=out)
    range_lines()
    print("\n", file=out)
    return out.getvalue()


@dataclass
class ProbeResult:
    base_psnr: float
    psnr: np.ndarray                 # per flip
    improved: np.ndarray             # psnr > base (strict)
    attempted_bins: np.ndarray = field(default_factory=lambda: np.zeros(10, np.int64))
    improved_bins: np.ndarray = field(default_factory=lambda: np.zeros(10, np.int64))
    delta_bins: np.ndarray = field(default_factory=lambda: np.zeros(10, np.float64))
    shard: Optional[tuple] = None            # probe_sharded: this rank's [lo, hi) of the flips
    improved_total: Optional[int] = None     # probe_sharded: improved flips over all ranks


def premodel_bins(values: np.ndarray) -> np.ndarray:
    """[0,.1),...,[.8,.9),[.9,1.0] -> 0..9; outside -> -1 (DBS_1024_24.py:289-300)."""
    v = np.asarray(values, np.float64)
    b = np.full(v.shape, -1, np.int64)
    for i in range(10):
        lo, hi = OUTPUT_BINS[i], OUTPUT_BINS[i + 1]
        sel = (v >= lo) & ((v <= hi) if i == 9 else (v < hi))
        b[sel & (b < 0)] = i
    return b


def probe(plan: Plan, mask: torch.Tensor, target: torch.Tensor, flips, pre_model: Optional[np.ndarray] = None,
          stream=None) -> ProbeResult:
    dev = plan.device
    flips_t = torch.as_tensor(np.asarray(flips, np.int64)).to(dev)
    _, stats, psnr0 = plan.propagate(mask.unsqueeze(0), target.unsqueeze(0), want_intensity=False,
                                     stream=stream)
    base = float(psnr0.item())
    out = torch.empty(flips_t.shape[0], dtype=torch.float64, device=dev)
    gst = torch.empty((flips_t.shape[0], 3), dtype=torch.float64, device=dev)
    plan.eval_flips(mask, target, stats[0].contiguous(), flips_t, out, gst, stream=stream)
    ps = out.cpu().numpy()
    improved = ps > base
    res = ProbeResult(base, ps, improved)
    if pre_model is not None:
        c = plan.cfg
        f = np.asarray(flips, np.int64)
        ch, k = f // (c.height * c.width), f % (c.height * c.width)
        vals = np.asarray(pre_model)[ch, k // c.width, k % c.width]
        bins = premodel_bins(vals)
        for i in range(10):
            sel = bins == i
            res.attempted_bins[i] = int(sel.sum())
            res.improved_bins[i] = int((sel & improved).sum())
            res.delta_bins[i] = float(np.sum((ps - base)[sel & improved]))
    return res


def probe_sharded(plan: Plan, mask: torch.Tensor, target: torch.Tensor, flips, pre_model=None,
                  stream=None) -> ProbeResult:
    """The probe sweep of DBS_1024_24-128.py:310-373 / range.py:294-335 split across
    the ranks of the default process group: rank r evaluates its
    contiguous share of `flips` (hbx.dist.shard_range) against the same fixed
    base, then the 10-bin pre-model histogram (attempted, improved, summed
    PSNR gain) and the improved count are all-reduced (RCCL over xGMI on GPUs,
    gloo on CPU) -- the only exchange.  Returns the global histogram on every
    rank; `psnr` / `improved` hold this rank's share (positions lo..hi of
    `flips`, given by the returned `.shard`)."""
    from . import dist as hd
    flips = np.asarray(flips, np.int64)
    rank, world = 0, 1
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        rank, world = torch.distributed.get_rank(), torch.distributed.get_world_size()
    lo, hi = hd.shard_range(len(flips), rank, world)
    res = probe(plan, mask, target, flips[lo:hi], pre_model=pre_model, stream=stream)
    # histogram rows + improved count in one f64 all-reduce (device of the collective's backend;
    # runs whenever a process group exists, world 1 included)
    buf = torch.zeros(31, dtype=torch.float64, device=hd.collective_device(plan.device))
    buf[0:10] = torch.as_tensor(res.attempted_bins, dtype=torch.float64)
    buf[10:20] = torch.as_tensor(res.improved_bins, dtype=torch.float64)
    buf[20:30] = torch.as_tensor(res.delta_bins, dtype=torch.float64)
    buf[30] = float(np.count_nonzero(res.improved))
    hd.allreduce_hist(buf)
    out = buf.cpu().numpy()
    res.attempted_bins = out[0:10].round().astype(np.int64)
    res.improved_bins = out[10:20].round().astype(np.int64)
    res.delta_bins = out[20:30].copy()
    res.shard = (lo, hi)
    res.improved_total = int(round(out[30]))
    return res


def probe_map(plan: Plan, mask: torch.Tensor, target: torch.Tensor, flips=None,
              pre_model=None, stream=None) -> ProbeResult:
    """The probe sweep from the all-flip PSNR-change map (hbx_flip_map):
    every flip of the fixed base at once, then the requested ``flips`` (or all
    CH*H*W of them) read out of the map.  Same result fields as probe();
    the pre-model histogram is binned on the device."""
    dev = plan.device
    dmap, base_t = plan.flip_map(mask, target, stream=stream)
    base = float(base_t.item())
    flat = dmap.reshape(-1)
    if flips is None:
        idx = None
        delta = flat.double()
    else:
        idx = torch.as_tensor(np.asarray(flips, np.int64)).to(dev)
        delta = flat[idx].double()
    improved = delta > 0
    res = ProbeResult(base, (delta + base).cpu().numpy(), improved.cpu().numpy())
    if pre_model is not None:
        pm = torch.as_tensor(np.asarray(pre_model, np.float32)).to(dev).reshape(-1)
        vals = (pm if idx is None else pm[idx]).double()
        edges = torch.as_tensor(OUTPUT_BINS[1:10], dtype=torch.float64, device=dev)
        bins = torch.bucketize(vals, edges, right=True)
        bins = torch.where((vals < 0) | (vals > 1.0), torch.full_like(bins, -1), bins)
        ok = bins >= 0
        b = bins.clamp(min=0)
        att = torch.zeros(10, dtype=torch.int64, device=dev).index_add_(0, b[ok], torch.ones_like(b[ok]))
        sel = ok & improved
        imp = torch.zeros(10, dtype=torch.int64, device=dev).index_add_(0, b[sel], torch.ones_like(b[sel]))
        dsum = torch.zeros(10, dtype=torch.float64, device=dev).index_add_(0, b[sel], delta[sel])
        res.attempted_bins = att.cpu().numpy()
        res.improved_bins = imp.cpu().numpy()
        res.delta_bins = dsum.cpu().numpy()
    return res
