"""One process per GPU: shard independent envs, gather per-step metrics to rank 0.

SURVEY 8e: env instances shard with no exchange on the compute path; the
only collective is a small gather of rewards / psnr / done flags to rank 0
(torch.distributed, backend "nccl" = RCCL over xGMI on ROCm; "gloo" in CPU
tests).  Probe sweeps shard the flip range and all-reduce a 10-bin histogram.

Every collective here runs whenever a process group exists, including a
world of one: ``init(force=True)`` (or ``HBX_DIST_FORCE_PG=1``) builds that
group without a launcher, so a one-GPU run executes the same RCCL calls as
the 8-GPU one (train-PPO.py:296-322's caller, BASELINE configs[3]).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def env_rank_world() -> Tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def active() -> bool:
    """A process group exists (any world size): the collectives below run."""
    return dist.is_available() and dist.is_initialized()


def init(backend: Optional[str] = None, force: Optional[bool] = None) -> Tuple[int, int, int]:
    """Initialise the default process group from torchrun's env vars.

    World > 1 always builds the group.  At world 1 the group is built only when
    ``force`` (default: ``HBX_DIST_FORCE_PG=1`` in the environment); without
    torchrun's MASTER_PORT it rendezvouses through an in-process HashStore.
    backend None -> "nccl" (RCCL) when a GPU is visible, else "gloo".  The nccl
    group is bound to cuda:LOCAL_RANK (device_id), so its communicator is
    created eagerly here -- before any other GPU work of the caller."""
    rank, world, local = env_rank_world()
    if force is None:
        force = os.environ.get("HBX_DIST_FORCE_PG") == "1"
    if active() or not (world > 1 or force):
        return rank, world, local
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device("cuda", local)
    if world == 1 and "MASTER_PORT" not in os.environ:
        dist.init_process_group(backend, store=dist.HashStore(), rank=0, world_size=1, **kw)
    else:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend, **kw)
    return rank, world, local


def shutdown():
    if active():
        dist.destroy_process_group()


def backend() -> str:
    return dist.get_backend() if active() else "none"


def collective_device(home: Optional[torch.device] = None) -> torch.device:
    """Where the backend's collectives take their tensors: the current GPU for
    nccl (RCCL), the host for gloo."""
    if backend() == "nccl":
        return home if home is not None and home.type == "cuda" else \
            torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, stop) share of `total` items for `rank` (balanced to +-1)."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_to_rank0(t: torch.Tensor, out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """Concatenate equal-shaped per-rank tensors on rank 0 (None elsewhere):
    one dist.gather, so only rank 0 receives (RCCL send/recv to the root over
    xGMI; gloo on CPU).  ``out`` (rank 0, on the backend's device, shape
    [world * t.shape[0], ...]) receives the rows in place.  Without a process
    group: t itself."""
    if not active():
        return t
    home = t.device
    t = t.contiguous().to(collective_device(home))
    if dist.get_rank() == 0:
        world = dist.get_world_size()
        if out is None or out.device != t.device:
            out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        rows = t.shape[0]
        dist.gather(t, gather_list=[out[r * rows:(r + 1) * rows] for r in range(world)], dst=0)
        return out.to(home)
    dist.gather(t, dst=0)
    return None


class StepMetricGather:
    """Per-step env metrics gathered to rank 0 every ``every`` steps (SURVEY 8e:
    "batch K steps per gather").  Each step owns one byte row of a device buffer
    [every, 19 B] laid out as the step kernel writes its outputs (reward f64[B],
    psnr f64[B], accepted / terminated / truncated u8[B]); slot() hands that row
    to VecEnv.step_device(out=...) so a step costs no packing kernel at all, and
    one dist.gather moves the raw rows (the collective's latency is paid once per
    ``every`` steps).  flush() returns rank 0's [world * every, B, 5] f64 block
    (rank r's rows at [r * every, (r + 1) * every)) or None elsewhere / when empty.

    Measured on the 256x256x8 mono step (B = 128, 0.350 ms): a stack + cast pack
    per step plus a gather every step cost +24 us/step, packing alone ~10 us."""

    def __init__(self, n_env: int, every: int = 1, device=None):
        self.every = max(1, int(every))
        self.n_env = int(n_env)
        row = 19 * self.n_env
        self.row_bytes = -(-row // 8) * 8
        self.raw = torch.zeros((self.every, self.row_bytes), dtype=torch.uint8, device=device)
        self.n = 0
        self.gathered: List[torch.Tensor] = []

    def _views(self, raw_row: torch.Tensor):
        B = self.n_env
        return (raw_row[:8 * B].view(torch.float64), raw_row[8 * B:16 * B].view(torch.float64),
                raw_row[16 * B:17 * B], raw_row[17 * B:18 * B], raw_row[18 * B:19 * B])

    def slot(self):
        """Destinations for the next step's (reward, psnr, accepted, terminated, truncated)."""
        return self._views(self.raw[self.n])

    def add(self, reward, psnr, accepted, terminated, truncated):
        dst = self.slot()
        for s, d in zip((reward, psnr, accepted, terminated, truncated), dst):
            if s.data_ptr() != d.data_ptr():     # not written in place through slot()
                d.copy_(s.reshape(-1))
        self.n += 1
        if self.n == self.every:
            return self.flush()
        return None

    def _decode(self, raw: torch.Tensor) -> torch.Tensor:
        return torch.stack([torch.stack(self._views(r), dim=1).to(torch.float64) for r in raw])

    def flush(self) -> Optional[torch.Tensor]:
        if self.n == 0:
            return None
        got = gather_to_rank0(self.raw[:self.n])
        self.n = 0
        if got is None:
            return None
        out = self._decode(got)      # a fresh tensor: the rows are overwritten by the next steps
        self.gathered.append(out)
        return out


def describe_world(device=None) -> List[List]:
    """[rank, world, local_rank, backend] as every rank saw it, gathered to rank 0
    over the group's own backend (the bench prints it so a multi-GPU line is
    self-checking)."""
    rank, world, local = env_rank_world()
    if active():
        rank, world = dist.get_rank(), dist.get_world_size()
    be = backend()
    row = torch.tensor([rank, world, local], dtype=torch.int64,
                       device=collective_device(torch.device(device) if device is not None else None))
    allr = gather_to_rank0(row.unsqueeze(0))
    if allr is None:
        return []
    return [[int(a), int(b), int(c), be] for a, b, c in allr.cpu().tolist()]


_ID_BYTES = 64      # pci id (16 B) + uuid (48 B) per rank, as 8 int64 words


def device_identity(device=None) -> Tuple[int, str, str]:
    """(torch.cuda.current_device(), PCI address "dddd:bb:dd", uuid) of the GPU this process
    actually runs on; (-1, "cpu", "") without one.  HIP_VISIBLE_DEVICES can renumber the
    devices of a process (every rank may see its GPU as index 0), so the PCI address and the
    uuid are what tell two ranks' GPUs apart."""
    if device is not None and torch.device(device).type != "cuda":
        return -1, "cpu", ""
    if not torch.cuda.is_available():
        return -1, "cpu", ""
    cur = torch.cuda.current_device()
    p = torch.cuda.get_device_properties(cur)
    pci = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    return cur, pci, str(getattr(p, "uuid", ""))


def _id_words(pci: str, uuid: str) -> List[int]:
    raw = pci.encode()[:16].ljust(16, b"\0") + uuid.encode()[:48].ljust(48, b"\0")
    return [int.from_bytes(raw[i:i + 8], "little", signed=True) for i in range(0, _ID_BYTES, 8)]


def _id_strings(words: List[int]) -> Tuple[str, str]:
    raw = b"".join(int(w).to_bytes(8, "little", signed=True) for w in words)
    return raw[:16].rstrip(b"\0").decode(errors="replace"), raw[16:].rstrip(b"\0").decode(errors="replace")


def describe_devices(device=None) -> List[List]:
    """[rank, world, local_rank, backend, device index, PCI address, uuid] as every rank saw
    it, gathered to rank 0 (empty elsewhere): the device each rank ACTUALLY used (its current
    device), not the LOCAL_RANK it was handed.  A multi-GPU bench line carries these rows and
    refuses to report unless they name `world` distinct GPUs (distinct_devices)."""
    rank, world, local = env_rank_world()
    if active():
        rank, world = dist.get_rank(), dist.get_world_size()
    cur, pci, uuid = device_identity(device)
    row = torch.tensor([rank, world, local, cur] + _id_words(pci, uuid), dtype=torch.int64,
                       device=collective_device(torch.device(device) if device is not None else None))
    allr = gather_to_rank0(row.unsqueeze(0))
    if allr is None:
        return []
    out = []
    for r in allr.cpu().tolist():
        p, u = _id_strings(r[4:])
        out.append([int(r[0]), int(r[1]), int(r[2]), backend(), int(r[3]), p, u])
    return out


def distinct_devices(rows: List[List]) -> int:
    """How many different GPUs the describe_devices rows name (by PCI address and uuid;
    CPU-only ranks count as none)."""
    return len({(r[5], r[6]) for r in rows if r[5] != "cpu"})


def pack_step_metrics(reward: torch.Tensor, psnr: torch.Tensor, accepted: torch.Tensor,
                      terminated: torch.Tensor, truncated: torch.Tensor,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One f64 row per env: reward, psnr, accepted, terminated, truncated (<= 40 B/env)."""
    return torch.stack([reward, psnr, accepted, terminated, truncated], dim=1,
                       out=out).to(torch.float64)


def allreduce_hist(counts: torch.Tensor) -> torch.Tensor:
    """Sum `counts` over the ranks in place (on the backend's device; the result
    is copied back when `counts` lives elsewhere)."""
    if not active():
        return counts
    dev = collective_device(counts.device)
    if counts.device == dev:
        dist.all_reduce(counts)
        return counts
    t = counts.to(dev)
    dist.all_reduce(t)
    counts.copy_(t)
    return counts


def max_over_ranks(x: float, device: Optional[torch.device] = None) -> float:
    if not active():
        return x
    t = torch.tensor([x], dtype=torch.float64,
                     device=collective_device(torch.device(device) if device is not None else None))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    if active():
        dist.barrier()
