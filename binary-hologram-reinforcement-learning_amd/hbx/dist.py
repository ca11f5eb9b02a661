"""One process per GPU: shard independent envs, gather per-step metrics to rank 0.

SURVEY 8e: env instances shard with no exchange on the compute path; the
only collective is a small gather of rewards / psnr / done flags to rank 0
(torch.distributed, backend "nccl" = RCCL over xGMI on ROCm; "gloo" in CPU
tests).  Probe sweeps shard the flip range and all-reduce a 10-bin histogram.
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


def init(backend: Optional[str] = None) -> Tuple[int, int, int]:
    """Initialise the default process group from torchrun's env vars (no-op at world 1)."""
    rank, world, local = env_rank_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, stop) share of `total` items for `rank` (balanced to +-1)."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_to_rank0(t: torch.Tensor) -> Optional[torch.Tensor]:
    """Concatenate equal-shaped per-rank tensors on rank 0 (None elsewhere):
    one dist.gather, so only rank 0 receives (RCCL send/recv to the root over
    xGMI; gloo on CPU)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return t
    home = t.device
    t = t.contiguous()
    if dist.get_backend() == "gloo" and t.is_cuda:   # gloo's gather takes host tensors
        t = t.cpu()
    if dist.get_rank() == 0:
        parts: List[torch.Tensor] = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.gather(t, gather_list=parts, dst=0)
        return torch.cat(parts).to(home)
    dist.gather(t, dst=0)
    return None


class StepMetricGather:
    """Per-step env metrics gathered to rank 0 every ``every`` steps (SURVEY 8e:
    "batch K steps per gather"): rows accumulate in a device buffer [every, B, 5]
    and one dist.gather moves them, so the collective's latency is paid once per
    ``every`` steps.  flush() returns rank 0's [world * every, B, 5] block (rank
    r's rows at [r * every, (r + 1) * every)) or None elsewhere / when empty."""

    def __init__(self, n_env: int, every: int = 1, device=None):
        self.every = max(1, int(every))
        self.buf = torch.zeros((self.every, n_env, 5), dtype=torch.float64, device=device)
        self.n = 0
        self.gathered: List[torch.Tensor] = []

    def add(self, reward, psnr, accepted, terminated, truncated):
        self.buf[self.n] = pack_step_metrics(reward, psnr, accepted, terminated, truncated)
        self.n += 1
        if self.n == self.every:
            return self.flush()
        return None

    def flush(self) -> Optional[torch.Tensor]:
        if self.n == 0:
            return None
        out = gather_to_rank0(self.buf[:self.n])
        self.n = 0
        if out is not None:
            self.gathered.append(out)
        return out


def describe_world(device=None) -> List[List]:
    """[rank, world, local_rank, backend] as every rank saw it, gathered to rank 0
    (the bench prints it so a multi-GPU line is self-checking)."""
    rank, world, local = env_rank_world()
    backend = dist.get_backend() if dist.is_initialized() else "none"
    row = torch.tensor([rank, world, local], dtype=torch.int64,
                       device=device if backend == "nccl" else "cpu")
    allr = gather_to_rank0(row.unsqueeze(0))
    if allr is None:
        return []
    return [[int(a), int(b), int(c), backend] for a, b, c in allr.cpu().tolist()]


def pack_step_metrics(reward: torch.Tensor, psnr: torch.Tensor, accepted: torch.Tensor,
                      terminated: torch.Tensor, truncated: torch.Tensor) -> torch.Tensor:
    """One f64 row per env: reward, psnr, accepted, terminated, truncated (<= 40 B/env)."""
    return torch.stack([reward.double(), psnr.double(), accepted.double(), terminated.double(),
                        truncated.double()], dim=1)


def allreduce_hist(counts: torch.Tensor) -> torch.Tensor:
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(counts)
    return counts


def max_over_ranks(x: float, device: Optional[torch.device] = None) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
