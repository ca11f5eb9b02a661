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
    """Concatenate equal-shaped per-rank tensors on rank 0 (None elsewhere).

    Uses all_gather (supported by both nccl and gloo for any dtype)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return t
    parts: List[torch.Tensor] = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t.contiguous())
    return torch.cat(parts) if dist.get_rank() == 0 else None


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
