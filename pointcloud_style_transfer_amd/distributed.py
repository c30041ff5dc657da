"""One process per GPU.

Inference shards independent clouds across ranks with no data-path collective: each rank
runs the guided loop on its own contiguous slice of the cloud list and writes its own
outputs; `gather_clouds` is the optional gather to rank 0.  Timing is max-over-ranks.
Training uses DistributedDataParallel (training/trainer.py) -- the only collective on the
path is its bucketed gradient all-reduce.

On the GPU the process group is RCCL ("nccl"); the same helpers run on "gloo" for the CPU
tests (tests/test_distributed.py).
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist


def init_from_env(backend: str | None = None) -> Tuple[int, int, int]:
    """Read RANK / LOCAL_RANK / WORLD_SIZE (torchrun); initialise the group when world > 1.
    Returns (world, rank, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def shard(n_items: int, rank: int, world: int) -> range:
    """Contiguous, balanced slice of `n_items` for `rank` (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def max_over_ranks(value: float, device=None) -> float:
    """Wall time of a timed region as the slowest rank saw it."""
    if not is_distributed():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, device=None) -> float:
    if not is_distributed():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_clouds(local: Sequence[torch.Tensor], n_items: int) -> List[torch.Tensor] | None:
    """Optional gather of every rank's output clouds to rank 0 (in global cloud order), via
    object collectives on host copies -- outside any timed region.  Other ranks get None."""
    if not is_distributed():
        return [c.cpu() for c in local]
    world, rank = dist.get_world_size(), dist.get_rank()
    host = [c.detach().cpu() for c in local]
    out = [None] * world if rank == 0 else None
    dist.gather_object(host, out, dst=0)
    if rank != 0:
        return None
    flat = [c for part in out for c in part]
    assert len(flat) == n_items, (len(flat), n_items)
    return flat
