"""Scene sharding across the GPUs of one node + the single association gather.

Scenes are independent (each has its own fundamental matrices and
centroids, process_pose.py:154-159), so the matcher shards them across ranks
with no data-path collective: rank r owns a contiguous scene range.  The only
exchange is ONE gather of the per-row association result (int32 argmin +
float32 minimum) to rank 0 at the end -- over RCCL/xGMI with the "nccl"
backend on ROCm, or gloo for CPU tests.  Distance matrices stay shard-local.

One process per GPU; launch with ``torchrun --nproc-per-node N`` (rendezvous
on 127.0.0.1).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

__all__ = ["DistEnv", "init_from_env", "shard_range", "gather_rows", "max_over_ranks"]


class DistEnv:
    def __init__(self, rank: int, world: int, local_rank: int, device: torch.device,
                 initialised: bool):
        self.rank, self.world, self.local_rank = rank, world, local_rank
        self.device, self.initialised = device, initialised

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    def barrier(self) -> None:
        if self.initialised:
            if self.device.type == "cuda":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()


def init_from_env(backend: Optional[str] = None, use_gpu: bool = True) -> DistEnv:
    """Initialise torch.distributed from torchrun's env (single process if absent)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if use_gpu:
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
    else:
        device = torch.device("cpu")
    initialised = False
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or ("nccl" if use_gpu else "gloo")
        kw = {"device_id": device} if (use_gpu and backend == "nccl") else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
        initialised = True
    return DistEnv(rank, world, local_rank, device, initialised)


def shard_range(n_items: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, stop) of ``n_items`` for ``rank`` (sizes differ by <= 1)."""
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_rows(env: DistEnv, *tensors: torch.Tensor) -> Optional[List[torch.Tensor]]:
    """Gather equally-shaped 1-D per-rank tensors to rank 0 (concatenated in rank
    order).  Ragged shards are padded to the largest shard and trimmed on rank 0.
    Returns the gathered tensors on rank 0, None elsewhere; identity at world 1."""
    if not env.initialised:
        return list(tensors)
    n_local = torch.tensor([tensors[0].numel()], dtype=torch.int64, device=tensors[0].device)
    sizes = [torch.zeros_like(n_local) for _ in range(env.world)]
    dist.all_gather(sizes, n_local)
    sizes = [int(s.item()) for s in sizes]
    n_max = max(sizes)
    out = []
    for t in tensors:
        if t.numel() < n_max:
            pad = torch.zeros(n_max - t.numel(), dtype=t.dtype, device=t.device)
            t = torch.cat([t, pad])
        bufs = [torch.empty_like(t) for _ in range(env.world)] if env.is_root else None
        dist.gather(t.contiguous(), gather_list=bufs, dst=0)
        if env.is_root:
            out.append(torch.cat([b[:n] for b, n in zip(bufs, sizes)]))
    return out if env.is_root else None


def max_over_ranks(env: DistEnv, value: float) -> float:
    if not env.initialised:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=env.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
