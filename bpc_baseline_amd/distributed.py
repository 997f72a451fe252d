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

import datetime
import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

__all__ = ["DistEnv", "init_from_env", "shard_range", "gather_rows", "max_over_ranks",
           "sum_over_ranks", "ChunkedRowGather", "DEFAULT_TIMEOUT_S"]

# every collective (RCCL or gloo) of a process group made here fails after
# this long instead of hanging the job: a stuck gather on an 8-GPU run ends
# the run non-zero with a message (MVM_DIST_TIMEOUT_S overrides it)
DEFAULT_TIMEOUT_S = 300


class DistEnv:
    def __init__(self, rank: int, world: int, local_rank: int, device: torch.device,
                 initialised: bool, backend: Optional[str] = None):
        self.rank, self.world, self.local_rank = rank, world, local_rank
        self.device, self.initialised, self.backend = device, initialised, backend
        self._cpu_group = None
        self.timeout = datetime.timedelta(seconds=DEFAULT_TIMEOUT_S)

    def cpu_group(self):
        """A gloo group over the same ranks, for host-memory collectives next
        to an RCCL default group (collective: every rank must call it, in the
        same order).  None when the default group is already gloo."""
        if not self.initialised or self.backend == "gloo":
            return None
        if self._cpu_group is None:
            self._cpu_group = dist.new_group(backend="gloo", timeout=self.timeout)
        return self._cpu_group

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    def barrier(self) -> None:
        if self.initialised:
            if self.device.type == "cuda" and self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()


def init_from_env(backend: Optional[str] = None, use_gpu: bool = True,
                  timeout_s: Optional[float] = None) -> DistEnv:
    """Initialise torch.distributed from torchrun's env (single process if absent).

    One process per GPU: rank -> cuda:LOCAL_RANK.  ``backend`` defaults to
    "nccl" (RCCL over xGMI on ROCm) for GPU ranks and "gloo" otherwise;
    MVM_DIST_BACKEND overrides it (gloo rehearsals of several ranks on one
    GPU map LOCAL_RANK onto the visible devices round-robin).  Collectives
    time out after ``timeout_s`` (default MVM_DIST_TIMEOUT_S or 300 s); an
    RCCL rank with no GPU of its own raises."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("MVM_DIST_BACKEND") or backend or ("nccl" if use_gpu else "gloo")
    if use_gpu:
        n_dev = torch.cuda.device_count()
        if backend == "nccl" and local_rank >= n_dev:
            raise RuntimeError(f"rank {rank}: LOCAL_RANK {local_rank} but only {n_dev} visible GPU(s); "
                               "RCCL needs one GPU per rank")
        index = local_rank % n_dev if (backend == "gloo" and n_dev) else local_rank
        torch.cuda.set_device(index)
        device = torch.device("cuda", index)
    else:
        device = torch.device("cpu")
    if timeout_s is None:
        timeout_s = float(os.environ.get("MVM_DIST_TIMEOUT_S", DEFAULT_TIMEOUT_S))
    timeout = datetime.timedelta(seconds=timeout_s)
    initialised = False
    # MVM_DIST_FORCE=1 creates the process group even for one rank, so the
    # RCCL code path (device-bound group, async gathers) runs on a 1-GPU box
    if world > 1 or os.environ.get("MVM_DIST_FORCE") == "1":
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": device} if (use_gpu and backend == "nccl") else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, timeout=timeout, **kw)
        initialised = True
        # what the process group itself reports, not what the launcher's env said
        world, rank = dist.get_world_size(), dist.get_rank()
        backend = str(dist.get_backend())
    env = DistEnv(rank, world, local_rank, device, initialised, backend)
    env.timeout = timeout
    return env


def shard_range(n_items: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, stop) of ``n_items`` for ``rank`` (sizes differ by <= 1)."""
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_rows(env: DistEnv, *tensors: torch.Tensor, group=None) -> Optional[List[torch.Tensor]]:
    """Gather equally-shaped 1-D per-rank tensors to rank 0 (concatenated in rank
    order).  Ragged shards are padded to the largest shard and trimmed on rank 0.
    Returns the gathered tensors on rank 0, None elsewhere; identity at world 1.
    ``group``: a gloo group (``env.cpu_group()``) to gather host tensors over
    instead of the default group."""
    if not env.initialised:
        return list(tensors)
    on_host = group is not None or env.backend == "gloo"
    if on_host and tensors[0].device.type != "cpu":
        tensors = tuple(t.cpu() for t in tensors)   # gloo collectives run on host memory
    n_local = torch.tensor([tensors[0].numel()], dtype=torch.int64, device=tensors[0].device)
    sizes = [torch.zeros_like(n_local) for _ in range(env.world)]
    dist.all_gather(sizes, n_local, group=group)
    sizes = [int(s.item()) for s in sizes]
    n_max = max(sizes)
    out = []
    for t in tensors:
        if t.numel() < n_max:
            pad = torch.zeros(n_max - t.numel(), dtype=t.dtype, device=t.device)
            t = torch.cat([t, pad])
        bufs = [torch.empty_like(t) for _ in range(env.world)] if env.is_root else None
        dist.gather(t.contiguous(), gather_list=bufs, dst=0, group=group)
        if env.is_root:
            out.append(torch.cat([b[:n] for b, n in zip(bufs, sizes)]))
    return out if env.is_root else None


def max_over_ranks(env: DistEnv, value: float) -> float:
    if not env.initialised:
        return value
    dev = env.device if env.backend == "nccl" else torch.device("cpu")
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(env: DistEnv, value: int) -> int:
    if not env.initialised:
        return int(value)
    dev = env.device if env.backend == "nccl" else torch.device("cpu")
    t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


class ChunkedRowGather:
    """The association gather, split into pieces that overlap the compute.

    Every rank holds its rows in equally laid-out buffers.  ``issue(k)``
    enqueues an asynchronous gather of piece k to rank 0 right after the
    launch that produced it: the collective (RCCL on its own stream) waits
    only for work already enqueued on the compute stream, so piece k moves
    over xGMI while piece k+1 computes.  ``finish()`` makes the compute
    stream wait for every outstanding piece.  With world 1 it is a no-op.
    Row counts must be equal on all ranks (checked once at construction).
    """

    def __init__(self, env: DistEnv, tensors, pieces):
        self.env, self.tensors, self.pieces = env, list(tensors), list(pieces)
        self.handles = []
        self.recv = None
        self.copy_back = []    # (host staging, device destination) of gloo gathers
        if not env.initialised:
            return
        n = torch.tensor([self.tensors[0].numel()], dtype=torch.int64,
                         device=env.device if env.backend == "nccl" else "cpu")
        sizes = [torch.zeros_like(n) for _ in range(env.world)]
        dist.all_gather(sizes, n)
        if len({int(x.item()) for x in sizes}) != 1:
            raise ValueError("ChunkedRowGather needs the same row count on every rank")
        if env.is_root:
            self.recv = [torch.empty((env.world, t.numel()), dtype=t.dtype, device=t.device)
                         for t in self.tensors]

    def issue(self, k: int) -> None:
        if not self.env.initialised:
            return
        a, b = self.pieces[k]
        for i, t in enumerate(self.tensors):
            src = t[a:b]
            if self.env.backend == "gloo" and src.device.type != "cpu":
                src = src.cpu()
            dst = None
            if self.env.is_root:
                dst = [self.recv[i][r, a:b] for r in range(self.env.world)]
                if self.env.backend == "gloo" and dst[0].device.type != "cpu":
                    host = [torch.empty(d.shape, dtype=d.dtype) for d in dst]
                    self.copy_back.extend(zip(host, dst))
                    dst = host
            self.handles.append(dist.gather(src.contiguous(), gather_list=dst, dst=0,
                                            async_op=True))

    def finish(self):
        for h in self.handles:
            h.wait()
        self.handles = []
        for host, dev in self.copy_back:
            dev.copy_(host)
        self.copy_back = []
        return self.recv
