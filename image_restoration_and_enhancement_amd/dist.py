"""Multi-GPU data parallelism for the restoration engine: one process per GPU.

The reference runs one image per call on one device (no collectives at
inference).  Here a batch of independent images is sharded contiguously across ranks; the only
collective on the data path's setup is an RCCL (backend "nccl" on ROCm) broadcast of the packed
frozen-weight blobs from rank 0 over xGMI, once per process.  There are no per-step, cross-image
or gradient collectives; outputs stay on their rank (or are gathered once by the caller).
"""
from __future__ import annotations

import os
from typing import Dict, Tuple

import torch
import torch.distributed as dist


def env_rank() -> Tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def init(backend: str | None = None) -> Tuple[int, int, int]:
    """Initialise torch.distributed from the torchrun environment when WORLD_SIZE > 1."""
    rank, world, local = env_rank()
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


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous shard [start, end) of n items: ceil(n / world) per rank, the last ranks shorter."""
    per = (n + world - 1) // world
    start = min(n, rank * per)
    return start, min(n, start + per)


def broadcast_blobs(blobs: Dict[str, torch.Tensor], src: int = 0) -> Dict[str, torch.Tensor]:
    """Broadcast each packed weight blob (uint8, same size on every rank) from `src`, in name order."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        for k in sorted(blobs):
            dist.broadcast(blobs[k], src=src)
    return blobs


def gather_shards(shard: torch.Tensor, n_total: int) -> torch.Tensor:
    """Reassemble the per-rank contiguous shards (dim 0, as produced by shard_range) into the full batch
    on every rank — one all_gather of the outputs at the end of a job, never inside the step loop."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return shard
    world = dist.get_world_size()
    per = (n_total + world - 1) // world
    buf = torch.zeros((per,) + tuple(shard.shape[1:]), dtype=shard.dtype, device=shard.device)
    buf[:shard.shape[0]] = shard
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = []
    for r in range(world):
        s, e = shard_range(n_total, r, world)
        out.append(parts[r][:e - s])
    return torch.cat(out, 0)


def max_over_ranks(x: float, device=None) -> float:
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier() -> None:
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
