"""CPU tests of the multi-process data path with the gloo backend, world_size 2:
contiguous batch sharding, the frozen-weight blob broadcast, the end-of-job output gather and the
max-over-ranks timing reduction bench.py uses.  The same code runs over RCCL ("nccl") on MI355X."""
import os
import time
import socket

import pytest
import torch
import torch.multiprocessing as mp

from image_restoration_and_enhancement_amd import dist as D


@pytest.mark.parametrize("n,world", [(8, 1), (8, 2), (8, 8), (7, 2), (3, 4), (0, 2), (64, 8), (9, 8)])
def test_shard_range_partitions(n, world):
    covered = []
    for r in range(world):
        s, e = D.shard_range(n, r, world)
        assert 0 <= s <= e <= n
        covered.extend(range(s, e))
    assert covered == list(range(n))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        r, w, _ = D.init("gloo")
        assert (r, w) == (rank, world)
        # weight blobs: rank 0 holds the packed weights, the others receive them
        g = torch.Generator().manual_seed(123)
        ref = {"unet": torch.randint(0, 256, (1000,), dtype=torch.uint8, generator=g),
               "vae": torch.randint(0, 256, (333,), dtype=torch.uint8, generator=g)}
        blobs = {k: (v.clone() if rank == 0 else torch.zeros_like(v)) for k, v in ref.items()}
        D.broadcast_blobs(blobs)
        ok_bcast = all(torch.equal(blobs[k], ref[k]) for k in ref)
        # 5 images over 2 ranks: rank 0 gets 3, rank 1 gets 2
        n = 5
        s, e = D.shard_range(n, rank, world)
        shard = torch.arange(s, e, dtype=torch.uint8).view(-1, 1, 1, 1).expand(-1, 4, 4, 3).contiguous()
        full = D.gather_shards(shard, n)
        ok_gather = full.shape == (n, 4, 4, 3) and torch.equal(full[:, 0, 0, 0], torch.arange(n, dtype=torch.uint8))
        mx = D.max_over_ranks(1.5 + rank)
        D.barrier()
        q.put((rank, ok_bcast, ok_gather, mx))
    except Exception as ex:  # report instead of hanging the parent
        q.put((rank, repr(ex), None, None))
    finally:
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()


def test_gloo_world2_broadcast_gather_max():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, ok_b, ok_g, mx in res:
        assert ok_b is True, ok_b
        assert ok_g is True
        assert mx == 2.5


INIT_TIMEOUT_S = 2.0


class _Model:
    """Stand-in for a bound irx model: a handle and its packed weight blob."""

    def __init__(self, h, blob):
        self.h, self.blob = h, blob


def _stub_lib(L, rank, scenario, models, log):
    """_lib.call replaced by a stub: the RCCL entry points succeed or fail per `scenario`, and irx_weights_bcast
    moves the blob with a gloo broadcast so the data path can be checked end to end on the CPU.  The stubbed
    irx_rccl_comm_init_timeout models the C side's deadline: in scenario "inithang" rank 1's init never completes
    and rank 0's waits for it (the init is collective), so both return the C ABI's timeout error once
    `timeout_ms` has passed (the real form aborts the half-made communicator there: tests/test_rccl_gpu.py)."""
    import ctypes as C
    import torch.distributed as dist
    uid = bytes(range(128))

    def call(name, *args):
        log.append(name)
        if name == "irx_rccl_available":
            return 0 if (scenario == "nolib" and rank == 1) else 1
        if name == "irx_rccl_unique_id":
            if scenario == "noid":
                raise L.IrxError("ncclGetUniqueId: stub failure")
            C.memmove(args[0], uid, len(uid))
            return 0
        if name == "irx_rccl_comm_init_timeout":
            idb, world, r, timeout_ms, pcomm = args
            assert bytes(idb)[:128] == uid and world == 2 and r == rank and timeout_ms >= 1
            if scenario == "initfail" and rank == 1:
                raise L.IrxError("ncclCommInitRankConfig: stub failure")
            if scenario == "inithang":
                time.sleep(timeout_ms / 1000.0)
                raise L.IrxError(f"ncclCommInitRankConfig: rank {rank} of 2 did not finish within {timeout_ms} ms "
                                 "(communicator aborted)")
            pcomm._obj.value = 1000 + rank
            return 0
        if name == "irx_rccl_comm_destroy":
            assert args[0].value == 1000 + rank
            return 0
        if name == "irx_weights_bcast":
            h, comm, src, _s = args
            assert comm.value == 1000 + rank
            dist.broadcast(next(m.blob for m in models.values() if m.h == h), src=src)
            return 0
        raise AssertionError(f"unexpected call {name}")
    return call


def _bcast_worker(rank, world, port, scenario, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), IRX_RCCL_INIT_TIMEOUT_S=str(INIT_TIMEOUT_S))
    try:
        from image_restoration_and_enhancement_amd import _lib as L
        D.init("gloo")
        g = torch.Generator().manual_seed(7)
        ref = {"unet": torch.randint(0, 256, (4096,), dtype=torch.uint8, generator=g),
               "vae": torch.randint(0, 256, (513,), dtype=torch.uint8, generator=g)}
        models = {k: _Model(i + 1, v.clone() if rank == 0 else torch.zeros_like(v)) for i, (k, v) in enumerate(ref.items())}
        log = []
        L.call = _stub_lib(L, rank, scenario, models, log)
        D.barrier()
        t0 = time.monotonic()
        how = D.broadcast_models(models)
        dt = time.monotonic() - t0
        ok = all(torch.equal(models[k].blob, ref[k]) for k in ref)
        D.barrier()
        q.put((rank, how.split(" ")[0], ok, log.count("irx_rccl_comm_destroy"), log.count("irx_weights_bcast"), dt))
    except Exception as ex:  # report instead of hanging the parent
        q.put((rank, repr(ex), None, None, None, None))
    finally:
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()


@pytest.mark.parametrize("scenario", ["ok", "nolib", "noid", "initfail", "inithang"])
def test_broadcast_models_rank_consistent(scenario):
    """dist.broadcast_models with _lib.call stubbed: every rank takes
    the same path — irx_weights_bcast when RCCL comes up everywhere, the torch.distributed broadcast on every rank
    when librccl is missing on one rank, rank 0 cannot make the unique id, one rank's communicator init fails (the
    ranks that got a communicator destroy it), or one rank's init hangs (every rank leaves within the deadline) —
    and the blobs arrive intact either way."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, 2, port, scenario, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    want = "irx_rccl" if scenario == "ok" else "torch.distributed"
    for rank, how, ok, destroyed, bcasts, dt in res:
        assert how == want, (rank, how)
        if scenario == "inithang":   # out within the deadline (+ the agreement round trips and the fallback)
            assert INIT_TIMEOUT_S <= dt < INIT_TIMEOUT_S + 20, (rank, dt)
        assert ok is True
        assert bcasts == (2 if scenario == "ok" else 0)
        exp_destroy = 1 if scenario == "ok" or (scenario == "initfail" and rank == 0) else 0
        assert destroyed == exp_destroy, (rank, destroyed)
