"""CPU tests of the multi-process data path with the gloo backend, world_size 2:
contiguous batch sharding, the frozen-weight blob broadcast, the end-of-job output gather and the
max-over-ranks timing reduction bench.py uses.  The same code runs over RCCL ("nccl") on MI355X."""
import os
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
