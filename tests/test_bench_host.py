"""bench.py's N > 1 line arithmetic on the CPU: under a gloo world of 2 with the engine replaced
by a stub step, the timed region is the max over ranks of the bracketed steps, and `value` = the images every rank
processed / that time (weak scaling: batch per GPU x world x steps).  The driver's 8-GPU run uses the same code with
RCCL; no GPU, no native library needed here."""
import multiprocessing as mp
import os
import socket
import time

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench as B
    from image_restoration_and_enhancement_amd import dist as D
    D.init(backend="gloo")
    calls = []

    def step():                      # rank 1 is the slow rank: 30 ms per step against 10 ms
        time.sleep(0.03 if rank == 1 else 0.01)
        calls.append(1)
        return rank

    out, el = B.timed_steps(step, steps=4, warmup=2, device=None, sync=lambda: None)
    value, ms = B.throughput(batch=8, world=world, steps=4, elapsed=el)
    q.put((rank, out, len(calls), el, value, ms))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_bench_line_arithmetic_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    els = [r[3] for r in res]
    assert els[0] == els[1]                          # every rank reports the same (max) time
    assert els[0] >= 4 * 0.03                        # ... which is the slow rank's
    for rank, out, n_calls, el, value, ms in res:
        assert out == rank and n_calls == 2 + 4      # warmup + exactly `steps` timed steps
        assert value == pytest.approx(8 * 2 * 4 / el)  # whole-job images / s
        assert ms == pytest.approx(el / 4 * 1e3)


def test_throughput_single():
    import bench as B
    v, ms = B.throughput(8, 1, 20, 9.765)
    assert v == pytest.approx(16.3866, rel=1e-4) and ms == pytest.approx(488.25)
