#!/usr/bin/env python3
"""Do the two classifier-free-guidance halves of a UNet eval overlap when run on two HIP streams?

The batch-16 UNet eval of the bench (8 images x {uncond, cond}) is two independent batch-8 forwards until the
scheduler step.  Many of its kernels are latency-bound (one tile per CU, short K loops); run as two streams, one
half's kernels could fill the CUs the other's leave idle.  Times per eval (ms), eager and as a HIP graph:
  full      one batch-16 forward
  seq       two batch-8 forwards on one stream
  dual      two batch-8 forwards on two streams (fork / join events)
and checks that the halves' outputs equal the batch-16 output bit for bit (batch invariance).
"""
from __future__ import annotations

import argparse
import ctypes as C
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from image_restoration_and_enhancement_amd import weights as W  # noqa: E402
from image_restoration_and_enhancement_amd.configs import PipelineConfig  # noqa: E402
from image_restoration_and_enhancement_amd.engine import UNet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--res", type=int, default=64)
    ap.add_argument("--half", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    L.load()
    pc = PipelineConfig.default("denoise")
    sd = W.random_state_dict("unet", pc.unet, 0)
    u1 = UNet(pc.unet, a.dtype, dev)
    blob = u1.pack(sd).to(dev)
    u1.bind_blob(blob)
    u2 = UNet(pc.unet, a.dtype, dev)
    u2.bind_blob(blob)
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[a.dtype]
    B, h = a.half, a.res
    g = torch.Generator().manual_seed(0)
    x = torch.zeros(2 * B, h, h, u1.cin_pad)
    x[..., :4] = torch.randn(2 * B, h, h, 4, generator=g)
    x = x.to(tdt).to(dev).contiguous()
    kv = u1.prepare_context(torch.randn(2 * B, 77, 768, generator=g).to(tdt).to(dev).contiguous())
    t = torch.full((2 * B,), 481.0, device=dev)
    out_full = torch.empty(2 * B, h, h, 4, device=dev)
    out_half = torch.empty(2 * B, h, h, 4, device=dev)
    kvb = kv.numel() // (2 * B)            # bytes of one row's K|V block
    s_main = torch.cuda.Stream(dev)
    s_side = torch.cuda.Stream(dev)

    def full():
        u1.forward(x, t, kv, 77, out=out_full)

    def seq():
        u1.forward(x[:B], t, kv[:B * kvb], 77, out=out_half[:B])
        u1.forward(x[B:], t, kv[B * kvb:], 77, out=out_half[B:])

    def dual():
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        s_side.wait_event(ev)
        u1.forward(x[:B], t, kv[:B * kvb], 77, out=out_half[:B])
        with torch.cuda.stream(s_side):
            u2.forward(x[B:], t, kv[B * kvb:], 77, out=out_half[B:])
        ev2 = torch.cuda.Event()
        ev2.record(s_side)
        torch.cuda.current_stream().wait_event(ev2)

    def timed(fn, iters):
        with torch.cuda.stream(s_main):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) / iters * 1e3

    def graph(fn):
        h_ = C.c_void_p()
        with torch.cuda.stream(s_main):
            fn()                            # sizes the workspaces
            torch.cuda.synchronize()
            L.call("irx_graph_begin", C.c_void_p(s_main.cuda_stream))
            fn()
            L.call("irx_graph_end", C.c_void_p(s_main.cuda_stream), C.byref(h_))
        return lambda: L.call("irx_graph_launch", h_, C.c_void_p(s_main.cuda_stream))

    res = {}
    for name, fn in (("full", full), ("seq", seq), ("dual", dual)):
        res[name] = timed(fn, a.iters)
        if name != "full":
            torch.cuda.synchronize()
            same = torch.equal(out_full, out_half) if "full" in res else None
            print(f"{name}: halves == batch-16 output: {same}", flush=True)
        out_half.fill_(float("nan"))
    for name, fn in (("full", full), ("seq", seq), ("dual", dual)):
        res[name + "_graph"] = timed(graph(fn), a.iters)
    print(" | ".join(f"{k} {v:7.2f} ms" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
