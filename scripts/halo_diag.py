#!/usr/bin/env python3
"""What bounds the halo 3x3 conv (gemm2_kernel<256,160,...,HALO=2>)?  Times the UNet's halo-conv shapes (batch 16,
512x512) with parts of the ping-pong main loop knocked out through the timing-diagnostic bits of option gemm_dbg
(results are wrong when set): 2 no MFMAs, 4 no B DMA, 8 no halo DMA, 16 no fragment reads, 32 no barriers,
1 no epilogue.  Variants interleave in one process (HIP events, median of rounds).
  python scripts/halo_diag.py [--iters 20] [--rounds 3] [--dbg 0,1,2,4,8,16,32,36,44]
--stamps: with the timing-diagnostic library (scripts/build_stamps.sh), the loop's own s_memtime segment sums per tap,
averaged over the blocks of one launch, for each wave group (cycles; the stamps' fences forbid some overlaps the
real kernel has, so read the shares, not the totals)."""
from __future__ import annotations

import argparse
import math
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from tests import opref as O  # noqa: E402

SHAPES = [  # (label, N, H, W, C0, C1, Cout)
    ("conv320@64", 16, 64, 64, 320, 0, 320),
    ("cat640+320->320@64", 16, 64, 64, 640, 320, 320),
    ("conv640@32", 16, 32, 32, 640, 0, 640),
    ("conv1280@16 (split 2)", 16, 16, 16, 1280, 0, 1280),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--dbg", default="0,1,2,4,8,12,16,32,20,36")
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--variants", default="",
                    help="option sets to A/B instead of the dbg bits, interleaved: 'name:k=v,k=v;name2:k=v'")
    a = ap.parse_args()
    if a.stamps:
        return stamps()
    L.load()
    for o in a.opt:
        k, v = o.split("=")
        L.call("irx_set_option", k.encode(), int(v))
    dev, dt = torch.device("cuda"), torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    if a.variants:   # (name, {option: value}) sets, timed at dbg 0
        sets = []
        for part in a.variants.split(";"):
            name, _, kv = part.partition(":")
            sets.append((name, {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}))
    else:
        sets = [(f"dbg {int(x):3d}", {"gemm_dbg": int(x)}) for x in a.dbg.split(",")]
    for lab, N, H, W, C0, C1, Co in SHAPES:
        x0 = torch.randn(N, H, W, C0, device=dev, generator=g).to(dt)
        x1 = torch.randn(N, H, W, C1, device=dev, generator=g).to(dt) if C1 else None
        wk = (torch.randn(Co, 3, 3, C0 + C1, device=dev, generator=g) / math.sqrt(9 * (C0 + C1))).to(dt)
        b = torch.zeros(Co, device=dev)
        out = torch.empty(N, H, W, Co, dtype=dt, device=dev)
        flops = 2.0 * N * H * W * Co * (C0 + C1) * 9

        def run():
            L.call("irx_op_conv2d", O.S(), O.DT[dt], O.P(x0), O.P(x1), C0, C1, N, H, W, H, W, O.P(wk), O.P(b), Co,
                   3, 3, 1, 1, 1, H, W, None, 0, None, O.P(out), 0, 0)
        times = {n: [] for n, _ in sets}
        for _ in range(a.rounds):
            for n, opts in sets:
                with L.option(**opts):
                    for _ in range(2):
                        run()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        run()
                    e1.record()
                    torch.cuda.synchronize()
                times[n].append(e0.elapsed_time(e1) / a.iters * 1e3)
        base = statistics.median(times[sets[0][0]])
        print(f"{lab}: {flops / base / 1e6:.0f} TF/s at {sets[0][0]}", flush=True)
        for n, _ in sets:
            us = statistics.median(times[n])
            print(f"  {n:10s}: {us:8.1f} us  ({us / base:5.2f} x)  {flops / us / 1e6:6.0f} TF/s", flush=True)


DBG_STAMPS = [(0, "as is"), (2, "no MFMAs"), (12, "no DMA"), (16, "no fragment reads"), (128, "load phases prio 1"),
              (256, "compute phases prio 1")]


def stamps():
    import ctypes
    import numpy as np
    lib = Path(__file__).resolve().parent / "_skdbg" / "libirx_stamps.so"
    L.load(lib)
    dev, dt = torch.device("cuda"), torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    seg = ["DMA issue + frag reads", "B wait", "barrier (load)", "MFMA issue", "barrier (compute)"]
    for lab, N, H, W, C0, C1, Co in SHAPES:
        x0 = torch.randn(N, H, W, C0, device=dev, generator=g).to(dt)
        x1 = torch.randn(N, H, W, C1, device=dev, generator=g).to(dt) if C1 else None
        wk = (torch.randn(Co, 3, 3, C0 + C1, device=dev, generator=g) / math.sqrt(9 * (C0 + C1))).to(dt)
        b = torch.zeros(Co, device=dev)
        out = torch.empty(N, H, W, Co, dtype=dt, device=dev)
        for dbg, what in DBG_STAMPS:
            with L.option(gemm_dbg=64 | dbg):   # (bit 64: the HALO == 4 instantiation; + knock-out / priority bits)
                for _ in range(20):
                    L.call("irx_op_conv2d", O.S(), O.DT[dt], O.P(x0), O.P(x1), C0, C1, N, H, W, H, W, O.P(wk), O.P(b),
                           Co, 3, 3, 1, 1, 1, H, W, None, 0, None, O.P(out), 0, 0)
                torch.cuda.synchronize()
            nblk = min(2048, N * H * W // 256 * (Co // 160) * (2 if "split 2" in lab else 1))
            buf = np.zeros(nblk * 64, dtype=np.uint64)
            fn = L.load().irx_debug_halo_stamps
            fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
            fn(buf.ctypes.data, buf.size)
            st = buf.reshape(nblk, 8, 8).astype(np.float64)
            taps = st[:, :, 5]
            print(f"{lab} [{what}]: cycles per tap (mean over {nblk} blocks)", flush=True)
            for grp, ws in (("group 0 (halo)", slice(0, 4)), ("group 1 (B)", slice(4, 8))):
                per = st[:, ws, :5].sum(axis=(0, 1)) / taps[:, ws].sum()
                print(f"  {grp:15s} " + "  ".join(f"{n}: {v:6.0f}" for n, v in zip(seg, per)) +
                      f"  | total {per.sum():6.0f}", flush=True)


if __name__ == "__main__":
    main()
