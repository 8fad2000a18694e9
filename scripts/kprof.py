#!/usr/bin/env python3
"""Loop one hot op of the UNet at its batch-16 (8 images x CFG) 512x512 shape, for rocprofv3 PMC passes that
target a single kernel (`--kernel-include-regex`) without the rest of the bench around it.

  python scripts/kprof.py --op conv320      halo 3x3 conv, 64x64 level, 320 -> 320
  python scripts/kprof.py --op geglu320     GEGLU feed-forward projection, M 65536, K 320, N 2560
  python scripts/kprof.py --op geglu640     ... 32^2 level (M 16384, K 640); geglu1280: 16^2 (M 4096, K 1280)
  python scripts/kprof.py --op lin320       K = 320 projection (proj_in / to_q), M 65536, N 320
  python scripts/kprof.py --op lin320r      ... + residual (to_out / proj_out)
  python scripts/kprof.py --op qkv320       q|k|v projection, N 960 (row-major here)
  python scripts/kprof.py --op lin1280      16x16-level projection, M 4096, N 1280, K 1280
  python scripts/kprof.py --op attn40       self-attention, 8 heads x d 40, L 4096
options: --iters N (default 20), --opt name=value (irx_set_option, repeatable)
"""
from __future__ import annotations

import argparse
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from image_restoration_and_enhancement_amd.engine import geglu64_order  # noqa: E402
from tests import opref as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", required=True)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--lib", default=None, help="alternate libirx.so (timing-diagnostic builds)")
    a = ap.parse_args()
    L.load(a.lib)
    for o in a.opt:
        k, v = o.split("=")
        L.call("irx_set_option", k.encode(), int(v))
    dev, dt = torch.device("cuda"), torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)

    def rn(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(dt)

    if a.op == "conv320":
        x, w = rn(16, 64, 64, 320), rn(320, 320, 3, 3, scale=1 / math.sqrt(2880)).float()
        b = torch.zeros(320, device=dev)
        fn = lambda: O.conv2d(x, w, b)                                       # noqa: E731
    elif a.op in ("geglu320", "geglu640", "geglu1280"):
        C = int(a.op[5:])
        M = {320: 65536, 640: 16384, 1280: 4096}[C]
        A, Wt = rn(M, C), rn(8 * C, C, scale=1 / math.sqrt(C))[geglu64_order(8 * C)].contiguous()
        bias = torch.zeros(8 * C, device=dev)
        out = torch.empty(M, 4 * C, dtype=dt, device=dev)
        fn = lambda: L.call("irx_op_gemm_geglu", O.S(), O.DT[dt], M, 8 * C, C, O.P(A), O.P(Wt), O.P(bias),  # noqa: E731
                            O.P(out))
    elif a.op == "ff1_320":
        A, Bw = rn(65536, 320), rn(2560, 320, scale=1 / math.sqrt(320))
        fn = lambda: O.gemm(A, Bw)                                            # noqa: E731
    elif a.op == "ff2_320":
        A, Bw = rn(65536, 1280), rn(320, 1280, scale=1 / math.sqrt(1280))
        fn = lambda: O.gemm(A, Bw)                                            # noqa: E731
    elif a.op == "lin320":
        A, Bw = rn(65536, 320), rn(320, 320, scale=1 / math.sqrt(320))
        fn = lambda: O.gemm(A, Bw)                                            # noqa: E731
    elif a.op == "lin320r":                                                    # to_out / proj_out: + residual
        A, Bw, R = rn(65536, 320), rn(320, 320, scale=1 / math.sqrt(320)), rn(65536, 320)
        bias = torch.zeros(320, device=dev)
        fn = lambda: O.gemm(A, Bw, bias=bias, residual=R)                      # noqa: E731
    elif a.op == "qkv320":
        A, Bw = rn(65536, 320), rn(960, 320, scale=1 / math.sqrt(320))
        fn = lambda: O.gemm(A, Bw)                                            # noqa: E731
    elif a.op == "lin640":
        A, Bw = rn(16384, 640), rn(640, 640, scale=1 / math.sqrt(640))
        fn = lambda: O.gemm(A, Bw)                                            # noqa: E731
    elif a.op == "lin1280":
        A, Bw = rn(4096, 1280), rn(1280, 1280, scale=1 / math.sqrt(1280))
        fn = lambda: O.gemm(A, Bw)                                            # noqa: E731
    elif a.op == "attn40":
        q, k, v = rn(16, 4096, 320), rn(16, 4096, 320), rn(16, 4096, 320)
        fn = lambda: O.attention(q, k, v, 8)                                  # noqa: E731
    elif a.op == "cross40":
        q, k, v = rn(16, 4096, 320), rn(16, 77, 320), rn(16, 77, 320)
        fn = lambda: O.attention(q, k, v, 8)                                  # noqa: E731
    else:
        raise SystemExit(f"unknown op {a.op}")
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{a.op}: {e0.elapsed_time(e1) / a.iters * 1e3:.1f} us per call", flush=True)


if __name__ == "__main__":
    main()
