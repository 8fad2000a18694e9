#!/usr/bin/env python3
"""Attention micro-benchmark at the batch-16 UNet shapes, per d=40 kernel variant (irx_set_option attn_d40),
interleaved rounds in one process.  Usage: python scripts/attnbench.py [--iters 20] [--variants 0,2,3]"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from tests import opref as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--variants", default="0,1,2,3")
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda")
L.load()
g = torch.Generator(device=dev).manual_seed(0)
dt = torch.bfloat16
for lab, B, Lq, Lk, C in [("self d40 L4096", 16, 4096, 4096, 320), ("cross d40", 16, 4096, 77, 320),
                          ("self d80 L1024", 16, 1024, 1024, 640), ("self d160 L256", 16, 256, 256, 1280)]:
    q = torch.randn(B, Lq, C, device=dev, generator=g).to(dt)
    k = torch.randn(B, Lk, C, device=dev, generator=g).to(dt)
    v = torch.randn(B, Lk, C, device=dev, generator=g).to(dt)
    flops = 4.0 * B * Lq * Lk * C
    vs = [int(x) for x in a.variants.split(",")] if C == 320 else [0]
    best = {x: 1e9 for x in vs}
    for _ in range(a.rounds):
        for x in vs:
            L.call("irx_set_option", b"attn_d40", x)
            O.attention(q, k, v, 8)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                O.attention(q, k, v, 8)
            e1.record()
            torch.cuda.synchronize()
            best[x] = min(best[x], e0.elapsed_time(e1) / a.iters * 1e3)
    L.call("irx_set_option", b"attn_d40", 2)
    print(f"{lab:18s} " + " | ".join(f"v{x} {t:8.1f}us {flops / t / 1e6:6.1f}TF" for x, t in best.items()), flush=True)
