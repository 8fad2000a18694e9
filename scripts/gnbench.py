#!/usr/bin/env python3
"""GroupNorm(+SiLU) / LayerNorm micro-benchmark at the batch-16 UNet / batch-8 VAE shapes (HIP events),
per option variant in one process.  Usage: python scripts/gnbench.py [--iters 50]"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from tests import opref as O  # noqa: E402

SHAPES = [(16, 64, 64, 320, 0), (16, 32, 32, 640, 0), (16, 16, 16, 1280, 0), (16, 8, 8, 2560, 0),
          (16, 8, 8, 1280, 1280), (16, 64, 64, 320, 320), (8, 512, 512, 128, 0), (8, 256, 256, 256, 0)]
ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=50)
a = ap.parse_args()
dev = torch.device("cuda")
L.load()
g = torch.Generator(device=dev).manual_seed(0)
VARIANTS = [("v3", [("gn_v2", 1)]), ("v1", [("gn_v2", 0)])]


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.iters * 1e3


for N, H, W, C0, C1 in SHAPES:
    x0 = torch.randn(N, H, W, C0, device=dev, generator=g).to(torch.bfloat16)
    x1 = torch.randn(N, H, W, C1, device=dev, generator=g).to(torch.bfloat16) if C1 else None
    gm = torch.ones(C0 + C1, device=dev)
    bt = torch.zeros(C0 + C1, device=dev)
    mb = (x0.numel() + (x1.numel() if C1 else 0)) * 2 / 1e6
    res = []
    for name, opts in VARIANTS:
        for k, v in opts:
            L.call("irx_set_option", k.encode(), v)
        us = timeit(lambda: O.group_norm(x0, gm, bt, 1e-5, silu=True, x1=x1))
        res.append(f"{name} {us:7.1f}us {3 * mb / us / 1e6:5.2f}TB/s")
    print(f"N{N} {H}x{W} C{C0}+{C1} ({mb:.1f} MB): " + " | ".join(res), flush=True)
L.call("irx_set_option", b"gn_v2", 1)
for rows, C in [(65536, 320), (16384, 640), (4096, 1280), (1024, 1280)]:
    x = torch.randn(rows, C, device=dev, generator=g).to(torch.bfloat16)
    gm = torch.ones(C, device=dev)
    bt = torch.zeros(C, device=dev)
    us = timeit(lambda: O.layer_norm(x, gm, bt, 1e-5))
    print(f"LN {rows}x{C}: {us:7.1f}us {2 * x.numel() * 2 / us / 1e6:5.2f}TB/s", flush=True)
