#!/usr/bin/env python3
"""Run one conv / GEMM shape repeatedly (for rocprofv3 PMC passes and option A/B tests).
Usage: python scripts/kshape.py gemm M N K [--iters 50] [--opt name=value ...]
       python scripts/kshape.py conv N H W C0 C1 Cout k [--iters 50] [--opt ...]"""
import argparse
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from tests import opref as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("kind")
ap.add_argument("dims", type=int, nargs="+")
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--opt", action="append", default=[])
a = ap.parse_args()
dev = torch.device("cuda")
L.load()
for o in a.opt:
    k, v = o.split("=")
    L.call("irx_set_option", k.encode(), int(v))
g = torch.Generator(device=dev).manual_seed(0)
dt = torch.bfloat16
if a.kind == "gemm":
    M, N, K = a.dims
    A = torch.randn(M, K, device=dev, generator=g).to(dt)
    Bw = (torch.randn(N, K, device=dev, generator=g) / math.sqrt(K)).to(dt)
    fn, flops = (lambda: O.gemm(A, Bw)), 2.0 * M * N * K
else:
    N, H, W, C0, C1, Co, k = a.dims
    x0 = torch.randn(N, H, W, C0, device=dev, generator=g).to(dt)
    x1 = torch.randn(N, H, W, C1, device=dev, generator=g).to(dt) if C1 else None
    w = (torch.randn(Co, C0 + C1, k, k, device=dev, generator=g) / math.sqrt((C0 + C1) * k * k)).to(dt)
    b = torch.zeros(Co, device=dev)
    fn, flops = (lambda: O.conv2d(x0, w, b, x1=x1)), 2.0 * N * H * W * Co * (C0 + C1) * k * k
for _ in range(3):
    fn()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.iters):
    fn()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.iters
print(f"{a.kind} {a.dims} {a.opt}: {ms * 1e3:.1f} us  {flops / ms / 1e9:.1f} TF/s")
