#!/usr/bin/env python3
"""Tile / split-K sweep over the conv and GEMM shapes of one batch-16 UNet eval and a batch-8 VAE pass.
For every shape: time the heuristic's choice (gemm_force 0) and every forced (BM, BN, splits) candidate
(HIP events, interleaved repeats); print the best and the heuristic's loss.  Calibration data for
gemm2.hip choose().  Usage: python scripts/gemm_sweep.py [--iters 10] [--only unet|vae]"""
import argparse
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from tests import opref as O  # noqa: E402

B = 16
UNET_CONV = [  # (count per eval, N, H, W, C0, C1, Cout, k, stride, up)
    (4, B, 64, 64, 320, 0, 320, 3, 1, None), (1, B, 64, 64, 320, 0, 320, 3, 2, None),
    (1, B, 32, 32, 320, 0, 640, 3, 1, None), (1, B, 32, 32, 320, 0, 640, 1, 1, None),
    (3, B, 32, 32, 640, 0, 640, 3, 1, None), (1, B, 32, 32, 640, 0, 640, 3, 2, None),
    (1, B, 16, 16, 640, 0, 1280, 3, 1, None), (1, B, 16, 16, 640, 0, 1280, 1, 1, None),
    (3, B, 16, 16, 1280, 0, 1280, 3, 1, None), (1, B, 16, 16, 1280, 0, 1280, 3, 2, None),
    (11, B, 8, 8, 1280, 0, 1280, 3, 1, None), (3, B, 8, 8, 1280, 1280, 1280, 3, 1, None),
    (3, B, 8, 8, 1280, 1280, 1280, 1, 1, None), (1, B, 8, 8, 1280, 0, 1280, 3, 1, (16, 16)),
    (2, B, 16, 16, 1280, 1280, 1280, 3, 1, None), (1, B, 16, 16, 1280, 640, 1280, 3, 1, None),
    (2, B, 16, 16, 1280, 1280, 1280, 1, 1, None), (1, B, 16, 16, 1280, 0, 1280, 3, 1, (32, 32)),
    (1, B, 32, 32, 1280, 640, 640, 3, 1, None), (1, B, 32, 32, 640, 640, 640, 3, 1, None),
    (1, B, 32, 32, 640, 320, 640, 3, 1, None), (1, B, 32, 32, 1280, 640, 640, 1, 1, None),
    (1, B, 32, 32, 640, 0, 640, 3, 1, (64, 64)),
    (1, B, 64, 64, 640, 320, 320, 3, 1, None), (2, B, 64, 64, 320, 320, 320, 3, 1, None),
    (1, B, 64, 64, 640, 320, 320, 1, 1, None), (3, B, 64, 64, 320, 0, 320, 3, 1, None),
]
UNET_GEMM = []  # (count, M, N, K, geglu)
for M, C, nx in [(65536, 320, 5), (16384, 640, 5), (4096, 1280, 5), (1024, 1280, 1)]:
    UNET_GEMM += [(5 * nx, M, C, C, 0), (nx, M, 3 * C, C, 0), (nx, M, 8 * C, C, 1), (nx, M, C, 4 * C, 0)]
V = 8
VAE_CONV = [
    (4, V, 512, 512, 128, 0, 128, 3, 1, None), (1, V, 512, 512, 128, 0, 128, 3, 2, None),
    (1, V, 256, 256, 128, 0, 256, 3, 1, None), (3, V, 256, 256, 256, 0, 256, 3, 1, None),
    (1, V, 256, 256, 256, 0, 256, 3, 2, None), (1, V, 128, 128, 256, 0, 512, 3, 1, None),
    (3, V, 128, 128, 512, 0, 512, 3, 1, None), (1, V, 128, 128, 512, 0, 512, 3, 2, None),
    (13, V, 64, 64, 512, 0, 512, 3, 1, None), (1, V, 64, 64, 512, 0, 512, 3, 1, (128, 128)),
    (6, V, 128, 128, 512, 0, 512, 3, 1, None), (1, V, 128, 128, 512, 0, 512, 3, 1, (256, 256)),
    (1, V, 256, 256, 512, 0, 256, 3, 1, None), (1, V, 256, 256, 512, 0, 256, 1, 1, None),
    (5, V, 256, 256, 256, 0, 256, 3, 1, None), (1, V, 256, 256, 256, 0, 256, 3, 1, (512, 512)),
    (1, V, 512, 512, 256, 0, 128, 3, 1, None), (1, V, 512, 512, 256, 0, 128, 1, 1, None),
    (5, V, 512, 512, 128, 0, 128, 3, 1, None),
]
CANDS = [(bm, bn, sp) for bm, bn in [(256, 320), (256, 256), (128, 320), (128, 256), (128, 128)] for sp in (1, 2, 4, 8)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def sweep(label, cnt, fn, N, K, geglu):
    res = {}
    for bm, bn, sp in [(0, 0, 0)] + CANDS:
        if bm and (N % bn or (geglu and bn % 128) or (sp > 1 and geglu)):
            continue
        L.call("irx_set_option", b"gemm_force", bm * 100000 + bn * 100 + sp)
        res[(bm, bn, sp)] = timeit(fn, args.iters)
    L.call("irx_set_option", b"gemm_force", 0)
    best = min((v, k) for k, v in res.items() if k[0])
    h = res[(0, 0, 0)]
    top = sorted((v, k) for k, v in res.items() if k[0])[:4]
    print(f"{label:44s} x{cnt:<3d} heur {h:8.1f}us  best {best[1]} {best[0]:8.1f}us  loss {cnt * (h - best[0]):7.1f}us  "
          + " ".join(f"{k[0]}x{k[1]}/{k[2]}:{v:.0f}" for v, k in top), flush=True)
    return cnt * h, cnt * best[0]


ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--only", default="")
args = ap.parse_args()
dev = torch.device("cuda")
L.load()
g = torch.Generator(device=dev).manual_seed(0)
dt = torch.bfloat16
tot_h = tot_b = 0.0
convs = (UNET_CONV if args.only in ("", "unet") else []) + (VAE_CONV if args.only in ("", "vae") else [])
for cnt, N, H, W, C0, C1, Co, k, s, up in convs:
    x0 = torch.randn(N, H, W, C0, device=dev, generator=g).to(dt)
    x1 = torch.randn(N, H, W, C1, device=dev, generator=g).to(dt) if C1 else None
    w = (torch.randn(Co, C0 + C1, k, k, device=dev, generator=g) / math.sqrt((C0 + C1) * k * k)).to(dt)
    b = torch.zeros(Co, device=dev)
    lab = f"conv N{N} {H}x{W} {C0}+{C1}->{Co} k{k}s{s}" + (f" up{up[0]}" if up else "")
    a_, b_ = sweep(lab, cnt, lambda: O.conv2d(x0, w, b, stride=s, pad=(k // 2, k // 2), x1=x1, up_hw=up), Co,
                   (C0 + C1) * k * k, 0)
    tot_h += a_
    tot_b += b_
    del x0, x1, w
if args.only in ("", "unet"):
    for cnt, M, N, K, geglu in UNET_GEMM:
        A = torch.randn(M, K, device=dev, generator=g).to(dt)
        Bw = (torch.randn(N, K, device=dev, generator=g) / math.sqrt(K)).to(dt)
        if geglu:
            bias = torch.zeros(N, device=dev)
            out = torch.empty(M, N // 2, dtype=dt, device=dev)
            fn = lambda: L.call("irx_op_gemm_geglu", O.S(), L.IRX_BF16, M, N, K, O.P(A), O.P(Bw), O.P(bias), O.P(out))
        else:
            R = torch.randn(M, N, device=dev, generator=g).to(dt)
            fn = lambda: O.gemm(A, Bw, residual=R)
        a_, b_ = sweep(f"gemm M{M} N{N} K{K}" + (" geglu" if geglu else ""), cnt, fn, N, K, geglu)
        tot_h += a_
        tot_b += b_
print(f"TOTAL heuristic {tot_h / 1e3:.2f} ms  best {tot_b / 1e3:.2f} ms per pass")
