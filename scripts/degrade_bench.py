#!/usr/bin/env python3
"""Throughput of the synthetic-degradation kernels on a resident uint8 batch (64 x 512 x 512 x 3):
algorithmic HBM bytes per launch / event time, against the 8 TB/s HBM peak."""
import random
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import degrade as D  # noqa: E402
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402

dev = torch.device("cuda")
B, H, W = 64, 512, 512
x = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev)
n = x.numel()


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


out = torch.empty_like(x)
z = torch.randn(x.shape, device=dev)
gray = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
ks = torch.full((B,), 7, dtype=torch.int32, device=dev)
blur = torch.empty_like(x)
lr = torch.empty((B, H // 4, W // 4, 3), dtype=torch.uint8, device=dev)
random.seed(0)
strokes = [D.draw_free_form_strokes(H, W, (8, 15), (20, 40)) for _ in range(B)]
S, P = D._s, D._p
segs, thick, off = [], [], [0]
for st in strokes:
    for pts, t in st:
        for (x0, y0), (x1, y1) in zip(pts[:-1], pts[1:]):
            segs.append((x0, y0, x1, y1))
            thick.append(t)
    off.append(len(segs))
sg = torch.tensor(segs, dtype=torch.int32, device=dev)
th = torch.tensor(thick, dtype=torch.int32, device=dev)
of = torch.tensor(off, dtype=torch.int32, device=dev)
mask = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
rows = [
    ("noise (in-kernel Philox)", lambda: L.call("irx_degrade_noise", S(), P(x), n, 6.0, None, 1, P(out)), 2 * n),
    ("noise (given fp32 draws)", lambda: L.call("irx_degrade_noise", S(), P(x), n, 6.0, P(z), 0, P(out)), 6 * n),
    ("gauss 7x7 + cubic /4", lambda: L.call("irx_degrade_blur_down", S(), P(x), B, H, W, 3, P(ks), 4, P(blur), P(lr)),
     3 * n + n // 16),
    ("gray lab", lambda: L.call("irx_degrade_gray", S(), P(x), n // 3, 1, 0, P(gray)), n + n // 3),
    ("strokes + masked", lambda: L.call("irx_degrade_strokes", S(), B, H, W, P(sg), P(th), P(of), P(mask), P(x),
                                        P(out)), n // 3 + 2 * n),
]
for name, fn, byt in rows:
    t = timeit(fn)
    print(f"{name:28s} {t * 1e6:9.1f} us  {byt / t / 1e9:8.1f} GB/s  ({byt / t / 8e12:.3f} of 8 TB/s)  "
          f"{B / t:10.0f} img/s")
