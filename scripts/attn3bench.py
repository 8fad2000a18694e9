#!/usr/bin/env python3
"""attn3 micro-benchmark at the bench's UNet shapes (batch 16 = 8 images x CFG): interleaved rounds in one
process over variants (v3 interleaved heads / v3 head-major / v3 without the XCD grouping / round-1 kernel),
bf16 and fp16.  HIP events on the current stream.  Usage: python scripts/attn3bench.py [--iters 20]"""
import argparse
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from tests import opref as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--dtypes", default="bf16,fp16")
ap.add_argument("--only", default="", help="run only shapes whose label contains this (e.g. 'self d40 L4096')")
ap.add_argument("--variants", default="", help="comma list of variants to run (default all)")
a = ap.parse_args()
dev = torch.device("cuda")
L.load()
g = torch.Generator(device=dev).manual_seed(0)
DT = {"bf16": torch.bfloat16, "fp16": torch.float16}


def variants(dt, B, Lq, Lk, C):
    H, d = 8, C // 8
    q = torch.randn(B, Lq, C, device=dev, generator=g).to(dt)
    k = torch.randn(B, Lk, C, device=dev, generator=g).to(dt)
    v = torch.randn(B, Lk, C, device=dev, generator=g).to(dt)
    hm = [x.view(B, x.shape[1], H, d).transpose(1, 2).contiguous() for x in (q, k, v)]
    o = torch.empty(B, H, Lq, d, dtype=dt, device=dev)

    def opt(**kw):
        for n, val in kw.items():
            L.call("irx_set_option", n.encode(), val)

    def run_il():
        O.attention(q, k, v, H)

    def run_hm():
        L.call("irx_op_attention_hm", O.S(), O.DT[dt], B, H, Lq, Lk, d, O.P(hm[0]), O.P(hm[1]), O.P(hm[2]),
               O.P(o), 1.0 / math.sqrt(d))
    vs = {"v3": (lambda: opt(attn_xcd=1), run_il),
          "v3-hm": (lambda: opt(attn_xcd=1), run_hm),
          "v3-noxcd": (lambda: opt(attn_xcd=0), run_il)}
    return vs


for dname in a.dtypes.split(","):
    dt = DT[dname]
    for lab, B, Lq, Lk, C in [("self d40 L4096", 16, 4096, 4096, 320), ("cross d40", 16, 4096, 77, 320),
                              ("self d80 L1024", 16, 1024, 1024, 640), ("self d160 L256", 16, 256, 256, 1280),
                              ("self d40 L9216 b16", 16, 9216, 9216, 320)]:
        if a.only and a.only not in lab:
            continue
        vs = variants(dt, B, Lq, Lk, C)
        if a.variants:
            vs = {k: v for k, v in vs.items() if k in a.variants.split(",")}
        flops = 4.0 * B * Lq * Lk * C
        best = {x: 1e9 for x in vs}
        for _ in range(a.rounds):
            for name, (setup, fn) in vs.items():
                setup()
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                best[name] = min(best[name], e0.elapsed_time(e1) / a.iters * 1e3)
        L.call("irx_set_option", b"attn_xcd", 1)
        print(f"{dname} {lab:20s} " + " | ".join(f"{x} {t:8.1f}us {flops / t / 1e6:6.1f}TF"
                                               for x, t in best.items()), flush=True)
