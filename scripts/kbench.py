#!/usr/bin/env python3
"""Per-shape micro-benchmark of the MFMA conv/GEMM/attention kernels at the UNet's batch-16 (CFG x 8
images) 512x512 shapes.  Times each op with HIP events over N iterations (interleaved variants in
one process) and prints TF/s.  Usage: python scripts/kbench.py [--iters 20] [--only conv|gemm|attn]
"""
from __future__ import annotations

import argparse
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from tests import opref as O  # noqa: E402

CONVS = [  # (label, N, H, W, C0, C1, Cout, k, stride, up)
    ("conv320@64", 16, 64, 64, 320, 0, 320, 3, 1, None),
    ("conv640@32", 16, 32, 32, 640, 0, 640, 3, 1, None),
    ("conv1280@16", 16, 16, 16, 1280, 0, 1280, 3, 1, None),
    ("conv1280@8", 16, 8, 8, 1280, 0, 1280, 3, 1, None),
    ("cat1280+1280->1280@8", 16, 8, 8, 1280, 1280, 1280, 3, 1, None),
    ("cat640+320->320@64", 16, 64, 64, 640, 320, 320, 3, 1, None),
    ("cat320+320->320@64", 16, 64, 64, 320, 320, 320, 3, 1, None),
    ("cat1280+1280->1280@16", 16, 16, 16, 1280, 1280, 1280, 3, 1, None),
    ("cat1280+640->640@32", 16, 32, 32, 1280, 640, 640, 3, 1, None),
    ("up1280@16->32", 16, 16, 16, 1280, 0, 1280, 3, 1, (32, 32)),
    ("vae512@128", 8, 128, 128, 512, 0, 512, 3, 1, None),
    ("vae256@256", 8, 256, 256, 256, 0, 256, 3, 1, None),
    ("vae128@512", 8, 512, 512, 128, 0, 128, 3, 1, None),
    # one parity of a nearest-2x upsampler as a 2x2 conv of the low-resolution input (IRX_LAYOUT_CONV_UP2)
    ("up2p1280@8", 16, 8, 8, 1280, 0, 1280, 2, 1, None),
    ("up2p1280@16", 16, 16, 16, 1280, 0, 1280, 2, 1, None),
    ("up2p640@32", 16, 32, 32, 640, 0, 640, 2, 1, None),
    ("vaeup2p512@64", 8, 64, 64, 512, 0, 512, 2, 1, None),
    ("vaeup2p512@128", 8, 128, 128, 512, 0, 512, 2, 1, None),
    ("vaeup2p256@256", 8, 256, 256, 256, 0, 256, 2, 1, None),
    # ff.net.2 folded through proj_out: 1x1 conv over the concat (h | g)
    ("chain320@64", 16, 64, 64, 320, 1280, 320, 1, 1, None),
    ("chain640@32", 16, 32, 32, 640, 2560, 640, 1, 1, None),
    ("chain1280@16", 16, 16, 16, 1280, 5120, 1280, 1, 1, None),
]
GEMMS = [  # (label, M, N, K)
    ("lin320x320@64", 65536, 320, 320),
    ("lin640x640@32", 16384, 640, 640),
    ("lin1280@16b", 4096, 1280, 1280),
    ("qkv@64", 65536, 960, 320),
    ("ff1@64", 65536, 2560, 320),
    ("ff2@64", 65536, 320, 1280),
    ("lin640@32", 16384, 640, 640),
    ("ff1@32", 16384, 5120, 640),
    ("ff2@32", 16384, 640, 2560),
    ("lin1280@16", 4096, 1280, 1280),
    ("ff1@16", 4096, 10240, 1280),
    # + residual (attn to_out at each level: the store pass reads the residual stream)
    ("chain-as-gemm@32", 16384, 640, 3200),
    ("chain-as-gemm@16", 4096, 1280, 6400),
    ("lin320x320@64+res", 65536, 320, 320, "res"),
    ("lin640x640@32+res", 16384, 640, 640, "res"),
    ("lin1280@16b+res", 4096, 1280, 1280, "res"),
]
ATTNS = [  # (label, B, L, Lk, C)
    ("self d40 L4096", 16, 4096, 4096, 320),
    ("self d80 L1024", 16, 1024, 1024, 640),
    ("self d160 L256", 16, 256, 256, 1280),
    ("cross d40", 16, 4096, 77, 320),
    ("cross d80", 16, 1024, 77, 640),
    ("cross d160", 16, 256, 77, 1280),
]


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--match", default="", help="only shapes whose label contains this")
    ap.add_argument("--ref", action="store_true", help="also time torch (hipBLASLt / MIOpen) on the same shapes")
    ap.add_argument("--variants", default="s2,ring64,small")
    ap.add_argument("--attn-qrep", action="store_true", help="cross-attention: sweep the resident-K/V query groups")
    ap.add_argument("--pf80", action="store_true", help="d = 80 self-attention: option attn_pf80 on / off")
    ap.add_argument("--lnout", action="store_true", help="residual-stream producers with / without LayerNorm partials")
    args = ap.parse_args()
    dev = torch.device("cuda")
    L.load()
    dt = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    base = {"large_tiles": 1, "gemm_deep": 0, "gemm_small": 0, "tile_256x320": 1, "splitk_inkernel": 1, "halo_pipe": 1,
            "gemm_pp": 0, "gemm_force": 0, "gemm_dbg": 0}
    allv = {"s2": {}, "ring64": {"gemm_deep": 2}, "ring32": {"gemm_deep": 1}, "small": {"gemm_small": 1}, "4wave": {"large_tiles": 0},
            "no320": {"tile_256x320": 0}, "redk": {"splitk_inkernel": 0}, "no320redk": {"tile_256x320": 0, "splitk_inkernel": 0},
            "halo1": {"halo_pipe": 0}, "halo2": {"halo_pipe": 1}, "pp0": {"gemm_pp": 0}, "pp1": {"gemm_pp": 1}, "pp2": {"gemm_pp": 2},
            "nm0": {"gemm_nmajor": 0},
            # timing diagnostics (results wrong): 1 no epilogue, 2 no MFMAs, 3 neither
            "dbg1": {"gemm_dbg": 1}, "dbg2": {"gemm_dbg": 2}, "dbg3": {"gemm_dbg": 3},
            # forced tile / split (gemm_force = BM*100000 + BN*100 + splits): the 8x8-level split-K sweep
            **{f"f{bm}x{bn}s{sp}": {"gemm_force": bm * 100000 + bn * 100 + sp}
               for bm in (256, 128) for bn in (320, 256, 128) for sp in (1, 2, 4, 8)}, "nm1": {"gemm_nmajor": 1}, "nm2": {"gemm_nmajor": 2}}
    variants = [(v, allv[v]) for v in args.variants.split(",")]

    def setv(opts):
        for k, v in {**base, **opts}.items():
            L.call("irx_set_option", k.encode(), v)
    if args.only in ("", "conv"):
        for lab, N, H, W, C0, C1, Co, k, s, up in CONVS:
            if args.match not in lab:
                continue
            x0 = torch.randn(N, H, W, C0, device=dev, generator=g).to(dt)
            x1 = torch.randn(N, H, W, C1, device=dev, generator=g).to(dt) if C1 else None
            w = (torch.randn(Co, C0 + C1, k, k, device=dev, generator=g) / math.sqrt((C0 + C1) * k * k)).to(dt)
            b = torch.zeros(Co, device=dev)
            Ho, Wo = up if up else (H, W)
            flops = 2.0 * N * Ho * Wo * Co * (C0 + C1) * k * k
            res = []
            for vn, opts in variants:
                setv(opts)
                ms = timeit(lambda: O.conv2d(x0, w, b, pad=(k // 2, k // 2) if k != 2 else (1, 1), x1=x1, up_hw=up,
                                             out_hw=(H, W) if k == 2 else None), args.iters)
                res.append(f"{vn} {ms * 1e3:8.1f}us {flops / ms / 1e9:7.1f}TF")
            if args.ref:   # MIOpen (torch) channels-last bf16 conv on the same data: a known-good reference
                xr = (torch.cat([x0, x1], -1) if x1 is not None else x0).permute(0, 3, 1, 2)
                if up:
                    xr = torch.nn.functional.interpolate(xr, size=up, mode="nearest")
                xr = xr.contiguous(memory_format=torch.channels_last)
                wr = w.contiguous(memory_format=torch.channels_last)
                ms = timeit(lambda: torch.nn.functional.conv2d(xr, wr, None, s, k // 2), args.iters)
                res.append(f"miopen {ms * 1e3:8.1f}us {flops / ms / 1e9:7.1f}TF")
            print(f"{lab:24s} " + " | ".join(res), flush=True)
    if args.lnout:   # the transformer residual-stream producers: + residual, in place, with / without LN partials
        for M, N, K in ((65536, 320, 320), (16384, 640, 640)):
            A = torch.randn(M, K, device=dev, generator=g).to(dt)
            Bw = (torch.randn(N, K, device=dev, generator=g) / math.sqrt(K)).to(dt)
            bias = torch.zeros(N, device=dev)
            R = torch.randn(M, N, device=dev, generator=g).to(dt)
            C = R.clone()
            parts = torch.empty(M, max(1, N // 320), 2, device=dev)
            flops = 2.0 * M * N * K
            setv({})
            res = []
            runs = [("res", lambda: O.gemm(A, Bw, bias=bias, residual=R)),
                    ("inplace", lambda: O.gemm(A, Bw, bias=bias, residual=C)),
                    ("lnout", lambda: L.call("irx_op_gemm_ln_out", O.S(), O.DT[dt], M, N, K, O.P(A), O.P(Bw), O.P(bias),
                                             O.P(C), O.P(C), O.P(parts), 1 if N == 320 else 0, 1e-5))]
            for vn, fn in runs:
                ms = timeit(fn, args.iters)
                res.append(f"{vn} {ms * 1e3:8.1f}us {flops / ms / 1e9:7.1f}TF")
            print(f"lnout M{M} N{N} K{K}      " + " | ".join(res), flush=True)
    if args.only in ("", "gemm"):
        for lab, M, N, K, *extra in GEMMS:
            if args.match not in lab:
                continue
            A = torch.randn(M, K, device=dev, generator=g).to(dt)
            Bw = (torch.randn(N, K, device=dev, generator=g) / math.sqrt(K)).to(dt)
            R = torch.randn(M, N, device=dev, generator=g).to(dt) if "res" in extra else None
            bias = torch.zeros(N, device=dev) if R is not None else None
            flops = 2.0 * M * N * K
            res = []
            for vn, opts in variants:
                setv(opts)
                ms = timeit(lambda: O.gemm(A, Bw, bias=bias, residual=R), args.iters)
                res.append(f"{vn} {ms * 1e3:8.1f}us {flops / ms / 1e9:7.1f}TF")
            if args.ref:   # hipBLASLt (torch.matmul) on the same data: a known-good reference
                Bt = Bw.t()
                ms = timeit(lambda: torch.matmul(A, Bt), args.iters)
                res.append(f"hipblaslt {ms * 1e3:8.1f}us {flops / ms / 1e9:7.1f}TF")
            print(f"{lab:24s} " + " | ".join(res), flush=True)
    setv({})
    if args.only in ("", "attn"):
        for lab, B, Lq, Lk, C in ATTNS:
            q = torch.randn(B, Lq, C, device=dev, generator=g).to(dt)
            k = torch.randn(B, Lk, C, device=dev, generator=g).to(dt)
            v = torch.randn(B, Lk, C, device=dev, generator=g).to(dt)
            flops = 4.0 * B * Lq * Lk * C
            res = []
            avs = (("pf", {"attn_pf": 1, "attn_q2": 0}), ("q2", {"attn_pf": 1, "attn_q2": 1}))
            if C // 8 == 160:   # d = 160: with / without the whole-tile fragment prefetch
                avs = (("pf160", {"attn_pf160": 1}), ("nopf", {"attn_pf160": 0}))
            if args.pf80 and C // 8 == 80 and Lk > 128:   # d = 80 self-attention: with / without the fragment prefetch
                avs = (("pf80", {"attn_pf80": 2}), ("base", {"attn_pf80": 0}))
            if args.attn_qrep and Lk <= 128:   # resident-K/V query groups per block: auto vs forced counts
                avs = (("auto", {"attn_qrep": 1}),) + tuple((f"qr{q}", {"attn_qrep": q}) for q in (2, 4, 8, 16)) + \
                      (("auto", {"attn_qrep": 1}),)
            for vn, opts in avs:
                with L.option(**opts):
                    ms = timeit(lambda: O.attention(q, k, v, 8), args.iters)
                res.append(f"{vn} {ms * 1e3:8.1f}us {flops / ms / 1e9:7.1f}TF")
            if args.ref:   # torch SDPA (the ROCm flash / CK path) on the same data
                hd = C // 8
                qh, kh, vh = (t.view(B, -1, 8, hd).transpose(1, 2) for t in (q, k, v))
                ms = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(qh, kh, vh), args.iters)
                res.append(f"sdpa {ms * 1e3:8.1f}us {flops / ms / 1e9:7.1f}TF")
            print(f"{lab:24s} " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
