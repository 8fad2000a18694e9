#!/usr/bin/env python3
"""Is the large-tile GEMM epilogue's arithmetic independent of a row's position in its tile?  (VERDICT r3 #2a: fp16
GEGLU outputs 1-2 ulp apart between batchings.)  Every one of 16 "images" of 64 rows holds the SAME data, so every
image's output must be identical bit for bit within one call; prints, per variant, the images whose output differs
from image 0's (max |d|).  Variants at the 8x8-level shape (K = 1280, 256 x 256 tiles):
  geglu+ln    folded LayerNorm + fused GEGLU (irx_op_gemm_ln_fold, geglu)
  ln          folded LayerNorm, plain epilogue, 256x256 tiles forced (gemm_force)
  plain       plain epilogue, 256x256 tiles forced
  geglu       fused GEGLU, no LayerNorm (irx_op_gemm_geglu)
  python scripts/diag_geglu_pos.py [--opt name=value ...]"""
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
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--hw", type=int, default=64)
    ap.add_argument("--K", type=int, default=1280)
    a = ap.parse_args()
    L.load()
    for o in a.opt:
        k, v = o.split("=")
        L.call("irx_set_option", k.encode(), int(v))
    dev = torch.device("cuda")
    hw, C = a.hw, a.K
    N = 8 * C
    g = torch.Generator().manual_seed(0)
    x1 = torch.randn(hw, C, generator=g) + 0.3
    W = torch.randn(N, C, generator=g) / math.sqrt(C)
    b = torch.randn(N, generator=g) * 0.3
    gamma = torch.randn(C, generator=g) * 0.2 + 1
    beta = torch.randn(C, generator=g) * 0.1
    perm = geglu64_order(N)
    for dt in (torch.float16, torch.bfloat16):
        x = x1.repeat(16, 1).to(dt).to(dev).contiguous()
        xf = x.float()
        mean = xf.mean(-1)
        rstd = torch.rsqrt(((xf - mean[:, None]) ** 2).mean(-1) + 1e-5)
        rs = torch.stack([rstd, rstd * mean], -1).contiguous()
        Wg = (W * gamma)[perm].to(dt).to(dev).contiguous()
        u = Wg.double().sum(1).float().contiguous()
        v = (W.double() @ beta.double() + b.double()).float()[perm].to(dev).contiguous()
        Wp = W[perm].to(dt).to(dev).contiguous()
        bp = b[perm].to(dev).contiguous()
        M = x.shape[0]

        def ln_fold(geglu):
            out = torch.empty(M, N // 2 if geglu else N, dtype=dt, device=dev)
            L.call("irx_op_gemm_ln_fold", O.S(), O.DT[dt], M, N, C, O.P(x), O.P(Wg), O.P(u), O.P(v), O.P(rs), None, 0,
                   int(geglu), O.P(out))
            return out

        def geglu_plain():
            out = torch.empty(M, N // 2, dtype=dt, device=dev)
            L.call("irx_op_gemm_geglu", O.S(), O.DT[dt], M, N, C, O.P(x), O.P(Wp), O.P(bp), O.P(out))
            return out
        variants = {
            "geglu+ln": (lambda: ln_fold(True), {}),
            "ln": (lambda: ln_fold(False), {"gemm_force": 25625601}),
            "plain": (lambda: O.gemm(x, Wp, bias=bp), {"gemm_force": 25625601}),
            "geglu": (geglu_plain, {}),
        }
        for name, (fn, opts) in variants.items():
            try:
                with L.option(op_imgs=16, **opts):
                    out = fn()
                torch.cuda.synchronize()
            except L.IrxError as e:
                print(f"{dt} {name}: not run ({e})", flush=True)
                continue
            o = out.float().view(16, hw, -1)
            d = (o - o[:1]).abs().amax(dim=(1, 2))
            bad = [(i, float(d[i])) for i in range(16) if d[i] > 0]
            rows = (o - o[:1]).abs().amax(dim=(0, 2))
            print(f"{dt} {name}: images differing from image 0: {bad}; rows (within an image) ever differing: "
                  f"{[int(r) for r in torch.nonzero(rows > 0).flatten().tolist()][:32]}", flush=True)


if __name__ == "__main__":
    main()
