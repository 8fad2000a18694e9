#!/usr/bin/env python3
"""Check bf16 attention head-dim-40 variants against the fp32 reference (debug aid)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from tests import opref as O  # noqa: E402

dev = torch.device("cuda")
L.load()
g = torch.Generator().manual_seed(0)
for (B, Lq, Lk, C) in [(2, 256, 256, 320), (2, 200, 77, 320), (1, 64, 64, 320), (1, 100, 100, 640)]:
    q, k, v = (torch.randn(B, n, C, generator=g) for n in (Lq, Lk, Lk))
    ref = O.ref_attention(q.bfloat16().float(), k.bfloat16().float(), v.bfloat16().float(), 8, False)
    for var in (0, 1):
        L.call("irx_set_option", b"attn_d40", var)
        got = O.attention(q.bfloat16().to(dev), k.bfloat16().to(dev), v.bfloat16().to(dev), 8)
        print(B, Lq, Lk, C, "variant", var, "rel_err", float(O.rel_err(got, ref)))
L.call("irx_set_option", b"attn_d40", 0)
