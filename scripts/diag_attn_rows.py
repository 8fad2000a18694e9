#!/usr/bin/env python3
"""Row-wise check of the attention op at the UNet's cross- / self-attention shapes: a batch of B rows with distinct
K / V per row vs the fp32 reference (per-row relative error) and vs the same rows run as two smaller batches.
  python scripts/diag_attn_rows.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tests import opref as O  # noqa: E402


def main():
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    for dt in (torch.float16, torch.bfloat16):
        for (Lq, Lk, C) in [(1024, 77, 320), (256, 77, 640), (64, 77, 1280), (16, 77, 1280), (1024, 1024, 320),
                            (4096, 77, 320)]:
            B = 16
            q = (torch.randn(B, Lq, C, generator=g)).to(dt)
            k = (torch.randn(B, Lk, C, generator=g)).to(dt)
            v = (torch.randn(B, Lk, C, generator=g)).to(dt)
            qd, kd, vd = q.to(dev), k.to(dev), v.to(dev)
            whole = O.attention(qd, kd, vd, 8).float().cpu()
            parts = torch.cat([O.attention(qd[:6].contiguous(), kd[:6].contiguous(), vd[:6].contiguous(), 8),
                               O.attention(qd[6:].contiguous(), kd[6:].contiguous(), vd[6:].contiguous(), 8)]).float().cpu()
            ref = O.ref_attention(q.float(), k.float(), v.float(), 8)
            err = ((whole - ref).abs().flatten(1).amax(1) / ref.abs().flatten(1).amax(1)).tolist()
            dpart = (whole - parts).abs().flatten(1).amax(1).tolist()
            print(f"{dt} Lq {Lq} Lk {Lk} C {C}: rel err per row max {max(err):.3g} (worst row {err.index(max(err))}), "
                  f"whole vs parts max {max(dpart):.3g}", flush=True)


if __name__ == "__main__":
    main()
