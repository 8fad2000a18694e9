#!/usr/bin/env python3
"""Batch invariance per model (which of VAE encode / UNet / VAE decode / CLIP-context depends on the batch):
the same rows as one batch and as two parts; prints max |difference| per model.
  python scripts/diag_bi_models.py --dtype fp16 --res 256"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from image_restoration_and_enhancement_amd.configs import PipelineConfig  # noqa: E402
from image_restoration_and_enhancement_amd.pipelines import SDEngine  # noqa: E402
from tests import models_common as MC  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp16")
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    L.load()
    for o in a.opt:
        k, v = o.split("=")
        L.call("irx_set_option", k.encode(), int(v))
    dev = torch.device("cuda")
    pc, sd = MC.state_dicts("denoise")
    cfg = PipelineConfig.default("denoise")
    eng = SDEngine(cfg, a.dtype, dev, state_dicts=sd)
    eng.use_graphs = False
    g = torch.Generator(device="cpu").manual_seed(0)
    B, h = 8, a.res // 8

    def cmp(name, f, x, cut):
        whole = f(x).float()
        parts = torch.cat([f(x[:cut]).float(), f(x[cut:]).float()])
        d = (whole - parts).abs().flatten(1).amax(1)
        print(f"{a.dtype} {a.res} {a.opt} {name}: max|d| per row {['%.3g' % v for v in d.tolist()]}", flush=True)

    imgs = torch.from_numpy(np.stack([MC.smooth_image(a.res, a.res, seed=50 + i) for i in range(B)])).to(dev)
    cmp("vae.encode", lambda u: eng.vae.encode(eng.to_tensor(u.contiguous())), imgs, 3)
    z = (torch.randn(B, h, h, 8, generator=g) * 0.8).to(eng.tdt).to(dev)
    cmp("vae.decode", lambda t: eng.vae.decode(t.contiguous()), z, 3)
    emb = eng.text_embeddings("clean high quality photo, no noise, sharp details", True)
    x = (torch.randn(2 * B, h, h, eng.unet.cin_pad, generator=g)).to(eng.tdt).to(dev)
    t = torch.full((2 * B,), 500.0, device=dev)

    def unet(xx):
        n = xx.shape[0]
        kv = eng.unet.prepare_context(emb[1:2].expand(n, -1, -1).contiguous())
        out = torch.empty((n, h, h, 4), dtype=torch.float32, device=dev)
        eng.unet.forward(xx.contiguous(), t[:n].contiguous(), kv, 77, out=out)
        return out
    cmp("unet", unet, x, 6)


if __name__ == "__main__":
    main()
