#!/usr/bin/env python3
"""Batch invariance, stage by stage through SDEngine.img2img (8 images as one batch vs 3 + 5): encode, latent sample,
cross-attention K|V, each UNet evaluation's eps (CFG rows), each step's latents, decode.
  python scripts/diag_bi2.py --dtype fp16 --res 256"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from image_restoration_and_enhancement_amd.configs import PipelineConfig  # noqa: E402
from image_restoration_and_enhancement_amd.pipelines import SDEngine, draw_noise, make_planner  # noqa: E402
from tests import models_common as MC  # noqa: E402

PROMPT = "clean high quality photo, no noise, sharp details"


def stages(eng, u8, n_evals):
    B, H, W_, _ = u8.shape
    h, w = H // 8, W_ // 8
    planner = make_planner(eng.cfg.scheduler)
    planner.set_timesteps(50)
    ts, _ = planner.get_timesteps(50, 0.5)
    plans = planner.plan(ts)[:n_evals]
    out = {}
    emb = eng.text_embeddings(PROMPT, True)
    kv = eng.context_kv(emb, B)
    out["kv"] = kv.view(2, B, -1)
    eps1, nz = (x.to(eng.device) for x in draw_noise(42, h, w, 2)[:2])
    img = eng.to_tensor(u8)
    mom = eng.vae.encode(img)
    out["mom"] = mom
    a, b = planner.add_noise_coeffs(int(ts[0]))
    lat = eng.sample_latents(mom, eps1, nz, a, b)
    out["lat0"] = lat.clone()
    for n in range(1, len(plans) + 1):           # the loop over the first n plans, from the same start
        x = lat.clone()
        bufs = eng._loop_buffers(x, plans[:n], True)
        eng._loop_body(x, kv, plans[:n], 5.0, True, None, None, bufs)
        out[f"eps{n - 1}"] = bufs["eps"].view(2, B, h, w, 4).clone()
        out[f"lat{n}"] = x
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp16")
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--split", type=int, default=3, help="first part size (of 8)")
    a = ap.parse_args()
    L.load()
    for o in a.opt:
        k, v = o.split("=")
        L.call("irx_set_option", k.encode(), int(v))
    dev = torch.device("cuda")
    pc, sd = MC.state_dicts("denoise")
    cfg = PipelineConfig.default("denoise")
    cfg.scheduler.kind = "ddim"
    eng = SDEngine(cfg, a.dtype, dev, state_dicts=sd)
    eng.use_graphs = False
    imgs = torch.from_numpy(np.stack([MC.smooth_image(a.res, a.res, seed=50 + i) for i in range(8)])).to(dev)
    W = stages(eng, imgs.contiguous(), 2)
    c = a.split
    P1, P2 = stages(eng, imgs[:c].contiguous(), 2), stages(eng, imgs[c:].contiguous(), 2)
    for k in W:
        dim = 1 if k.startswith("eps") or k == "kv" else 0
        p = torch.cat([P1[k], P2[k]], dim=dim)
        d = (W[k].float() - p.float()).abs()
        d = d.flatten(dim + 1).amax(-1)
        nan = int((~torch.isfinite(W[k].float())).sum()) + int((~torch.isfinite(p.float())).sum())
        print(f"{a.dtype} {a.res} split {a.split} {a.opt} {k}: non-finite {nan}, max|d| {['%.3g' % v for v in d.flatten().tolist()]}",
              flush=True)


if __name__ == "__main__":
    main()
