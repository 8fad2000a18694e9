#!/usr/bin/env python3
"""Which stage's 16-bit rounding moves the configs[0] PSNR / SSIM?

  --make-ref OUT.npz   (CPU, this container) run bench.py's configs[0] parity images through the fp32 CPU
                       restatement (oracle/pipeline_ref.py) and save noisy / clean / reference outputs;
  --ref OUT.npz        (GPU) run the same images through the engine with per-model dtypes
                       (UNet / VAE / CLIP) and print per variant: PSNR vs the reference output, mean PSNR /
                       SSIM vs the clean image at full precision and at 3 s.f., and whether they match the
                       reference's at 3 s.f. (bench.py's `psnr_ssim_3sf_match`).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench as B  # noqa: E402
from image_restoration_and_enhancement_amd import metrics as M  # noqa: E402
from image_restoration_and_enhancement_amd import weights as W  # noqa: E402
from image_restoration_and_enhancement_amd.configs import PipelineConfig  # noqa: E402


def make_ref(out: str, n: int) -> None:
    from oracle import pipeline_ref as PR
    from image_restoration_and_enhancement_amd.tokenizer import PromptTokenizer
    from PIL import Image
    prompt, strength, steps, guidance = PR.TASKS["denoise"]
    cfg = PipelineConfig.default("denoise")
    tok = PromptTokenizer()
    ids_p, ids_n = torch.from_numpy(tok(prompt))[None], torch.from_numpy(tok(""))[None]
    sds = {k: W.random_state_dict(k, getattr(cfg, k), 0) for k in ("unet", "vae", "clip")}
    models = PR.Models(sds["unet"], cfg.unet, sds["vae"], cfg.vae, sds["clip"], cfg.clip)
    clean, noisy = B.synthetic_pairs(n, 512, seed=1000)
    refs, dec = [], []
    with torch.no_grad():
        for i in range(n):
            t0 = time.perf_counter()
            r = PR.img2img_ref(models, Image.fromarray(noisy[i]), ids_p, ids_n, strength, steps, guidance, 42, "pndm")
            refs.append(np.asarray(r.image))
            dec.append(r.decoded_float.astype(np.float32))
            print(f"ref {i + 1}/{n}: {time.perf_counter() - t0:.1f} s", flush=True)
    np.savez_compressed(out, clean=clean, noisy=noisy, ref=np.stack(refs), ref_f=np.stack(dec))


def sf3(x: float) -> float:
    return float(f"{x:.3g}")


def run(ref_path: str, variants: list, opts: list) -> None:
    from image_restoration_and_enhancement_amd import _lib as L
    from image_restoration_and_enhancement_amd.pipelines import SDEngine
    from oracle import pipeline_ref as PR
    d = np.load(ref_path)
    clean, noisy, ref, ref_f = d["clean"], d["noisy"], d["ref"], d["ref_f"]
    n = len(ref)
    prompt, strength, steps, guidance = PR.TASKS["denoise"]
    cfg = PipelineConfig.default("denoise")
    sds = {k: W.random_state_dict(k, getattr(cfg, k), 0) for k in ("unet", "vae", "clip")}
    dev = torch.device("cuda", 0)
    L.load()
    for o in opts:
        k, v = o.split("=")
        L.call("irx_set_option", k.encode(), int(v))
    u8 = torch.from_numpy(noisy).to(dev).contiguous()
    gt_ref = [(M.psnr(clean[i], ref[i]), M.ssim(clean[i], ref[i])) for i in range(n)]
    rp, rs = float(np.mean([g[0] for g in gt_ref])), float(np.mean([g[1] for g in gt_ref]))
    print(json.dumps({"variant": "cpu_ref", "psnr_gt": round(rp, 5), "ssim_gt": round(rs, 6),
                      "3sf": [sf3(rp), sf3(rs)]}), flush=True)
    for v in variants:
        ud, vd, cd = (v.split(",") + [None, None])[:3]
        eng = SDEngine(cfg, ud, dev, state_dicts=sds, vae_dtype=vd or None, clip_dtype=cd or None)
        eng.cfg.scheduler.kind = "pndm"
        res = eng.img2img(u8, prompt, strength, steps, guidance, seed=42, want_float=True)
        torch.cuda.synchronize()
        out = res.images_u8.cpu().numpy()
        f = res.decoded01.cpu().numpy()
        ps = [M.psnr(ref[i], out[i]) for i in range(n)]
        gp = [M.psnr(clean[i], out[i]) for i in range(n)]
        gs = [M.ssim(clean[i], out[i]) for i in range(n)]
        mp, ms = float(np.mean(gp)), float(np.mean(gs))
        print(json.dumps({"variant": v, "psnr_vs_ref": [round(x, 3) for x in ps],
                          "rel_l2_float_vs_ref": float(np.linalg.norm(f - ref_f) / np.linalg.norm(ref_f)),
                          "max_abs_float_vs_ref": float(np.abs(f - ref_f).max()),
                          "psnr_gt": round(mp, 5), "ssim_gt": round(ms, 6),
                          "d_psnr_gt": round(mp - rp, 5), "d_ssim_gt": round(ms - rs, 6),
                          "d_ssim_gt_per_image": [round(gs[i] - gt_ref[i][1], 6) for i in range(n)],
                          "3sf": [sf3(mp), sf3(ms)], "match": sf3(mp) == sf3(rp) and sf3(ms) == sf3(rs)}),
              flush=True)
        del eng, res
        torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--make-ref")
    ap.add_argument("--n", type=int, default=4)
    ap.add_argument("--ref")
    ap.add_argument("--variants", default="fp32;bf16;bf16,fp16;bf16,fp32;fp32,bf16;bf16,bf16,fp32;fp16",
                    help="';'-separated unet[,vae[,clip]] dtypes")
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    if a.make_ref:
        make_ref(a.make_ref, a.n)
    if a.ref:
        run(a.ref, a.variants.split(";"), a.opt)


if __name__ == "__main__":
    main()
