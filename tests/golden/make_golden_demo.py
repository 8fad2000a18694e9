#!/usr/bin/env python3
"""Generate the demo-fixture goldens tests/golden/demo_<case>.npz (run once in the build container; outputs
committed, the oracle never travels to the GPU box).

Inputs are the reference's own demo fixtures, `data/demo/images/*` and `data/demo/mask/*` — the files the Gradio
app feeds to `RestorationPipeline.process` (app.py:296-330) — copied byte for byte into
tests/golden/demo/ (their sha256 is stored in each golden and re-checked by the test).  Their odd sizes give odd
latents (500x333 -> 496x328 -> 62x41, 640x457 -> 80x57, 160x114 -> 20x14, 125x83 -> 15x10), which exercise the
LANCZOS resize to a multiple of 8 and the UNet's `forward_upsample_size` path; two of them are grayscale `L` PNGs.

Each case is one `RestorationPipeline` entry point at its reference parameters, run through the CPU fp32
restatement of the diffusers call it makes (oracle/pipeline_ref.py) with the seeded random SD-1.5 weights
(weights.random_state_dict, seed 0 — what `config[task]["weights"] = "random"` loads):
  denoise   src/inference.py:478-495   img2img, strength 0.5, 20 PNDM steps (11 evals), CFG 5.0
  sr        src/inference.py:549-573   img2img at the literal input size, strength 0.8, 20 PNDM steps, no CFG
  colorize  src/inference.py:612-672   L -> channel 0 replicated (:633-639), strength 0.75, 30 PNDM steps, CFG 7.5
  inpaint   src/inference.py:705-767   mask normalised to the image (:778-803), 512x512, strength 0.6,
                                       30 DDIM steps, CFG 5.0

Stored per case: image (uint8 PIL output), decoded16 (round(decoded [0, 1] * 65535), for the |d| < 1e-3 check),
latents (final, [4, h, w]), timesteps, fp_<model> weight fingerprints, sha_<input> of the fixture files.

Usage:  python tests/golden/make_golden_demo.py [--only denoise1] [--threads 8]
"""
from __future__ import annotations

import argparse
import hashlib
import sys
import time
from pathlib import Path

import numpy as np
import torch
from PIL import Image

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))

from oracle import pipeline_ref as PR  # noqa: E402
from tests import models_common as MC  # noqa: E402

DEMO = HERE / "demo"

DEMO_CASES = MC.DEMO_CASES


def sha256(p: Path) -> str:
    return hashlib.sha256(p.read_bytes()).hexdigest()


def gray_to_rgb(image: Image.Image) -> Image.Image:
    """src/inference.py:633-639: the single (or first) channel replicated to RGB."""
    a = np.array(image)
    if a.ndim == 2:
        return Image.fromarray(np.repeat(a[..., None], 3, axis=2))
    return Image.fromarray(np.repeat(a[..., :1], 3, axis=2))


def run_case(name: str):
    task, img_f, mask_f = DEMO_CASES[name]
    model_task = "inpaint" if task == "inpaint" else "denoise"
    prompt, strength, steps, guidance = PR.TASKS[task]
    pc, sd = MC.state_dicts(model_task)
    models = MC.oracle_models(model_task)
    image = Image.open(DEMO / img_f)
    image.load()
    ids_n = MC.prompt_ids("") if guidance > 1 else None
    t0 = time.perf_counter()
    with torch.no_grad():
        if task == "inpaint":
            mask = PR.normalize_mask_ref(Image.open(DEMO / mask_f), image.size)
            r = PR.inpaint_ref(models, image, mask, MC.prompt_ids(prompt), ids_n, strength, steps, guidance, 42,
                               pc.scheduler.kind)
        else:
            image = gray_to_rgb(image) if task == "colorize" else image.convert("RGB")
            r = PR.img2img_ref(models, image, MC.prompt_ids(prompt), ids_n, strength, steps, guidance, 42, pc.scheduler.kind)
    dt = time.perf_counter() - t0
    out = {"image": np.asarray(r.image), "decoded16": np.round(r.decoded_float * 65535.0).astype(np.uint16),
           "latents": r.latents[0].float().numpy(), "timesteps": np.array(r.timesteps, np.int64),
           "cpu_seconds": np.array(dt), "sha_image": np.array(sha256(DEMO / img_f))}
    if mask_f:
        out["sha_mask"] = np.array(sha256(DEMO / mask_f))
    for k in ("unet", "vae", "clip"):
        out[f"fp_{k}"] = MC.weight_fingerprint(sd[k])
    np.savez_compressed(HERE / f"demo_{name}.npz", **out)
    print(f"demo_{name}: {task} {img_f} -> {out['image'].shape}, latents {out['latents'].shape}, "
          f"{len(r.timesteps)} evals, {dt:.0f} s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", action="append", default=[])
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args()
    if a.threads:
        torch.set_num_threads(a.threads)
    for name in DEMO_CASES:
        if not a.only or name in a.only:
            run_case(name)


if __name__ == "__main__":
    main()
