"""__graft_entry__.smoke(): one tiny img2img denoise (64x64 image, 2 UNet evaluations with CFG,
VAE encode + decode, CLIP) through the native path on cuda:0, checked against the CPU oracle."""
from __future__ import annotations

import time

import numpy as np
import torch


def run_smoke() -> None:
    from image_restoration_and_enhancement_amd import _lib
    from image_restoration_and_enhancement_amd.pipelines import SDEngine
    from oracle import pipeline_ref as PR
    from tests import models_common as MC

    assert torch.cuda.is_available(), "smoke() needs a GPU"
    _lib.load()
    dev = torch.device("cuda:0")
    t0 = time.time()
    prompt, strength, steps, guidance = PR.TASKS["denoise"]
    pc, sd = MC.state_dicts("denoise")
    eng = SDEngine(pc, "fp32", dev, state_dicts=sd)
    img = MC.smooth_image(64, 64, seed=11)
    got = eng.img2img(torch.from_numpy(img).to(dev)[None].contiguous(), prompt, strength, steps, guidance,
                      seed=42, want_float=True, n_evals=2)
    torch.cuda.synchronize()
    ref = PR.img2img_ref(MC.oracle_models("denoise"), MC.pil(img), MC.prompt_ids(prompt), MC.prompt_ids(""),
                         strength, steps, guidance, 42, "pndm", n_evals=2)
    d = float(np.abs(got.decoded01[0].cpu().numpy() - ref.decoded_float).max())
    print(f"smoke: native fp32 img2img (2 evals) vs CPU oracle max|d|={d:.2e} ({time.time() - t0:.1f}s)")
    assert d < 1e-3, d
