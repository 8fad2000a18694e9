"""PSNR / SSIM reproduced to 3 significant figures (north star; src/metrics.py:82-95 semantics) on bench.py's
configs[0] parity images, against the CPU reference path's values committed in tests/golden/parity_cfg0_metrics.json
(tests/golden/make_golden_parity.py).

Stage isolation (profiles/r05_parity_stages.txt, scripts/parity_stages.py): with the UNet in bf16 the mean SSIM moves
by +1e-5 (VAE fp16 or fp32); with the VAE in bf16 it moves by -1.3e-4 whatever the UNet's type (fp32 / fp16 / bf16
UNet), which crosses the third figure (0.0660 vs 0.0661).  So the bench engine runs the UNet and CLIP in bf16 and the
VAE in fp16 (the same MFMA rate), and RestorationPipeline defaults to fp16 (the reference's GPU dtype,
src/inference.py:57).  Both must match at 3 s.f.; the all-bf16 engine is reported, not asserted (its known miss).

This is a random-weight proxy: with seeded random SD-1.5 weights the outputs are far from the clean
images (PSNR ~ 9.7 dB, SSIM ~ 0.066 against them), so a 3 s.f. match of noise-level SSIM is weak evidence on its own.
Each engine is therefore also held per pixel to the fp32 engine's output on the same inputs (the fp32 engine is
within 1e-3 per pixel of the CPU reference path, test_e2e_golden_gpu.py): PSNR >= PIX_PSNR_MIN, measured on MI355X
in round 5 as the bench line's psnr_vs_ref (bf16 + fp16 VAE 53.0 dB, fp16 59.6 dB, bf16 49.5 dB) minus a margin.
Parity on real weights is unpinned (no checkpoint is available offline).
"""
import json
from pathlib import Path

import numpy as np
import pytest
import torch

from image_restoration_and_enhancement_amd import metrics as M

pytestmark = pytest.mark.gpu

PIX_PSNR_MIN = {("bf16", "fp16"): 50.0, ("fp16", "fp16"): 56.0, ("bf16", "bf16"): 46.0}

GOLD = json.loads((Path(__file__).resolve().parent / "golden" / "parity_cfg0_metrics.json").read_text())


def sf3(x):
    return float(f"{x:.3g}")


@pytest.fixture(scope="module")
def parity_inputs():
    import bench as B
    from tests import models_common as MC
    pc, sd = MC.state_dicts("denoise")
    clean, noisy = B.synthetic_pairs(len(GOLD["ssim_gt"]), 512, seed=1000)
    return pc, sd, clean, noisy


_fp32_out = {}


def run_engine(device, parity_inputs, unet, vae):
    from oracle import pipeline_ref as PR
    from image_restoration_and_enhancement_amd.pipelines import SDEngine
    pc, sd, clean, noisy = parity_inputs
    prompt, strength, steps, guidance = PR.TASKS["denoise"]
    eng = SDEngine(pc, unet, device, state_dicts=sd, vae_dtype=vae)
    eng.cfg.scheduler.kind = "pndm"          # the saved scheduler (configs[0])
    out = eng.img2img(torch.from_numpy(noisy).to(device).contiguous(), prompt, strength, steps, guidance, seed=42)
    return out.images_u8.cpu().numpy()


def fp32_images(device, parity_inputs):
    if "x" not in _fp32_out:
        _fp32_out["x"] = run_engine(device, parity_inputs, "fp32", "fp32")
    return _fp32_out["x"]


@pytest.mark.parametrize("unet,vae,assert_match", [("bf16", "fp16", True), ("fp16", "fp16", True),
                                                   ("bf16", "bf16", False)])
def test_psnr_ssim_3sf(device, parity_inputs, unet, vae, assert_match):
    pc, sd, clean, noisy = parity_inputs
    imgs = run_engine(device, parity_inputs, unet, vae)
    ref32 = fp32_images(device, parity_inputs)
    pix = [float(M.psnr(ref32[i], imgs[i])) for i in range(len(imgs))]
    ps = [M.psnr(clean[i], imgs[i]) for i in range(len(imgs))]
    ss = [M.ssim(clean[i], imgs[i]) for i in range(len(imgs))]
    rp, rs = float(np.mean(GOLD["psnr_gt"])), float(np.mean(GOLD["ssim_gt"]))
    mp, ms = float(np.mean(ps)), float(np.mean(ss))
    d_ssim = [s - r for s, r in zip(ss, GOLD["ssim_gt"])]
    d_psnr = [p - r for p, r in zip(ps, GOLD["psnr_gt"])]
    print(f"\nUNet {unet} VAE {vae}: PSNR {mp:.5f} (ref {rp:.5f}), SSIM {ms:.6f} (ref {rs:.6f}); per image dSSIM "
          f"{[round(x, 6) for x in d_ssim]} dPSNR {[round(x, 5) for x in d_psnr]}; PSNR vs the fp32 engine "
          f"{[round(x, 2) for x in pix]} dB")
    assert min(pix) >= PIX_PSNR_MIN[(unet, vae)], pix
    if not assert_match:
        return
    assert sf3(mp) == sf3(rp) and sf3(ms) == sf3(rs), (mp, rp, ms, rs)
    assert max(abs(x) for x in d_ssim) < 6e-5 and max(abs(x) for x in d_psnr) < 2e-3
