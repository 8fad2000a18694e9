#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run once in the build container, outputs committed).

Oracles used (none of them travels to the GPU box; only the small outputs below are committed):
  * transformers `CLIPTokenizer.from_pretrained(<reference>/outputs/models/denoising/best/tokenizer)`
    -> tokens.json   (the tokenizer the reference's diffusers pipelines call inside encode_prompt,
       src/inference.py:162-172 -> tokenizer_config.json of the saved model dirs)
  * transformers `CLIPTextModel(CLIPTextConfig.from_pretrained(<reference>/.../text_encoder))` with the
    seeded weights `weights.random_state_dict("clip", cfg, seed=0)` -> clip_text.npz (selected token rows
    and per-token norms of last_hidden_state for ["", denoise prompt])
  * scikit-image 0.18.3 under /opt/conda/bin/python3.9 (peak_signal_noise_ratio, structural_similarity
    multichannel=True, color.rgb2lab) -> metrics.json on the uint8 pairs stored in metrics_inputs.npz
    (the calls the reference makes at src/metrics.py:82-95, :115-148)

Usage:  python tests/golden/make_golden.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))

PROMPTS = [
    "",
    "clean high quality photo, no noise, sharp details",
    "high quality, detailed, sharp",
    "vibrant realistic natural colors, colorful, high quality photo, detailed, full color, rich colors",
    "high quality detailed photo",
    "high quality detailed photo, realistic",
    "A photo of a cat sitting on the window-sill at dusk!",
    "restore this OLD photograph: remove scratches & fix the torn corner (1950s, b/w)",
    " ".join(["very"] * 90) + " long prompt that must be truncated",
]
CLIP_ROWS = list(range(12)) + [40, 76]


def make_tokens(ref: Path):
    from transformers import CLIPTokenizer
    tok = CLIPTokenizer.from_pretrained(str(ref / "outputs/models/denoising/best/tokenizer"))
    out = {p: tok(p, padding="max_length", max_length=77, truncation=True).input_ids for p in PROMPTS}
    (HERE / "tokens.json").write_text(json.dumps(out, indent=0))
    return out


def make_clip(ref: Path, tokens):
    import torch
    from transformers import CLIPTextConfig, CLIPTextModel
    from image_restoration_and_enhancement_amd import weights as W
    from image_restoration_and_enhancement_amd.configs import CLIPConfig

    cfg_dir = ref / "outputs/models/denoising/best/text_encoder"
    hf_cfg = CLIPTextConfig.from_pretrained(str(cfg_dir))
    model = CLIPTextModel(hf_cfg).eval()
    cfg = CLIPConfig.from_dict(json.loads((cfg_dir / "config.json").read_text()))
    sd = W.random_state_dict("clip", cfg, seed=0)
    if not any(k.startswith("text_model.") for k in model.state_dict()):   # transformers >= 5 drops the prefix
        sd = {k[len("text_model."):]: v for k, v in sd.items()}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    missing = [m for m in missing if not m.endswith("position_ids")]
    assert not missing and not unexpected, (missing[:3], unexpected[:3])
    ids = torch.tensor([tokens[""], tokens[PROMPTS[1]]], dtype=torch.int64)
    with torch.no_grad():
        h = model(input_ids=ids).last_hidden_state.float()
    np.savez(HERE / "clip_text.npz", ids=ids.numpy(), rows=np.array(CLIP_ROWS),
             hidden_rows=h[:, CLIP_ROWS].numpy(), token_norms=h.norm(dim=-1).numpy())


SKIMAGE_SCRIPT = r"""
import json, sys, numpy as np
from skimage.metrics import peak_signal_noise_ratio as psnr, structural_similarity as ssim
from skimage import color
d = np.load(sys.argv[1])
out = []
for i in range(int(d["n"])):
    gt, pr = d[f"gt{i}"], d[f"pred{i}"]
    mc = gt.ndim == 3
    r = {"psnr": float(psnr(gt, pr, data_range=255.0)),
         "ssim": float(ssim(gt, pr, data_range=255.0, multichannel=mc))}
    if mc:
        a = color.rgb2lab(pr.astype(np.float32) / 255.0); b = color.rgb2lab(gt.astype(np.float32) / 255.0)
        r["delta_e"] = float(np.mean(np.sqrt(np.sum((a - b) ** 2, axis=2))))
        r["lab_px"] = b[1, 2].tolist()
    out.append(r)
print(json.dumps(out))
"""


def make_metrics():
    rng = np.random.default_rng(7)
    pairs = []
    for shape, sigma in (((40, 48, 3), 6.0), ((33, 29, 3), 20.0), ((64, 64, 3), 2.0), ((31, 37), 9.0)):
        yy, xx = np.mgrid[0:shape[0], 0:shape[1]]
        base = 128 + 60 * np.sin(xx / 5.0) * np.cos(yy / 7.0)
        gt = base[..., None] + rng.normal(0, 20, shape if len(shape) == 3 else shape + (1,))
        gt = np.clip(gt.reshape(shape), 0, 255).astype(np.uint8)
        pred = np.clip(gt + rng.normal(0, sigma, shape), 0, 255).astype(np.uint8)
        pairs.append((gt, pred))
    arrs = {"n": np.array(len(pairs))}
    for i, (g, p) in enumerate(pairs):
        arrs[f"gt{i}"], arrs[f"pred{i}"] = g, p
    np.savez(HERE / "metrics_inputs.npz", **arrs)
    py39 = "/opt/conda/bin/python3.9"
    res = subprocess.run([py39, "-c", SKIMAGE_SCRIPT, str(HERE / "metrics_inputs.npz")], check=True,
                         capture_output=True, text=True)
    ver = subprocess.run([py39, "-c", "import skimage; print(skimage.__version__)"], check=True,
                         capture_output=True, text=True).stdout.strip()
    (HERE / "metrics.json").write_text(json.dumps({"skimage": ver, "results": json.loads(res.stdout)}, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    ref = Path(a.reference)
    if a.only in ("", "tokens", "clip"):
        toks = make_tokens(ref)
        if a.only in ("", "clip"):
            make_clip(ref, toks)
    if a.only in ("", "metrics"):
        make_metrics()


if __name__ == "__main__":
    main()
