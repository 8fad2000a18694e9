#!/usr/bin/env python3
"""Generate the full-length end-to-end goldens tests/golden/e2e_<case>.npz (run once in the build container;
outputs committed, the oracle never travels to the GPU box).

For every case in tests/models_common.E2E_CASES (BASELINE.json configs[0..4] at their real step counts) this
runs row 0 of the case's synthetic batch through the CPU fp32 restatement of the diffusers pipeline the
reference calls (oracle/pipeline_ref.py: img2img_ref = src/inference.py:486-495 / :566-573 / :664-672,
inpaint_ref = :758-767) with the seeded random SD-1.5 weights (weights.random_state_dict, seed 0), and stores:

  image       uint8 [H, W, 3]   the PIL output (postprocess round)
  decoded16   uint16 [H, W, 3]  round(decoded [0, 1] float * 65535)  (fp32 cases only: the |d| < 1e-3 check;
                                7.6e-6 step)
  latents     fp32 [4, h, w]    the final latents before VAE decode (drift over the whole loop)
  timesteps   int64 [n]         the executed grid
  fp_<model>  fp64 [2]          weights fingerprint (sum, sum |x|) of unet / vae / clip

Usage:  python tests/golden/make_golden_e2e.py [--only cfg2_denoise_bf16] [--threads 8] [--rows first|last|both]
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))

from oracle import pipeline_ref as PR  # noqa: E402
from tests import models_common as MC  # noqa: E402


def run_case(name: str, c: dict, row: int = 0):
    """Row `row` of the case's batch (image seed c["seed"] + row) through the oracle -> e2e_<name>.npz (row 0) or
    e2e_<name>_last.npz (the batch's last row: the engine runs it at the end of the batch, off the row-tile start)."""
    task = c["task"]
    model_task = "inpaint" if task == "inpaint" else "denoise"
    prompt, strength, _, guidance = PR.TASKS[task]
    pc, sd = MC.state_dicts(model_task)
    models = MC.oracle_models(model_task)
    imgs, masks = MC.task_images(task, c["res"], 1, c["seed"] + row)
    ids_n = MC.prompt_ids("") if guidance > 1 else None
    t0 = time.perf_counter()
    with torch.no_grad():
        if task == "inpaint":
            r = PR.inpaint_ref(models, MC.pil(imgs[0]), MC.pil((masks[0] * 255).astype(np.uint8)),
                               MC.prompt_ids(prompt), ids_n, strength, c["steps"], guidance, 42, c["sched"],
                               height=c["res"], width=c["res"])
        else:
            r = PR.img2img_ref(models, MC.pil(imgs[0]), MC.prompt_ids(prompt), ids_n, strength, c["steps"],
                               guidance, 42, c["sched"])
    dt = time.perf_counter() - t0
    out = {"image": np.asarray(r.image), "latents": r.latents[0].float().numpy(),
           "timesteps": np.array(r.timesteps, np.int64), "cpu_seconds": np.array(dt), "row": np.array(row)}
    if c["dtype"] == "fp32":
        out["decoded16"] = np.round(r.decoded_float * 65535.0).astype(np.uint16)
    for k in ("unet", "vae", "clip"):
        out[f"fp_{k}"] = MC.weight_fingerprint(sd[k])
    tag = name if row == 0 else f"{name}_last"
    np.savez_compressed(HERE / f"e2e_{tag}.npz", **out)
    print(f"{tag}: row {row}, {len(r.timesteps)} evals, {dt:.0f} s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", action="append", default=[])
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--rows", default="first", choices=["first", "last", "both"],
                    help="first: row 0 (e2e_<case>.npz); last: the batch's last row (e2e_<case>_last.npz)")
    a = ap.parse_args()
    if a.threads:
        torch.set_num_threads(a.threads)
    for name, c in MC.E2E_CASES.items():
        if a.only and name not in a.only:
            continue
        if "golden" in c:            # another engine on an existing case's inputs: that case's golden serves
            continue
        if a.rows in ("first", "both"):
            run_case(name, c)
        if a.rows in ("last", "both") and c["batch"] > 1:
            run_case(name, c, c["batch"] - 1)


if __name__ == "__main__":
    main()
