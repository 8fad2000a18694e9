#!/usr/bin/env python3
"""Prediction driver over the native engine — same CLI and on-disk layout as the reference's
`scripts/generate_predictions.py` (`{output_root}/{task}/{split}/<input file name>`, PIL save by extension),
sharded across GPUs when launched with torchrun (one process per GPU, contiguous shards of each task's
file list, no collectives besides the initial barrier).

Modes:
  --mode faithful  (default) calls `RestorationPipeline.process(img, [task], **kwargs)` per image exactly as the
                   reference does, including its quirk that denoise / sr reached through process() run the
                   classical fallbacks (src/inference.py:859-870);
  --mode batched   runs the diffusion path in engine batches of --batch equal-size images
                   (`RestorationPipeline.restore_batch`).
"""
from __future__ import annotations

import argparse
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from PIL import Image  # noqa: E402

from image_restoration_and_enhancement_amd import dist as D  # noqa: E402
from image_restoration_and_enhancement_amd.inference import RestorationPipeline  # noqa: E402

TASKS = {"denoise": (["denoise"], {}), "sr_x4": (["sr"], {"sr_scale": 4}), "colorize": (["colorize"], {}),
         "inpaint": (["inpaint"], {})}
ENGINE_TASK = {"denoise": "denoise", "sr_x4": "sr", "colorize": "colorize", "inpaint": "inpaint"}


def main():
    ap = argparse.ArgumentParser(description="Generate predictions on test set")
    ap.add_argument("--test_root", default="data/pairs")
    ap.add_argument("--output_root", default="outputs/predictions")
    ap.add_argument("--split", default="test", choices=["train", "val", "test"])
    ap.add_argument("--mode", default="faithful", choices=["faithful", "batched"])
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--random-weights", action="store_true", help="seeded random SD-1.5 weights (smoke runs)")
    ap.add_argument("--dtype", default=None, help="engine dtype: fp16 (default, the reference GPU dtype) | bf16 | fp32")
    a = ap.parse_args()
    # the driver needs no data collectives (shards are independent; one closing barrier): gloo, so several
    # ranks may also share one GPU
    rank, world, local = D.init(backend="gloo")
    test_root, output_root = Path(a.test_root).resolve(), Path(a.output_root).resolve()
    if not test_root.exists():
        print(f"Error: Test root not found: {test_root}")
        sys.exit(1)
    import torch
    n_dev = torch.cuda.device_count()
    device = f"cuda:{local % n_dev}" if world > 1 and n_dev else "auto"
    cfg = None
    if a.random_weights:
        rnd = {"fine_tuned_dir": "unused", "pretrained_id": "unused", "weights": "random"}
        cfg = {t: dict(rnd) for t in ("denoise", "sr", "colorize", "inpaint")}
    if a.dtype:
        cfg = dict(cfg or {})
        cfg["engine"] = {"dtype": a.dtype}
    pipe = RestorationPipeline(device=device, config=cfg)
    for task, (task_list, kwargs) in TASKS.items():
        in_dir = test_root / task / a.split / "input"
        out_dir = output_root / task / a.split
        if not in_dir.exists():
            if rank == 0:
                print(f"Skipping {task}: input directory not found: {in_dir}")
            continue
        out_dir.mkdir(parents=True, exist_ok=True)
        files = sorted(list(in_dir.glob("*.jpg")) + list(in_dir.glob("*.png")))
        s, e = D.shard_range(len(files), rank, world)
        mine = files[s:e]
        mask_dir = test_root / task / a.split / "mask" if task == "inpaint" else None

        def mask_for(p):
            mp = mask_dir / p.name if mask_dir else None
            return Image.open(mp).convert("L") if mp is not None and mp.exists() else None

        if a.mode == "faithful":
            for p in mine:
                try:
                    img = Image.open(p).convert("RGB")
                    kw = dict(kwargs)
                    if task == "inpaint":
                        kw["mask"] = mask_for(p)
                    pipe.process(img, task_list, **kw)["final"].save(out_dir / p.name)
                except Exception as ex:  # same per-file error handling as the reference driver
                    print(f"\nError processing {p.name}: {ex}")
        else:
            for k in range(0, len(mine), a.batch):
                chunk = mine[k:k + a.batch]
                imgs = [Image.open(p).convert("RGB") for p in chunk]
                masks = [mask_for(p) for p in chunk] if task == "inpaint" else None
                outs = pipe.restore_batch(ENGINE_TASK[task], imgs, masks=masks, max_batch=a.batch)
                for p, o in zip(chunk, outs):
                    o.save(out_dir / p.name)
        print(f"[rank {rank}] {task}: {len(mine)} images processed")
    D.barrier()
    if rank == 0:
        print(f"\nPredictions saved to: {output_root}")


if __name__ == "__main__":
    main()
