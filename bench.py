#!/usr/bin/env python3
"""Throughput benchmark of the MI355X restoration engine (BASELINE.json metric).

Workload (BASELINE.json configs[1]): the reference's denoise task — SD-1.5 img2img at 512x512,
batch 8 images per GPU, 50 DDIM steps at strength 0.5 (25 UNet evaluations, classifier-free
guidance 5.0 -> UNet batch 16), bf16, seeded random weights of the SD-1.5 architecture (no
checkpoints are available offline), synthetic noisy images.  One "step" is one full pass of the hot
path over one batch: uint8 pixels resident in HBM -> CLIP text encoding -> VAE encode -> posterior
sample + add_noise -> 25 x (UNet + fused CFG/DDIM step) -> VAE decode -> uint8 pixels.

`python bench.py --gpus N --steps K --warmup W` (N > 1 under torch.distributed.run, one rank per
GPU, weak scaling: 8 images per rank).  Rank 0 prints one JSON line.  Also reported:
  roofline     — the dominant MFMA kernel's algorithmic TFLOP/s (HIP events around every launch
                 of it during a profiled repeat of the timed steps) against the 2.5 PF bf16 dense peak;
  cpu_baseline — the fp32 PyTorch-CPU restatement of the reference path (oracle/, the reference's
                 own CPU path through diffusers cannot run here), timed on a bounded sample on the
                 host cores (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from image_restoration_and_enhancement_amd import dist as D  # noqa: E402
from image_restoration_and_enhancement_amd import weights as W  # noqa: E402
from image_restoration_and_enhancement_amd.configs import PipelineConfig  # noqa: E402
from image_restoration_and_enhancement_amd.pipelines import SDEngine, draw_noise  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, spec; no sparsity)
PEAK_F32_TFLOPS = 157.3
PROMPT = "clean high quality photo, no noise, sharp details"       # src/inference.py:87
# algorithmic GFLOP per unit (SURVEY.md §8d / BASELINE.md §2, 2*MAC over conv + linear + attention)
F_UNET_512, F_ENC_512, F_DEC_512 = 808.0, 1118.7, 2518.3


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synthetic_batch(n: int, res: int, seed: int) -> np.ndarray:
    """Smooth structured images + Gaussian noise sigma in [5, 8] (scripts/make_synthetic_pairs.py:29-35)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:res, 0:res].astype(np.float32)
    out = []
    for i in range(n):
        f = rng.uniform(0.01, 0.05, size=(3, 2))
        ph = rng.uniform(0, 6.28, size=3)
        img = np.stack([128 + 100 * np.sin(f[c, 0] * xx + f[c, 1] * yy + ph[c]) for c in range(3)], -1)
        img = img + rng.normal(0, rng.uniform(5, 8), img.shape)
        out.append(np.clip(img, 0, 255).astype(np.uint8))
    return np.stack(out)


def build_engine(cfg, dtype, device, rank):
    eng = SDEngine(cfg, dtype, device, weights="none")
    models = eng.models()
    sds = None
    if rank == 0:
        sds = {k: W.random_state_dict(k, getattr(cfg, k), 0) for k in models}
        blobs = {k: m.pack(sds[k]).to(device) for k, m in models.items()}
    else:
        blobs = {k: torch.empty(m.blob_bytes(), dtype=torch.uint8, device=device) for k, m in models.items()}
    D.broadcast_blobs(blobs)            # RCCL broadcast of the frozen weights over xGMI (N > 1)
    for k, m in models.items():
        m.bind_blob(blobs[k])
    return eng, sds


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes (scripts/pmc_traffic.py;
    FETCH_SIZE x2 + WRITE_SIZE per the gfx950 note), or None when no pass for this kernel is committed."""
    for f in sorted(Path(__file__).resolve().parent.glob("profiles/*pmc_traffic*.json"), reverse=True):
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        if d.get("kernel") and d["kernel"] in kernel:
            return round(d["bytes_per_launch"])
    return None


def cpu_baseline(cfg, sds, res: int, steps: int, strength: float, threads: int) -> dict:
    """fp32 CPU restatement: 1 image; VAE encode + 1 CFG UNet eval (batch 2) + VAE decode, extrapolated
    to the full per-image schedule (n_evals UNet evals)."""
    from oracle import sd_ref
    torch.set_num_threads(threads)
    n_evals = min(int(steps * strength), steps)
    h = res // 8
    g = torch.Generator().manual_seed(0)
    img = torch.rand(1, 3, res, res, generator=g) * 2 - 1
    ctx = torch.randn(2, 77, 768, generator=g)
    with torch.no_grad():
        t0 = time.perf_counter()
        mom = sd_ref.vae_encode_moments(sds["vae"], cfg.vae, img)
        t1 = time.perf_counter()
        x = torch.randn(2, 4, h, h, generator=g)
        sd_ref.unet_forward(sds["unet"], cfg.unet, x, torch.tensor(481), ctx)
        t2 = time.perf_counter()
        sd_ref.vae_decode(sds["vae"], cfg.vae, mom[:, :4])
        t3 = time.perf_counter()
    per_img = (t1 - t0) + n_evals * (t2 - t1) + (t3 - t2)
    return {"value": round(1.0 / per_img, 6), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"1 image {res}x{res}: VAE encode {t1 - t0:.2f}s + 1 CFG UNet eval (batch 2) "
                      f"{t2 - t1:.2f}s x {n_evals} + VAE decode {t3 - t2:.2f}s, fp32 PyTorch-CPU restatement "
                      f"(oracle/sd_ref.py), {per_img:.1f}s/image extrapolated"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=8, help="images per GPU")
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--sched-steps", type=int, default=50)
    ap.add_argument("--strength", type=float, default=0.5)
    ap.add_argument("--guidance", type=float, default=5.0)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--opt", action="append", default=[], help="irx_set_option name=value (A/B experiments)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    args = ap.parse_args()

    rank, world, local = D.init()
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    L.load()
    for o in args.opt:
        k, v = o.split("=")
        L.call("irx_set_option", k.encode(), int(v))

    cfg = PipelineConfig.default("denoise")
    cfg.scheduler.kind = "ddim"          # BASELINE.json: "50 DDIM steps" (explicit override of the saved PNDM)
    t_init = time.perf_counter()
    eng, sds = build_engine(cfg, args.dtype, device, rank)
    imgs = torch.from_numpy(synthetic_batch(args.batch, args.res, seed=rank)).to(device).contiguous()
    noise = draw_noise(42, args.res // 8, args.res // 8, 2)
    log(f"[rank {rank}] engine ready in {time.perf_counter() - t_init:.1f}s")

    def step():
        eng._ctx_cache.clear()              # text encoding is part of every pass
        return eng.img2img(imgs, PROMPT, args.strength, args.sched_steps, args.guidance, seed=42, noise=noise)

    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    el = D.max_over_ranks(time.perf_counter() - t0, device)
    n_evals = len(out.timesteps)
    images = args.batch * world * args.steps
    value = images / el
    cfg_f = 2 if args.guidance > 1 else 1
    tflop_img = (n_evals * cfg_f * F_UNET_512 + F_ENC_512 + F_DEC_512) / 1000.0 * (args.res / 512) ** 2

    roofline = None
    if not args.no_roofline:
        torch.cuda.synchronize()
        L.profile_begin()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        prof = L.profile_end()
        tot_ms = sum(p[2] for p in prof if p[3] > 0)
        tot_fl = sum(p[3] for p in prof)
        prof.sort(key=lambda p: -p[2])
        if rank == 0:
            log(f"profiled {args.steps} steps: {tot_fl / 1e12 / (args.steps * args.batch):.2f} TFLOP/img counted, "
                f"MFMA-kernel time {tot_ms / args.steps:.1f} ms/step")
            for name, cnt, ms, fl in prof[:18]:
                log(f"  {ms / args.steps:8.1f} ms/step {cnt // args.steps:5d} launches/step "
                    f"{fl / ms / 1e9 if ms else 0:7.1f} TF/s  {name}")
        name, cnt, ms, fl = next(p for p in prof if p[3] > 0)   # dominant MFMA kernel
        peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
        ach = fl / (ms * 1e-3) / 1e12
        roofline = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                    "frac": round(ach / peak, 4), "traffic": pmc_traffic(name), "kernel": name,
                    "launches": cnt, "avg_launch_us": round(ms * 1e3 / cnt, 2),
                    "flops_per_launch": fl / cnt,
                    "all_mfma_kernels_tflops": round(tot_fl / (tot_ms * 1e-3) / 1e12, 2)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, sds, args.res, args.sched_steps, args.strength, args.cpu_threads)

    if rank == 0:
        line = {
            "metric": "restored images/sec @512x512, 50 DDIM steps",
            "value": round(value, 4), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic 512x512 noisy images (sigma 5-8), seeded random SD-1.5 weights",
            "config": {"workload": f"denoise img2img {args.res}x{args.res}, batch {args.batch}/GPU, "
                                   f"{args.sched_steps} DDIM steps x strength {args.strength} = {n_evals} UNet evals, "
                                   f"CFG {args.guidance} (UNet batch {args.batch * cfg_f})",
                       "global_batch": args.batch * world, "resolution": args.res, "parallelism": f"dp{world}",
                       "tflop_per_image": round(tflop_img, 2),
                       "achieved_tflops_end_to_end": round(value * tflop_img, 1)},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    D.barrier()


if __name__ == "__main__":
    main()
