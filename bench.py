#!/usr/bin/env python3
"""Throughput benchmark of the MI355X restoration engine (BASELINE.json metric).

Default workload (BASELINE.json configs[1]): the reference's denoise task — SD-1.5 img2img at
512x512, batch 8 images per GPU, 50 DDIM steps at strength 0.5 (25 UNet evaluations, classifier-free
guidance 5.0 -> UNet batch 16), bf16, seeded random weights of the SD-1.5 architecture (no checkpoints
are available offline), synthetic noisy images.  One "step" is one full pass of the hot path over one
batch: uint8 pixels resident in HBM -> CLIP text encoding -> VAE encode -> posterior sample + add_noise
-> n x (UNet + fused CFG/scheduler step) -> VAE decode -> uint8 pixels.

`--task` selects the other BASELINE configs as per-GPU shards (weak scaling; N > 1 under
torch.distributed.run, one rank per GPU):
  sr        configs[2]: sr_x4 128 -> 512 (bicubic pre-upscale), batch 16, strength 0.8, no CFG, 40 evals
  inpaint   configs[3]: 512x512 + stroke masks, 8 images per GPU (32 over 4 GPUs), 9-channel UNet,
            strength 0.6, CFG 5.0, 30 evals, two VAE encodes
  colorize  configs[4]: 768x768 gray, 8 images per GPU (64 over 8 GPUs), fp16, strength 0.75, CFG 7.5,
            37 evals
Algorithmic work per image comes from BASELINE.md §2 (per-resolution UNet / VAE GFLOP, attention
quadratic in the token count), not a (res/512)^2 scaling.

Also reported (rank 0):
  roofline     — the dominant MFMA kernel's algorithmic TFLOP/s (HIP events around every launch of it
                 during a profiled repeat of the timed steps) against the dense MFMA peak;
  cpu_baseline — BASELINE.md §3: the reference CPU path (fp32 PyTorch-CPU restatement, oracle/ — the
                 reference's own diffusers path cannot run here) on configs[0]: full 512x512 denoise
                 images, 20 PNDM steps x strength 0.5 (11 UNet evals, CFG), on this process's usable
                 host cores (N = 1 only);
  parity       — the same configs[0] images through the GPU engines (fp32; the bench's bf16 UNet + CLIP with
                 the fp16 VAE; all-bf16; all-fp16, the reference's GPU dtype): max |decoded pixel difference| of
                 the fp32 engine vs the CPU reference, PSNR/SSIM (metrics.py, pinned to scikit-image) of the
                 bench engine's output vs the CPU reference output, of every output vs the clean ground truth
                 (per image and as means), and whether each engine's mean PSNR / SSIM equal the CPU reference's
                 to 3 significant figures (the north star's "PSNR/SSIM reproduced to 3 s.f.").

Compute types: the bf16 tasks run the UNet and CLIP in bf16 and the VAE in fp16 (same MFMA rate): the bf16 VAE
is the stage whose rounding moves the configs[0] SSIM at the third figure (profiles/r05_parity_stages.txt,
DESIGN.md §5); `--vae-dtype bf16` gives the all-bf16 engine.
"""
from __future__ import annotations

import argparse
import json
import math
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

PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3}   # MI355X dense (MI355X_MICROARCH.md)
# algorithmic GFLOP per unit (2*MAC over conv + linear + attention QK^T / PV)
F_UNET = {128: 45.9, 512: 808.0, 768: 2168.9}
F_ENC = {128: 67.9, 512: 1118.7, 768: 2613.9}
F_DEC = {128: 155.4, 512: 2518.3, 768: 5763.0}
PROMPTS = {   # src/inference.py:86-91
    "denoise": "clean high quality photo, no noise, sharp details",
    "sr": "high quality, detailed, sharp",
    "colorize": "vibrant realistic natural colors, colorful, high quality photo, detailed, full color, rich colors",
    "inpaint": "high quality detailed photo",
}
# BASELINE.json configs[1..4] as per-GPU workloads
TASKS = {
    "denoise": dict(cfg=2, res=512, batch=8, strength=0.5, guidance=5.0, dtype="bf16", vae="fp16", n_enc=1),
    "sr": dict(cfg=3, res=512, lr=128, batch=16, strength=0.8, guidance=0.0, dtype="bf16", vae="fp16", n_enc=1),
    "inpaint": dict(cfg=4, res=512, batch=8, strength=0.6, guidance=5.0, dtype="bf16", vae="fp16", n_enc=2),
    "colorize": dict(cfg=5, res=768, batch=8, strength=0.75, guidance=7.5, dtype="fp16", vae="fp16", n_enc=1),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synthetic_pairs(n: int, res: int, seed: int):
    """(clean, noisy) uint8 [n, res, res, 3]: smooth structured images + Gaussian noise sigma in [5, 8]
    (scripts/make_synthetic_pairs.py:29-35)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:res, 0:res].astype(np.float32)
    clean, noisy = [], []
    for _ in range(n):
        f = rng.uniform(0.01, 0.05, size=(3, 2))
        ph = rng.uniform(0, 6.28, size=3)
        img = np.stack([128 + 100 * np.sin(f[c, 0] * xx + f[c, 1] * yy + ph[c]) for c in range(3)], -1)
        clean.append(np.clip(img, 0, 255).astype(np.uint8))
        img = img + rng.normal(0, rng.uniform(5, 8), img.shape)
        noisy.append(np.clip(img, 0, 255).astype(np.uint8))
    return np.stack(clean), np.stack(noisy)


def stroke_masks(n: int, res: int, seed: int) -> np.ndarray:
    """Free-form stroke masks {0, 1} (scripts/make_synthetic_pairs.py:104-114 shape statistics)."""
    rng = np.random.default_rng(seed)
    out = np.zeros((n, res, res), np.float32)
    for i in range(n):
        for _ in range(rng.integers(2, 5)):
            y, x = rng.integers(0, res, size=2)
            r = int(rng.integers(res // 64, res // 24))
            for _ in range(int(rng.integers(8, 20))):
                y = int(np.clip(y + rng.integers(-res // 16, res // 16), 0, res - 1))
                x = int(np.clip(x + rng.integers(-res // 16, res // 16), 0, res - 1))
                out[i, max(0, y - r):y + r, max(0, x - r):x + r] = 1.0
    return out


def task_inputs(task: str, spec: dict, batch: int, seed: int):
    """Per-task synthetic batch in host memory: (uint8 [B, H, W, 3], optional fp32 mask [B, H, W])."""
    res = spec["res"]
    if task == "sr":
        # LR 128x128 (blurred, 4x down) bicubic pre-upscaled to 512 before img2img
        _, lr = synthetic_pairs(batch, spec["lr"], seed)
        t = torch.from_numpy(lr).permute(0, 3, 1, 2).float()
        up = torch.nn.functional.interpolate(t, size=(res, res), mode="bicubic", align_corners=False)
        return up.round().clamp(0, 255).to(torch.uint8).permute(0, 2, 3, 1).numpy(), None
    clean, noisy = synthetic_pairs(batch, res, seed)
    if task == "colorize":
        gray = (0.299 * clean[..., 0] + 0.587 * clean[..., 1] + 0.114 * clean[..., 2]).round().astype(np.uint8)
        return np.repeat(gray[..., None], 3, axis=3), None
    if task == "inpaint":
        m = stroke_masks(batch, res, seed)
        return (clean * (1 - m[..., None])).astype(np.uint8), m
    return noisy, None


def build_engine(cfg, dtype, device, rank, vae_dtype=None):
    eng = SDEngine(cfg, dtype, device, weights="none", vae_dtype=vae_dtype)
    models = eng.models()
    sds = None
    if rank == 0:
        sds = {k: W.random_state_dict(k, getattr(cfg, k), 0) for k in models}
        blobs = {k: m.pack(sds[k]).to(device) for k, m in models.items()}
    else:
        blobs = {k: torch.empty(m.blob_bytes(), dtype=torch.uint8, device=device) for k, m in models.items()}
    for k, m in models.items():
        m.bind_blob(blobs[k])
    # RCCL broadcast of the frozen weights over xGMI (N > 1): irx_weights_bcast through the C ABI
    how = D.broadcast_models(models)
    return eng, sds, how


def _norm_kernel(name: str) -> str:
    return name.replace("(anonymous namespace)::", "").replace("void ", "").replace(" ", "")


def pmc_counters(kernel: str) -> dict:
    """Committed rocprofv3 PMC figures for `kernel` (scripts/pmc_top.py -> profiles/*pmc_top*.json, newest
    first; else the per-kernel FETCH / WRITE passes of scripts/pmc_traffic.py): HBM bytes per launch
    (FETCH_SIZE x2 + WRITE_SIZE per the gfx950 note), the HBM GB/s of that pass and the MFMA busy fraction
    (SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE / 8 x 1024 SIMDs).  Empty when no pass for it is committed."""
    want = _norm_kernel(kernel)
    for f in sorted(ROOT.glob("profiles/*pmc_top*.json"), reverse=True):
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        for k in d.get("kernels", []):
            if _norm_kernel(k["kernel"]) == want:
                return {"traffic": k["hbm_bytes_per_launch"], "hbm_gbps": k["hbm_gbps"],
                        "mfma_busy": k["mfma_busy"], "pmc_source": f.name}
    for f in sorted(ROOT.glob("profiles/*pmc_traffic*.json"), reverse=True):
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        if d.get("kernel") and kernel.endswith("::" + d["kernel"]):
            return {"traffic": round(d["bytes_per_launch"]), "pmc_source": f.name}
    return {}


def bucket(name: str) -> str:
    """Kernel family of a profiled launch: the step's time buckets."""
    n = _norm_kernel(name)
    if n.startswith("irx::gemm2_kernel<") or n.startswith("_ZN3irx12_GLOBAL__N_112gemm2_kernel"):
        args = n[n.index("<") + 1:].split(",") if "<" in n else []
        return "conv" if (len(args) > 7 and args[7] == "true") or "Lb1ELb0ELb0ELi" in n else "dense"
    if "gn_conv_narrow" in n:
        return "conv"
    if "gemm" in n or "splitk_reduce" in n:
        return "dense"
    if "attn" in n:
        return "attention"
    if n.startswith("irx::gn_") or n.startswith("irx::ln_") or "norm" in n:
        return "norm"
    return "other"


def bucket_summary(prof: list, steps: int) -> dict:
    """Per kernel family: ms/step, algorithmic TF/s, and HBM GB/s against the 8 TB/s peak over the launches whose
    HBM bytes a committed PMC pass holds (pmc_counters; `hbm_covered_ms` says how much of the bucket that is)."""
    out = {}
    for name, cnt, ms, fl in prof:
        b = out.setdefault(bucket(name), {"ms": 0.0, "fl": 0.0, "pmc_ms": 0.0, "bytes": 0.0})
        b["ms"] += ms
        b["fl"] += fl
        t = pmc_counters(name).get("traffic")
        if t:
            b["pmc_ms"] += ms
            b["bytes"] += float(t) * cnt
    res = {}
    for k, b in sorted(out.items(), key=lambda kv: -kv[1]["ms"]):
        gbps = b["bytes"] / (b["pmc_ms"] * 1e-3) / 1e9 if b["pmc_ms"] else None
        res[k] = {"ms_per_step": round(b["ms"] / steps, 2),
                  "tflops": round(b["fl"] / (b["ms"] * 1e-3) / 1e12, 1) if b["ms"] and b["fl"] else None,
                  "hbm_gbps": round(gbps, 1) if gbps else None,
                  "hbm_frac": round(gbps / 8000.0, 4) if gbps else None,
                  "hbm_covered_ms_per_step": round(b["pmc_ms"] / steps, 2)}
    return res


def usable_cpus() -> int:
    """CPUs this process may run on: sched affinity, capped by a cgroup CPU quota when one is set."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_and_parity(eng_bench, sds, device, n_images: int, threads: int) -> tuple:
    """configs[0] on the host cores through the fp32 CPU restatement, plus the same images
    through the GPU engines for the parity report."""
    from image_restoration_and_enhancement_amd import metrics as M
    from oracle import pipeline_ref as PR
    from image_restoration_and_enhancement_amd.tokenizer import PromptTokenizer
    from PIL import Image

    prompt, strength, steps, guidance = PR.TASKS["denoise"]
    cfg = PipelineConfig.default("denoise")               # saved scheduler: PNDM (configs[0])
    tok = PromptTokenizer()
    ids_p, ids_n = torch.from_numpy(tok(prompt))[None], torch.from_numpy(tok(""))[None]
    models = PR.Models(sds["unet"], cfg.unet, sds["vae"], cfg.vae, sds["clip"], cfg.clip)
    clean, noisy = synthetic_pairs(n_images, 512, seed=1000)
    torch.set_num_threads(threads)
    refs, t_img = [], []
    with torch.no_grad():
        for i in range(n_images):
            t0 = time.perf_counter()
            r = PR.img2img_ref(models, Image.fromarray(noisy[i]), ids_p, ids_n, strength, steps, guidance, 42, "pndm")
            t_img.append(time.perf_counter() - t0)
            refs.append(r)
            log(f"cpu_baseline: image {i + 1}/{n_images} in {t_img[-1]:.1f} s")   # (progress: one line per image)
    per_img = float(np.mean(t_img))
    cpu = {"value": round(1.0 / per_img, 6), "unit": "images/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
           "sample": f"BASELINE configs[0]: {n_images} full 512x512 denoise image(s), 20 PNDM steps x strength 0.5 "
                     f"= {len(refs[0].timesteps)} UNet evals with CFG 5.0 (batch 2), VAE encode + decode, fp32 "
                     f"PyTorch-CPU restatement (oracle/pipeline_ref.py), torch threads = usable CPUs of this "
                     f"process ({threads}); {per_img:.1f} s/image, model load excluded",
           "seconds_per_image": [round(t, 2) for t in t_img]}

    # the same images through the GPU engines: fp32, the bench engine, all-bf16, all-fp16 (the reference's GPU dtype)
    u8 = torch.from_numpy(noisy).to(device).contiguous()
    bench_key = "gpu_bf16_vae_fp16"

    def run(eng):
        kind = eng.cfg.scheduler.kind
        eng.cfg.scheduler.kind = "pndm"
        try:
            return eng.img2img(u8, prompt, strength, steps, guidance, seed=42, want_float=True)
        finally:
            eng.cfg.scheduler.kind = kind

    outs = {}
    for key, dt, vdt in (("gpu_fp32", "fp32", None), ("gpu_bf16", "bf16", "bf16"), ("gpu_fp16", "fp16", "fp16")):
        e = SDEngine(cfg, dt, device, state_dicts=sds, vae_dtype=vdt)
        outs[key] = run(e)
        del e
    outs[bench_key] = run(eng_bench)
    torch.cuda.synchronize()
    f32_max, u8_max, ps, ss = 0.0, 0, [], []
    keys = ("gpu_fp32", bench_key, "gpu_bf16", "gpu_fp16")
    gt = {k: ([], []) for k in keys + ("cpu_ref",)}   # (PSNR, SSIM) vs the clean image, per image
    for i, r in enumerate(refs):
        ref_u8 = np.asarray(r.image)
        f32_max = max(f32_max, float(np.abs(outs["gpu_fp32"].decoded01[i].cpu().numpy() - r.decoded_float).max()))
        imgs = {k: outs[k].images_u8[i].cpu().numpy() for k in keys}
        u8_max = max(u8_max, int(np.abs(imgs["gpu_fp32"].astype(int) - ref_u8.astype(int)).max()))
        ps.append(M.psnr(ref_u8, imgs[bench_key]))
        ss.append(M.ssim(ref_u8, imgs[bench_key]))
        for k, img in list(imgs.items()) + [("cpu_ref", ref_u8)]:
            gt[k][0].append(M.psnr(clean[i], img))
            gt[k][1].append(M.ssim(clean[i], img))
    mean_gt = {k: (float(np.mean(v[0])), float(np.mean(v[1]))) for k, v in gt.items()}

    def sf3(x: float) -> float:
        return float(f"{x:.3g}")
    # north star: "PSNR/SSIM reproduced to 3 s.f." — the task means (src/metrics.py:82-95 semantics: per-image PSNR /
    # SSIM against the clean image, averaged) of each GPU engine against the CPU reference's, both at 3 s.f.
    match = {k: sf3(mean_gt[k][0]) == sf3(mean_gt["cpu_ref"][0]) and sf3(mean_gt[k][1]) == sf3(mean_gt["cpu_ref"][1])
             for k in keys}
    per_img_d = {k: {"abs_d_psnr": [round(abs(a - b), 5) for a, b in zip(gt[k][0], gt["cpu_ref"][0])],
                     "abs_d_ssim": [round(abs(a - b), 7) for a, b in zip(gt[k][1], gt["cpu_ref"][1])]}
                 for k in keys}
    parity = {"workload": "BASELINE configs[0] images (512x512, 20 PNDM steps x 0.5, CFG 5.0, seed 42)",
              "images": n_images, "bench_engine": bench_key,
              "fp32_engine_max_abs_vs_ref": f32_max, "fp32_engine_u8_max_diff_vs_ref": u8_max,
              "psnr_vs_ref": round(float(np.mean(ps)), 3), "ssim_vs_ref": round(float(np.mean(ss)), 5),
              "psnr_vs_ref_per_image": [round(float(x), 3) for x in ps],
              "ssim_vs_ref_per_image": [round(float(x), 5) for x in ss],
              "psnr_gt": {k: round(v[0], 5) for k, v in mean_gt.items()},
              "ssim_gt": {k: round(v[1], 6) for k, v in mean_gt.items()},
              "per_image_vs_cpu_ref": per_img_d,
              "psnr_ssim_3sf": {k: [sf3(v[0]), sf3(v[1])] for k, v in mean_gt.items()},
              "psnr_ssim_3sf_match": match,
              "note": "psnr/ssim_vs_ref: the bench engine's output (bf16 UNet + CLIP, fp16 VAE) against the CPU fp32 "
                      "reference output (metrics.py = skimage 0.18.3 restatement); psnr_gt / ssim_gt: each output "
                      "against the clean image, mean over the images; per_image_vs_cpu_ref: per image |PSNR - "
                      "PSNR_ref| / |SSIM - SSIM_ref| (both against the clean image); psnr_ssim_3sf_match: an engine's "
                      "mean PSNR and SSIM equal the CPU reference's at 3 significant figures (a miss is reported as "
                      "false, not rounded away)"}
    return cpu, parity


def timed_steps(step, steps: int, warmup: int, device, sync=None) -> tuple:
    """The bench contract's timed region: `warmup` untimed steps, then exactly `steps` steps bracketed by a barrier and
    a device synchronisation on both sides; returns (last step's output, the MAX over ranks of the timed seconds)."""
    sync = sync or torch.cuda.synchronize
    out = None
    for _ in range(warmup):
        out = step()
    sync()
    D.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    sync()
    D.barrier()
    sync()
    return out, D.max_over_ranks(time.perf_counter() - t0, device)


def throughput(batch: int, world: int, steps: int, elapsed: float) -> tuple:
    """Whole-job images/s (every rank's `batch` images per step, weak scaling) and ms per step."""
    return batch * world * steps / elapsed, elapsed / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--task", default="denoise", choices=sorted(TASKS))
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (default: the config's shard)")
    ap.add_argument("--sched-steps", type=int, default=50)
    ap.add_argument("--dtype", default=None, help="bf16 | fp16 | fp32 (default: the config's)")
    ap.add_argument("--vae-dtype", default=None, help="VAE compute type (default: the task's, fp16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-images", type=int, default=4, help="configs[0] images for the CPU baseline (configs[0]: 4)")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--opt", action="append", default=[], help="irx_set_option name=value (A/B experiments)")
    args = ap.parse_args()
    spec = TASKS[args.task]
    batch = args.batch or spec["batch"]
    dtype = args.dtype or spec["dtype"]
    vae_dtype = args.vae_dtype or (spec["vae"] if dtype != "fp32" else "fp32")
    res = spec["res"]

    rank, world, local = D.init()
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    L.load()
    for o in args.opt:
        k, v = o.split("=")
        L.call("irx_set_option", k.encode(), int(v))

    cfg = PipelineConfig.default(args.task)
    cfg.scheduler.kind = "ddim"          # BASELINE.json: "50 DDIM steps" (explicit override of the saved PNDM)
    t_init = time.perf_counter()
    eng, sds, bcast = build_engine(cfg, dtype, device, rank, vae_dtype)
    u8_h, mask_h = task_inputs(args.task, spec, batch, seed=rank)
    imgs = torch.from_numpy(u8_h).to(device).contiguous()
    mask = torch.from_numpy(mask_h).to(device).contiguous() if mask_h is not None else None
    noise = draw_noise(42, res // 8, res // 8, 2)
    prompt = PROMPTS[args.task]
    log(f"[rank {rank}] engine ready in {time.perf_counter() - t_init:.1f}s ({args.task}, {dtype}, VAE {vae_dtype}, "
        f"batch {batch})")

    def step():
        eng._ctx_cache.clear()              # text encoding is part of every pass
        if args.task == "inpaint":
            return eng.inpaint(imgs, mask, prompt, spec["strength"], args.sched_steps, spec["guidance"], seed=42)
        return eng.img2img(imgs, prompt, spec["strength"], args.sched_steps, spec["guidance"], seed=42, noise=noise)

    out, el = timed_steps(step, args.steps, args.warmup, device)
    n_evals = len(out.timesteps)
    finite = bool(torch.isfinite(out.latents).all().item())
    value, ms_step = throughput(batch, world, args.steps, el)
    cfg_f = 2 if spec["guidance"] > 1 else 1
    tflop_img = (n_evals * cfg_f * F_UNET[res] + spec["n_enc"] * F_ENC[res] + F_DEC[res]) / 1000.0

    roofline = None
    if not args.no_roofline:
        torch.cuda.synchronize()
        graphs, eng.use_graphs = eng.use_graphs, False     # per-launch events need the eager launches
        L.profile_begin()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        prof = L.profile_end()
        eng.use_graphs = graphs
        tot_ms = sum(p[2] for p in prof if p[3] > 0)
        tot_fl = sum(p[3] for p in prof)
        prof.sort(key=lambda p: -p[2])
        if rank == 0:
            log(f"profiled {args.steps} steps: {tot_fl / 1e12 / (args.steps * batch):.2f} TFLOP/img counted, "
                f"MFMA-kernel time {tot_ms / args.steps:.1f} ms/step")
            for name, cnt, ms, fl in prof[:int(os.environ.get("IRX_PROF_TOP", "24"))]:
                log(f"  {ms / args.steps:8.1f} ms/step {cnt // args.steps:5d} launches/step "
                    f"{fl / ms / 1e9 if ms else 0:7.1f} TF/s  {name}")
        name, cnt, ms, fl = next(p for p in prof if p[3] > 0)   # dominant MFMA kernel
        peak = PEAK_TFLOPS[dtype]
        ach = fl / (ms * 1e-3) / 1e12
        pmc = pmc_counters(name)
        roofline = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                    "frac": round(ach / peak, 4), "traffic": pmc.get("traffic"),
                    "mfma_busy": pmc.get("mfma_busy"), "hbm_gbps": pmc.get("hbm_gbps"),
                    "hbm_peak_gbps": 8000.0, "pmc_source": pmc.get("pmc_source"), "kernel": name,
                    "launches": cnt, "avg_launch_us": round(ms * 1e3 / cnt, 2),
                    "flops_per_launch": fl / cnt,
                    "all_mfma_kernels_tflops": round(tot_fl / (tot_ms * 1e-3) / 1e12, 2),
                    "mfma_kernel_ms_per_step": round(tot_ms / args.steps, 2),
                    "buckets": bucket_summary(prof, args.steps)}

    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if args.task != "denoise":
            dn = PipelineConfig.default("denoise")
            sds = {k: W.random_state_dict(k, getattr(dn, k), 0) for k in ("unet", "vae", "clip")}
            eng = SDEngine(dn, "bf16", device, state_dicts=sds, vae_dtype="fp16")
        cpu, parity = cpu_baseline_and_parity(eng, sds, device, args.cpu_images, usable_cpus())

    if rank == 0:
        line = {
            "metric": "restored images/sec @512x512, 50 DDIM steps; PSNR/SSIM vs reference",
            "value": round(value, 4), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": dtype,
            "data": f"synthetic {res}x{res} {args.task} inputs, seeded random SD-1.5 weights",
            "config": {"workload": f"BASELINE configs[{spec['cfg'] - 1}] {args.task} {res}x{res}, batch {batch}/GPU, "
                                   f"{args.sched_steps} DDIM steps x strength {spec['strength']} = {n_evals} UNet "
                                   f"evals, " + (f"CFG {spec['guidance']} (UNet batch {batch * cfg_f})"
                                                 if cfg_f == 2 else "no CFG")
                                   + (", 9-channel UNet, 2 VAE encodes" if args.task == "inpaint" else ""),
                       "task": args.task, "global_batch": batch * world, "resolution": res,
                       "compute": f"UNet + CLIP {dtype}, VAE {vae_dtype} (fp32 accumulation)",
                       "parallelism": f"dp{world}", "weights_bcast": bcast,
                       "tflop_per_image": round(tflop_img, 2),
                       "achieved_tflops_end_to_end": round(value * tflop_img, 1), "outputs_finite": finite},
            "roofline": roofline, "cpu_baseline": cpu, "parity": parity,
        }
        print(json.dumps(line), flush=True)
    D.barrier()


if __name__ == "__main__":
    main()
