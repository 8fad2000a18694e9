"""Synthetic degradations on the GPU: the reference's `scripts/make_synthetic_pairs.py` helpers with the
same names, arguments and RNG draw order, operating on uint8 HWC device tensors (single images or
[B][H][W][C] batches) through `libirx.so` (csrc/degrade.hip).  Used to build large synthetic benchmark
batches without a host round trip per image.

Host-side randomness stays the reference's: `random.uniform / randint / choice` for the per-image
parameters and, with `exact_noise=True`, `np.random.randn` for the noise field (bit-identical pixels
to the numpy code).  With `exact_noise=False` the noise is drawn in-kernel (Philox4x32-10, seeded from
numpy's generator) and only its distribution matches.
"""
from __future__ import annotations

import ctypes as C
import random
from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import _lib as L


def _s():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _u8(img: torch.Tensor) -> torch.Tensor:
    if img.dtype != torch.uint8 or not img.is_cuda:
        raise ValueError("expected a uint8 CUDA tensor")
    return img.contiguous()


def add_gaussian_noise(img: torch.Tensor, sigma_range=(5, 8), exact_noise: bool = True) -> torch.Tensor:
    """make_synthetic_pairs.py:29-35."""
    img = _u8(img)
    sigma = random.uniform(*sigma_range)
    out = torch.empty_like(img)
    if exact_noise:
        z = torch.from_numpy(np.random.randn(*img.shape).astype(np.float32)).to(img.device)
        L.call("irx_degrade_noise", _s(), _p(img), img.numel(), sigma, _p(z), 0, _p(out))
    else:
        seed = int(np.random.randint(0, 2**63 - 1, dtype=np.int64))
        L.call("irx_degrade_noise", _s(), _p(img), img.numel(), sigma, None, seed, _p(out))
    return out


def gaussian_blur_down(img: torch.Tensor, ksizes: Sequence[int], scale: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """cv2.GaussianBlur(k, 0) per image, then cv2.resize(INTER_CUBIC) to (W//scale, H//scale)."""
    img = _u8(img)
    batched = img.dim() == 4
    x = img if batched else img[None]
    B, H, W, Cc = x.shape
    if len(ksizes) != B or any(k not in (1, 3, 5, 7) for k in ksizes):
        raise ValueError("one kernel size in {1, 3, 5, 7} per image")
    ks = torch.tensor(list(ksizes), dtype=torch.int32, device=img.device)
    blur = torch.empty_like(x)
    lr = torch.empty((B, H // scale, W // scale, Cc), dtype=torch.uint8, device=img.device)
    L.call("irx_degrade_blur_down", _s(), _p(x), B, H, W, Cc, _p(ks), scale, _p(blur), _p(lr))
    return (blur, lr) if batched else (blur[0], lr[0])


def degrade_sr(img: torch.Tensor, scale=4, use_jpeg: bool = False, use_motion_blur: bool = False) -> torch.Tensor:
    """make_synthetic_pairs.py:67-81, Gaussian branch (JPEG re-encoding and motion blur are host codecs /
    filters the GPU path does not cover)."""
    if use_jpeg or use_motion_blur:
        raise NotImplementedError("JPEG / motion-blur degradations are not on the GPU path")
    k = random.choice([3, 5, 7])
    return gaussian_blur_down(img, [k] * (img.shape[0] if img.dim() == 4 else 1), scale)[1]


def to_grayscale(img: torch.Tensor, mode: str = "lab", rgb: bool = False) -> torch.Tensor:
    """make_synthetic_pairs.py:84-90 (input channel order BGR as cv2.imread gives, or RGB with rgb=True)."""
    img = _u8(img)
    out = torch.empty(img.shape[:-1], dtype=torch.uint8, device=img.device)
    L.call("irx_degrade_gray", _s(), _p(img), img.numel() // 3, 1 if mode == "lab" else 0, int(rgb), _p(out))
    return out


def draw_free_form_strokes(h: int, w: int, num_strokes=(5, 15), thickness_range=(10, 40)):
    """The host half of random_free_form_mask (make_synthetic_pairs.py:104-114): the same `random` draws in
    the same order -> [(points, thickness)]."""
    strokes = []
    for _ in range(random.randint(*num_strokes)):
        pts = []
        for _ in range(random.randint(4, 8)):
            pts.append((random.randint(0, w - 1), random.randint(0, h - 1)))
        thickness = random.randint(*thickness_range)
        strokes.append((pts, thickness))
    return strokes


def rasterize_strokes(h: int, w: int, per_image: List[list], device, img: torch.Tensor = None):
    """Stroke lists (one per image) -> mask [B][h][w] (255 inside) and, with `img`, the masked input."""
    segs, thick, off = [], [], [0]
    for strokes in per_image:
        for pts, t in strokes:
            for (x0, y0), (x1, y1) in zip(pts[:-1], pts[1:]):
                segs.append((x0, y0, x1, y1))
                thick.append(t)
        off.append(len(segs))
    B = len(per_image)
    sg = torch.tensor(segs or [(0, 0, 0, 0)], dtype=torch.int32, device=device)
    th = torch.tensor(thick or [0], dtype=torch.int32, device=device)
    of = torch.tensor(off, dtype=torch.int32, device=device)
    mask = torch.empty((B, h, w), dtype=torch.uint8, device=device)
    masked = None
    if img is not None:
        img = _u8(img)
        masked = torch.empty_like(img)
    L.call("irx_degrade_strokes", _s(), B, h, w, _p(sg), _p(th), _p(of), _p(mask), _p(img), _p(masked))
    return mask, masked


def random_free_form_mask(h: int, w: int, num_strokes=(5, 15), thickness_range=(10, 40), device="cuda"):
    """make_synthetic_pairs.py:104-114 -> uint8 [h][w] device mask."""
    return rasterize_strokes(h, w, [draw_free_form_strokes(h, w, num_strokes, thickness_range)], device)[0][0]


def make_pairs(batch: torch.Tensor, sr_scale: int = 4, grayscale_mode: str = "lab",
               inpaint_easy_ratio: float = 0.7, rgb: bool = False) -> dict:
    """process_split's per-image degradations (make_synthetic_pairs.py:155-198) for a [B][H][W][3] batch in
    one set of launches: {task: input tensor} (+ "inpaint_mask").  Per-image parameters are drawn in the
    reference's order (denoise sigma + noise, sr kernel, inpaint mask) image by image."""
    batch = _u8(batch)
    B, H, W, _ = batch.shape
    sigmas, zs, ks, strokes = [], [], [], []
    for _ in range(B):
        sigmas.append(random.uniform(5, 8))
        zs.append(np.random.randn(H, W, 3).astype(np.float32))
        ks.append(random.choice([3, 5, 7]))
        if random.random() < inpaint_easy_ratio:
            strokes.append(draw_free_form_strokes(H, W, (3, 7), (5, 20)))
        else:
            strokes.append(draw_free_form_strokes(H, W, (8, 15), (20, 40)))
    noisy = torch.empty_like(batch)
    z = torch.from_numpy(np.stack(zs)).to(batch.device)
    n1 = H * W * 3
    for b in range(B):
        L.call("irx_degrade_noise", _s(), _p(batch[b]), n1, sigmas[b], _p(z[b]), 0, _p(noisy[b]))
    _, lr = gaussian_blur_down(batch, ks, sr_scale)
    gray = to_grayscale(batch, grayscale_mode, rgb)
    mask, masked = rasterize_strokes(H, W, strokes, batch.device, batch)
    return {"denoise": noisy, "sr": lr, "colorize": gray, "inpaint": masked, "inpaint_mask": mask}
