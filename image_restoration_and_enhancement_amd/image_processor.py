"""Host-side image preparation — diffusers `VaeImageProcessor` semantics.

Only the PIL resize runs on the host (the reference does it with PIL too); the uint8 -> [-1, 1]
conversion and the uint8 post-processing run in `irx_image_to_tensor` / `irx_tensor_to_image`.
References: img2img preprocess = LANCZOS resize to (W - W%8, H - H%8); inpaint
image/mask processors resize to 512x512 (A.2); `RestorationPipeline._normalize_mask`
(`src/inference.py:778-803`).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
from PIL import Image


def target_size(img: Image.Image, height=None, width=None) -> Tuple[int, int]:
    h = height if height is not None else img.height - img.height % 8
    w = width if width is not None else img.width - img.width % 8
    return h, w


def to_uint8(img: Image.Image, height=None, width=None) -> np.ndarray:
    """PIL -> HWC uint8 (3 channels) at the processor's size (LANCZOS, like the reference)."""
    h, w = target_size(img, height, width)
    img = img.resize((w, h), resample=Image.LANCZOS)
    a = np.asarray(img)
    if a.ndim == 2:
        a = np.repeat(a[..., None], 3, axis=2)
    if a.shape[2] == 4:
        a = a[..., :3]
    return np.ascontiguousarray(a, dtype=np.uint8)


def mask_to_binary(mask: Image.Image, height: int, width: int) -> np.ndarray:
    """mask_processor.preprocess: L, LANCZOS resize, /255, binarize at 0.5 -> float32 HxW of {0,1}."""
    m = mask.convert("L").resize((width, height), resample=Image.LANCZOS)
    a = np.asarray(m).astype(np.float32) / 255.0
    return (a >= 0.5).astype(np.float32)


def nearest_downsample(mask: np.ndarray, h: int, w: int) -> np.ndarray:
    """torch.nn.functional.interpolate(mask, size=(h, w)) in 'nearest' mode."""
    H, W = mask.shape[-2:]
    sy, sx = np.float32(H / h), np.float32(W / w)
    iy = np.minimum((np.arange(h, dtype=np.float32) * sy).astype(np.int64), H - 1)
    ix = np.minimum((np.arange(w, dtype=np.float32) * sx).astype(np.int64), W - 1)
    return np.ascontiguousarray(mask[..., iy[:, None], ix[None, :]])


def normalize_mask(mask: Image.Image, size: Tuple[int, int]) -> Image.Image:
    """RestorationPipeline._normalize_mask: resize to the image size, invert if < 10 % is white."""
    if mask.size != size:
        mask = mask.resize(size, Image.LANCZOS)
    a = np.array(mask.convert("L"))
    if np.sum(a > 128) / a.size < 0.1:
        a = 255 - a
        mask = Image.fromarray(a).convert("L")
    return mask


def from_uint8(a: np.ndarray) -> Image.Image:
    return Image.fromarray(np.ascontiguousarray(a))
