"""numpy restatement of the two filters after the NLM pass in the reference's classical denoise fallback
(`src/inference.py:517-520`: cv2.bilateralFilter(denoised, 9, 75, 75) if strength > 0.6, cv2.medianBlur(., 5) if
strength > 0.8), the checker for `csrc/filters.hip`.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Parity: cv2 is absent from this image and the reference holds no fixture of these filters' output, so against
cv2 itself this is **parity unpinned**.  It follows OpenCV 4.x's published 8-bit algorithms
(modules/imgproc/src/bilateral_filter.dispatch.cpp / .simd.hpp, median_blur.simd.hpp):
* bilateral: sigma <= 0 -> 1, radius = d // 2; color_w[i] = f32(exp(-i^2 / (2 sc^2))) for i < 256*cn; the circular
  window in row-major order (sqrt(i^2 + j^2) <= radius) with space_w = f32(exp(-r^2 / (2 ss^2))); per pixel
  w = space_w * color_w[|db| + |dg| + |dr|], fp32 sums in window order (one rounding per operation), result
  cvRound(sum * (1 / wsum)); BORDER_REFLECT_101.  (OpenCV's SIMD path may fuse multiply-adds; this restatement
  fixes one rounding per operation, as the kernel does.)
* medianBlur(5): per-channel median of the 5x5 window, BORDER_REPLICATE (exact).
"""
from __future__ import annotations

import numpy as np


def bilateral_tables(d: int, sigma_color: float, sigma_space: float, cn: int = 3):
    sigma_color = 1.0 if sigma_color <= 0 else sigma_color
    sigma_space = 1.0 if sigma_space <= 0 else sigma_space
    gc, gs = -0.5 / (sigma_color * sigma_color), -0.5 / (sigma_space * sigma_space)
    radius = max(int(np.rint(sigma_space * 1.5)) if d <= 0 else d // 2, 1)
    i = np.arange(256 * cn, dtype=np.float64)
    color_w = np.exp(i * i * gc).astype(np.float32)
    sw, dydx = [], []
    for y in range(-radius, radius + 1):
        for x in range(-radius, radius + 1):
            r = np.sqrt(float(y * y) + float(x * x))
            if r > radius:
                continue
            sw.append(np.float32(np.exp(r * r * gs)))
            dydx.append((y, x))
    return color_w, np.array(sw, np.float32), np.array(dydx, np.int32), radius


def bilateral_u8(img: np.ndarray, d: int = 9, sigma_color: float = 75.0, sigma_space: float = 75.0) -> np.ndarray:
    H, W, cn = img.shape
    cw, sw, dydx, r = bilateral_tables(d, sigma_color, sigma_space, cn)
    pad = np.pad(img, ((r, r), (r, r), (0, 0)), mode="reflect").astype(np.int64)
    ctr = pad[r:r + H, r:r + W]
    wsum = np.zeros((H, W), np.float32)
    acc = np.zeros((H, W, cn), np.float32)
    for k, (dy, dx) in enumerate(dydx):
        sh = pad[r + dy:r + dy + H, r + dx:r + dx + W]
        w = sw[k] * cw[np.abs(sh - ctr).sum(-1)]                  # float32 * float32
        wsum = wsum + w
        acc = acc + sh.astype(np.float32) * w[..., None]
    out = np.rint(acc * (np.float32(1.0) / wsum)[..., None])
    return np.clip(out, 0, 255).astype(np.uint8)


def median5_u8(img: np.ndarray) -> np.ndarray:
    H, W = img.shape[:2]
    pad = np.pad(img, ((2, 2), (2, 2), (0, 0)), mode="edge")
    win = np.stack([pad[i:i + H, j:j + W] for i in range(5) for j in range(5)], 0)
    return np.sort(win, axis=0)[12].astype(np.uint8)


def _morph5(m: np.ndarray, op: str) -> np.ndarray:
    """5x5 square dilation ('max', border 0) or erosion ('min', border 255) — OpenCV's default border value."""
    H, W = m.shape
    fill = 0 if op == "max" else 255
    pad = np.full((H + 4, W + 4), fill, np.uint8)
    pad[2:-2, 2:-2] = m
    win = np.stack([pad[i:i + H, j:j + W] for i in range(5) for j in range(5)], 0)
    return win.max(0) if op == "max" else win.min(0)


def auto_mask_u8(rgb: np.ndarray):
    """_auto_mask_from_image (src/inference.py:805-840): RGB2GRAY fixed point, THRESH_BINARY_INV at 30 |
    THRESH_BINARY at 225, MORPH_CLOSE then MORPH_OPEN (5x5 ones); returns (mask, keep = share >= 1 %)."""
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    gray = (r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14
    m = np.where((gray <= 30) | (gray > 225), 255, 0).astype(np.uint8)
    m = _morph5(_morph5(m, "max"), "min")
    m = _morph5(_morph5(m, "min"), "max")
    return m, np.sum(m > 0) / m.size >= 0.01
