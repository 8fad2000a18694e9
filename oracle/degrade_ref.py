"""numpy restatement of the pixel work of the reference's synthetic-pair generator
(`scripts/make_synthetic_pairs.py`), the checker for `csrc/degrade.hip`.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Parity: the reference calls OpenCV, which is absent from this image, so these restatements are
**parity unpinned** against cv2 itself.  They follow OpenCV's published 8-bit algorithms:
* `add_gaussian_noise`      — make_synthetic_pairs.py:29-35 (numpy only: exact given the same draws).
* `gaussian_blur_u8`        — cv2.GaussianBlur(k, sigmaX=0), k <= 7 (:75-76): the small-kernel binomial
                              table, fixed-point (weights * 256) rows then columns, round half up >> 16,
                              BORDER_REFLECT_101.
* `resize_cubic_down_u8`    — cv2.resize(INTER_CUBIC) to (w//s, h//s) (:78-79): A = -0.75, coefficients
                              * 2048 rounded, (sum + 2^21) >> 22 saturated, taps clamped.
* `gray_simple_u8`          — cv2.COLOR_BGR2GRAY (:90): (4899 R + 9617 G + 1868 B + 2^13) >> 14.
* `gray_lab_u8`             — L of cv2.COLOR_BGR2LAB (:86-88): sRGB linearisation, CIE L*, * 255/100
                              (float64 here; the GPU computes in fp32: within 1 level).
* `stroke_mask`             — random_free_form_mask (:104-114): cv2.line(thickness t) as a capsule of
                              radius t/2 around each segment (exact integer test).
"""
from __future__ import annotations

import numpy as np

GAUSS_SMALL = {1: [256], 3: [64, 128, 64], 5: [16, 64, 96, 64, 16], 7: [8, 28, 56, 72, 56, 28, 8]}


def add_gaussian_noise(img: np.ndarray, sigma: float, z: np.ndarray) -> np.ndarray:
    """make_synthetic_pairs.py:31-35 with the draws `z` (= np.random.randn(*img.shape)) given."""
    noise = z.astype(np.float32) * np.float32(sigma)
    return np.clip(img.astype(np.float32) + noise, 0, 255).astype(np.uint8)


def _reflect101(i: np.ndarray, n: int) -> np.ndarray:
    if n == 1:
        return np.zeros_like(i)
    i = np.abs(i)
    period = 2 * n - 2
    i = i % period
    return np.where(i >= n, period - i, i)


def gaussian_blur_u8(img: np.ndarray, k: int) -> np.ndarray:
    """img uint8 [H][W][C] -> uint8, exact integer arithmetic (cv2 8U fixed-point path)."""
    w = np.asarray(GAUSS_SMALL[k], dtype=np.int64)
    r = k // 2
    H, W = img.shape[:2]
    x = img.astype(np.int64)
    cols = _reflect101(np.arange(-r, W + r), W)
    rows = _reflect101(np.arange(-r, H + r), H)
    xp = x[:, cols]
    h = sum(w[j] * xp[:, j:j + W] for j in range(k))
    hp = h[rows]
    acc = sum(w[j] * hp[j:j + H] for j in range(k))
    return np.minimum((acc + 32768) >> 16, 255).astype(np.uint8)


def _cubic_coeffs(t: np.ndarray) -> np.ndarray:
    A = np.float32(-0.75)
    t = t.astype(np.float32)
    one = np.float32(1)
    c0 = ((A * (t + one) - 5 * A) * (t + one) + 8 * A) * (t + one) - 4 * A
    c1 = ((A + 2) * t - (A + 3)) * t * t + one
    c2 = ((A + 2) * (one - t) - (A + 3)) * (one - t) * (one - t) + one
    c3 = one - c0 - c1 - c2
    return np.rint(np.stack([c0, c1, c2, c3], -1) * np.float32(2048)).astype(np.int64)


def resize_cubic_down_u8(img: np.ndarray, scale: int) -> np.ndarray:
    H, W = img.shape[:2]
    Ho, Wo = H // scale, W // scale
    fx = (np.arange(Wo, dtype=np.float32) + np.float32(0.5)) * np.float32(W / Wo) - np.float32(0.5)
    fy = (np.arange(Ho, dtype=np.float32) + np.float32(0.5)) * np.float32(H / Ho) - np.float32(0.5)
    sx, sy = np.floor(fx).astype(np.int64), np.floor(fy).astype(np.int64)
    wx, wy = _cubic_coeffs(fx - sx), _cubic_coeffs(fy - sy)
    x = img.astype(np.int64)
    h = sum(wx[:, k][None, :, None] * x[:, np.clip(sx - 1 + k, 0, W - 1)] for k in range(4))
    acc = sum(wy[:, k][:, None, None] * h[np.clip(sy - 1 + k, 0, H - 1)] for k in range(4))
    return np.clip((acc + (1 << 21)) >> 22, 0, 255).astype(np.uint8)


def gray_simple_u8(img: np.ndarray, rgb: bool = False) -> np.ndarray:
    x = img.astype(np.int64)
    R, G, B = (x[..., 0], x[..., 1], x[..., 2]) if rgb else (x[..., 2], x[..., 1], x[..., 0])
    return ((R * 4899 + G * 9617 + B * 1868 + (1 << 13)) >> 14).astype(np.uint8)


def gray_lab_u8(img: np.ndarray, rgb: bool = False) -> np.ndarray:
    x = img.astype(np.float64) / 255.0
    lin = np.where(x <= 0.04045, x / 12.92, ((x + 0.055) / 1.055) ** 2.4)
    R, G, B = (lin[..., 0], lin[..., 1], lin[..., 2]) if rgb else (lin[..., 2], lin[..., 1], lin[..., 0])
    Y = 0.212671 * R + 0.715160 * G + 0.072169 * B
    L = np.where(Y > 0.008856, 116.0 * np.cbrt(Y) - 16.0, 903.3 * Y)
    return np.clip(np.rint(L * 2.55), 0, 255).astype(np.uint8)


def stroke_mask(h: int, w: int, strokes) -> np.ndarray:
    """strokes: list of (points [(x, y) ...], thickness) -> uint8 mask (255 inside)."""
    yy, xx = np.mgrid[0:h, 0:w].astype(np.int64)
    on = np.zeros((h, w), bool)
    for pts, t in strokes:
        for (x0, y0), (x1, y1) in zip(pts[:-1], pts[1:]):
            dx, dy = x1 - x0, y1 - y0
            vx, vy = xx - x0, yy - y0
            L2 = dx * dx + dy * dy
            dot = vx * dx + vy * dy
            d_start = 4 * (vx * vx + vy * vy) <= t * t
            d_end = 4 * ((xx - x1) ** 2 + (yy - y1) ** 2) <= t * t
            d_mid = 4 * ((vx * vx + vy * vy) * L2 - dot * dot) <= t * t * L2
            on |= np.where((L2 == 0) | (dot <= 0), d_start, np.where(dot >= L2, d_end, d_mid))
    return np.where(on, 255, 0).astype(np.uint8)
