"""Classical (non-diffusion) fallbacks of `RestorationPipeline` — numpy/scipy restatements of the OpenCV
calls the reference makes when no diffusion model is available.

cv2 is not installed on this image (neither here nor on the GPU box), so these are restatements of
OpenCV's documented algorithms; where OpenCV uses a private approximation the result may differ by a
few uint8 levels — parity unpinned (no oracle available), except where stated "exact":

* `denoise_opencv`   — src/inference.py:500-522: fastNlMeansDenoisingColored(h, hColor, 7, 21) (OpenCV's
                       integer NLM invoker, exact given the Lab bytes, on 8-bit LBGR-Lab: L with h, the a/b
                       pair with hColor; the GPU form is `nlmeans` / csrc/nlmeans.hip), then
                       bilateralFilter(9, 75, 75) if strength > 0.6 and medianBlur(5) if strength > 0.8.
* `sr_lanczos`       — src/inference.py:593-596: PIL LANCZOS resize (exact: same library call).
* `colorize_lab`     — src/inference.py:683-703: L of RGB->LAB, a = L*0.1-10, b = L*0.1-5 as int8
                       (negative values wrap through the uint8 cast exactly as the reference's
                       `astype(np.uint8)` does), LAB->RGB.
* `auto_mask`        — src/inference.py:805-840: RGB->GRAY (exact fixed-point), thresholds 30 / 225,
                       5x5 close then open (exact), keep when >= 1 % of pixels.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
from PIL import Image
from scipy.ndimage import grey_dilation, grey_erosion, median_filter

# ---------------------------------------------------------------------------------------- colour
_M_RGB2XYZ = np.array([[0.412453, 0.357580, 0.180423],
                       [0.212671, 0.715160, 0.072169],
                       [0.019334, 0.119193, 0.950227]])
_WHITE = np.array([0.950456, 1.0, 1.088754])
# np.linalg.inv(_M_RGB2XYZ), written out so the host and GPU forms share the exact doubles
_M_XYZ2RGB = [[3.240481343200526, -1.5371515162713185, -0.4985363261688878],
              [-0.9692549499965682, 1.8759900014898907, 0.04155592655829284],
              [0.05564663913517716, -0.20404133836651123, 1.0573110696453443]]


def rgb_to_gray_u8(rgb: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(RGB2GRAY) for uint8: (4899 R + 9617 G + 1868 B + 2^13) >> 14 (exact)."""
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    return ((r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14).astype(np.uint8)


def rgb_to_lab_u8(rgb: np.ndarray, srgb: bool = True) -> np.ndarray:
    """8-bit CIELAB as OpenCV stores it: L*255/100, a+128, b+128 (float64, rounded).
    srgb=False: the L-variants (COLOR_LRGB2Lab), no gamma linearisation.  Written as explicit elementwise
    operations in a fixed order (no matmul, whose BLAS summation order is unspecified) so that the GPU form
    (csrc/filters.hip lab_kernel, fp64 without contraction) computes the same bytes."""
    x = rgb.astype(np.float64) / 255.0
    if srgb:
        x = np.where(x > 0.04045, ((x + 0.055) / 1.055) ** 2.4, x / 12.92)
    r, g, b = x[..., 0], x[..., 1], x[..., 2]
    M = _M_RGB2XYZ
    xyz = [(M[i, 0] * r + M[i, 1] * g + M[i, 2] * b) / _WHITE[i] for i in range(3)]
    f = [np.where(t > 0.008856, np.cbrt(t), 7.787 * t + 16.0 / 116.0) for t in xyz]
    L = np.where(xyz[1] > 0.008856, 116.0 * f[1] - 16.0, 903.3 * xyz[1])
    a = 500.0 * (f[0] - f[1])
    bb = 200.0 * (f[1] - f[2])
    out = np.stack([L * 255.0 / 100.0, a + 128.0, bb + 128.0], -1)
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def lbgr_to_lab_u8(img: np.ndarray) -> np.ndarray:
    """cv2.COLOR_LBGR2Lab as fastNlMeansDenoisingColored applies it: channel 0 is taken as blue."""
    return rgb_to_lab_u8(img[..., ::-1], srgb=False)


def lab_u8_to_lbgr(lab: np.ndarray) -> np.ndarray:
    """cv2.COLOR_Lab2LBGR (the inverse of lbgr_to_lab_u8)."""
    return np.ascontiguousarray(lab_u8_to_rgb(lab, srgb=False)[..., ::-1])


def lab_u8_to_rgb(lab: np.ndarray, srgb: bool = True) -> np.ndarray:
    """Inverse of rgb_to_lab_u8 (explicit elementwise float64 operations, mirrored by lab_kernel)."""
    L = lab[..., 0].astype(np.float64) * 100.0 / 255.0
    a = lab[..., 1].astype(np.float64) - 128.0
    b = lab[..., 2].astype(np.float64) - 128.0
    fy = (L + 16.0) / 116.0
    fx, fz = fy + a / 500.0, fy - b / 200.0

    def finv(t):
        return np.where(t > 6.0 / 29.0, t * t * t, (t - 16.0 / 116.0) / 7.787)

    y = np.where(L > 903.3 * 0.008856, fy * fy * fy, L / 903.3)
    X, Y, Z = finv(fx) * _WHITE[0], y * _WHITE[1], finv(fz) * _WHITE[2]
    Mi = _M_XYZ2RGB
    rgb = np.stack([Mi[i][0] * X + Mi[i][1] * Y + Mi[i][2] * Z for i in range(3)], -1)
    rgb = np.clip(rgb, 0.0, 1.0)
    if srgb:
        rgb = np.where(rgb > 0.0031308, 1.055 * rgb ** (1 / 2.4) - 0.055, 12.92 * rgb)
    return np.clip(np.rint(rgb * 255.0), 0, 255).astype(np.uint8)


# ---------------------------------------------------------------------------------------- filters
def nlm_weights(h: float, cn: int, template: int = 7, search: int = 21) -> np.ndarray:
    """OpenCV FastNlMeansDenoisingInvoker's weight table: w[a] = cvRound(fpm * exp(-a * 2^s / template^2 /
    (f32(h)^2 * cn))), zero below 0.001 * fpm, fpm = INT_MAX // (search^2 * 255), 2^s >= template^2."""
    s = max(int(np.ceil(np.log2(template * template))), 0)
    mult = float(1 << s) / (template * template)
    fpm = (2 ** 31 - 1) // (search * search * 255)
    hf = np.float32(h)
    den = float(np.float32(np.float32(hf * hf) * np.float32(cn)))
    d = np.arange(int(255 * 255 * cn / mult + 1), dtype=np.float64) * mult
    with np.errstate(divide="ignore", invalid="ignore"):
        w = np.exp(-d / den)
    w = np.where(np.isnan(w), 1.0, w)
    wi = np.rint(fpm * w).astype(np.int64)
    wi[wi < 0.001 * fpm] = 0
    return wi


def nl_means_u8(img: np.ndarray, h: float, template: int = 7, search: int = 21) -> np.ndarray:
    """cv2.fastNlMeansDenoising's invoker on a uint8 [H, W, cn] channel group (exact integer arithmetic):
    patch SSD summed over the group, weight = table[SSD >> s], rounded integer weighted mean; reflect-101
    borders.  The CPU form of csrc/nlmeans.hip (used on hosts without a GPU)."""
    H, W, cn = img.shape
    tr, sr = template // 2, search // 2
    b = tr + sr
    ext = np.pad(img, ((b, b), (b, b), (0, 0)), mode="reflect").astype(np.int64)
    lut = nlm_weights(h, cn, template, search)
    s = max(int(np.ceil(np.log2(template * template))), 0)
    ctr = ext[sr:sr + H + 2 * tr, sr:sr + W + 2 * tr]
    est = np.zeros((H, W, cn), np.int64)
    wsum = np.zeros((H, W), np.int64)
    for dy in range(-sr, sr + 1):
        for dx in range(-sr, sr + 1):
            d = ((ctr - ext[sr + dy:sr + dy + H + 2 * tr, sr + dx:sr + dx + W + 2 * tr]) ** 2).sum(-1)
            dist = _box_sum_valid(d, template)
            w = lut[dist >> s]
            wsum += w
            est += w[..., None] * ext[b + dy:b + dy + H, b + dx:b + dx + W]
    return np.clip((est + (wsum // 2)[..., None]) // wsum[..., None], 0, 255).astype(np.uint8)


def _box_sum_valid(x: np.ndarray, k: int) -> np.ndarray:
    c = np.pad(x.cumsum(0).cumsum(1), ((1, 0), (1, 0)))
    return c[k:, k:] - c[:-k, k:] - c[k:, :-k] + c[:-k, :-k]


def fast_nl_means_denoising_colored(img: np.ndarray, h: float, h_color: float, template: int = 7,
                                    search: int = 21) -> np.ndarray:
    """cv2.fastNlMeansDenoisingColored (denoising.cpp): LBGR -> 8-bit Lab, L with h, (a, b) with hColor, back."""
    lab = lbgr_to_lab_u8(img)
    out = np.empty_like(lab)
    out[..., :1] = nl_means_u8(lab[..., :1], h, template, search)
    out[..., 1:] = nl_means_u8(lab[..., 1:], h_color, template, search)
    return lab_u8_to_lbgr(out)


def bilateral(img: np.ndarray, d: int = 9, sigma_color: float = 75.0, sigma_space: float = 75.0) -> np.ndarray:
    """cv2.bilateralFilter for uint8 images (BilateralFilter_8u): circular window of radius d//2 in row-major
    order, colour distance = sum of per-channel absolute differences, fp32 tables and sums (one rounding per
    operation, as csrc/filters.hip), cvRound(sum * (1 / wsum)), reflect-101 borders."""
    H, W, cn = img.shape
    sigma_color = 1.0 if sigma_color <= 0 else sigma_color
    sigma_space = 1.0 if sigma_space <= 0 else sigma_space
    r = max(d // 2 if d > 0 else int(np.rint(sigma_space * 1.5)), 1)
    i = np.arange(256 * cn, dtype=np.float64)
    cw = np.exp(i * i * (-0.5 / sigma_color ** 2)).astype(np.float32)
    pad = np.pad(img, ((r, r), (r, r), (0, 0)), mode="reflect").astype(np.int64)
    ctr = pad[r:r + H, r:r + W]
    acc = np.zeros((H, W, cn), np.float32)
    wsum = np.zeros((H, W), np.float32)
    for dy in range(-r, r + 1):
        for dx in range(-r, r + 1):
            rr = np.sqrt(float(dy * dy) + float(dx * dx))
            if rr > r:
                continue
            sw = np.float32(np.exp(rr * rr * (-0.5 / sigma_space ** 2)))
            sh = pad[r + dy:r + dy + H, r + dx:r + dx + W]
            w = sw * cw[np.abs(sh - ctr).sum(-1)]
            wsum = wsum + w
            acc = acc + sh.astype(np.float32) * w[..., None]
    return np.clip(np.rint(acc * (np.float32(1.0) / wsum)[..., None]), 0, 255).astype(np.uint8)


def median5(img: np.ndarray) -> np.ndarray:
    """cv2.medianBlur(img, 5): per-channel 5x5 median with replicated borders."""
    return median_filter(img, size=(5, 5, 1), mode="nearest")


# ---------------------------------------------------------------------------------------- tasks
def denoise_opencv(image: Image.Image, strength: float, nlm=None, bilateral_fn=None, median_fn=None) -> Image.Image:
    """src/inference.py:500-522.  `nlm` / `bilateral_fn` / `median_fn` = the fastNlMeansDenoisingColored,
    bilateralFilter(9, 75, 75) and medianBlur(5) implementations (the GPU ones from `nlmeans` on a ROCm device;
    this module's numpy forms otherwise)."""
    img = np.array(image.convert("RGB"))
    hs = float(np.clip(strength, 0.1, 1.0))
    h_value = hs * 10 if hs < 0.6 else 20          # luminance strength
    h_color = hs * 10 if hs < 0.6 else 20          # chroma strength (same rule in the reference)
    den = (nlm or fast_nl_means_denoising_colored)(img, h_value, h_color, 7, 21)
    if strength > 0.6:
        den = (bilateral_fn or bilateral)(den, 9, 75, 75)
    if strength > 0.8:
        den = (median_fn or median5)(den)
    return Image.fromarray(den)


def sr_lanczos(image: Image.Image, scale: int) -> Image.Image:
    w, h = image.size
    return image.resize((w * scale, h * scale), Image.LANCZOS)


def colorize_from_L(L: np.ndarray) -> np.ndarray:
    """src/inference.py:683-703 after the L channel: a = L*0.1-10, b = L*0.1-5 as int8 (negative values wrap
    through the uint8 cast exactly as the reference's `astype(np.uint8)` does), LAB -> RGB."""
    a = np.clip(L * 0.1 - 10, -127, 127).astype(np.int8)
    b = np.clip(L * 0.1 - 5, -127, 127).astype(np.int8)
    lab = np.stack([L, a, b], axis=-1)            # int8 promotes; the uint8 cast below wraps negatives
    return lab_u8_to_rgb(lab.astype(np.uint8))


def srgb_linear_lut() -> np.ndarray:
    """The sRGB linearisation of rgb_to_lab_u8 for the 256 byte values (same elementwise numpy operations)."""
    x = np.arange(256).astype(np.float64) / 255.0
    return np.where(x > 0.04045, ((x + 0.055) / 1.055) ** 2.4, x / 12.92)


def colorize_lab(image: Image.Image) -> Image.Image:
    img = np.array(image.convert("RGB"))
    return Image.fromarray(colorize_from_L(rgb_to_lab_u8(img)[..., 0]))


def auto_mask(image: Image.Image) -> Optional[Image.Image]:
    gray = rgb_to_gray_u8(np.array(image.convert("RGB")))
    m = np.where((gray <= 30) | (gray > 225), 255, 0).astype(np.uint8)
    fp = np.ones((5, 5), bool)
    m = grey_erosion(grey_dilation(m, footprint=fp, mode="constant", cval=0), footprint=fp, mode="constant",
                     cval=255)                                               # MORPH_CLOSE
    m = grey_dilation(grey_erosion(m, footprint=fp, mode="constant", cval=255), footprint=fp, mode="constant",
                      cval=0)                                                # MORPH_OPEN
    if np.sum(m > 0) / m.size < 0.01:
        return None
    return Image.fromarray(m).convert("L")
