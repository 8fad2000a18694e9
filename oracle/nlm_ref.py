"""numpy restatement of OpenCV's fast non-local-means denoiser as the reference's classical denoise
fallback calls it (`src/inference.py:500-522`: cv2.fastNlMeansDenoisingColored(img, None, h, hColor, 7, 21)),
the checker for `csrc/nlmeans.hip`.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Parity: cv2 (opencv-python, the reference's unpinned `opencv-python` requirement) is absent from this image
and the reference holds no fixture of its output, so against cv2 itself this is **parity unpinned**.  It
follows OpenCV 4.x's published algorithm (modules/photo/src/denoising.cpp + fast_nlmeans_denoising_invoker*.hpp):

* Colored: convert to 8-bit Lab (COLOR_LBGR2Lab: the reference hands RGB bytes to a BGR API, so channel 0 is
  taken as blue), denoise L alone with `h` and the (a, b) pair with `hColor`, convert back.  The colour
  conversions live on the host side; `nl_means_u8` below is the part the GPU kernel replaces.
* Invoker (per channel group of `cn` channels, uint8, integer type int):
  - border: copyMakeBorder(BORDER_REFLECT_101) by search/2 + template/2;
  - dist(p, q) = sum over the template window of sum_c (I_c(p+t) - I_c(q+t))^2 (exact integer);
  - bin shift s = smallest s with 2^s >= template^2; almost = dist >> s;
  - weight LUT: w[a] = cvRound(fpm * exp(-a * 2^s / template^2 / (f32(h)*f32(h)*cn))), 0 below 0.001 * fpm,
    fpm = INT_MAX // (search^2 * 255);
  - out_c = (sum_q w * I_c(q) + W/2) // W, W = sum_q w (unsigned integer division), saturated to uint8.
"""
from __future__ import annotations

import numpy as np

INT_MAX = 2 ** 31 - 1


def bin_shift(template: int) -> int:
    s = 0
    while (1 << s) < template * template:
        s += 1
    return s


def weight_lut(h: float, cn: int, template: int = 7, search: int = 21) -> np.ndarray:
    """almost_dist2weight_ of FastNlMeansDenoisingInvoker's constructor (DistSquared::calcWeight)."""
    tws2 = template * template
    s = bin_shift(template)
    mult = float(1 << s) / tws2
    fpm = min(INT_MAX // (search * search * 255), INT_MAX)
    almost_max = int(255 * 255 * cn / mult + 1)
    hf = np.float32(h)
    den = float(np.float32(np.float32(hf * hf) * np.float32(cn)))     # h[0]*h[0]*channels in float
    dist = np.arange(almost_max, dtype=np.float64) * mult
    with np.errstate(divide="ignore", invalid="ignore"):
        w = np.exp(-dist / den)
    w = np.where(np.isnan(w), 1.0, w)
    wi = np.rint(fpm * w).astype(np.int64)
    wi[wi < 0.001 * fpm] = 0
    return wi


def _reflect101(i: np.ndarray, n: int) -> np.ndarray:
    if n == 1:
        return np.zeros_like(i)
    i = np.asarray(i).copy()
    while True:
        lo, hi = i < 0, i >= n
        if not (lo.any() or hi.any()):
            return i
        i = np.where(lo, -i, np.where(hi, 2 * (n - 1) - i, i))


def nl_means_u8(img: np.ndarray, h: float, template: int = 7, search: int = 21) -> np.ndarray:
    """fastNlMeansDenoising on a uint8 [H, W, cn] image (cn = 1 or 2, one h for the group)."""
    assert img.dtype == np.uint8 and img.ndim == 3
    H, W, cn = img.shape
    tr, sr = template // 2, search // 2
    b = tr + sr
    ys, xs = _reflect101(np.arange(-b, H + b), H), _reflect101(np.arange(-b, W + b), W)
    ext = img[ys][:, xs].astype(np.int64)                  # [H+2b, W+2b, cn]
    lut = weight_lut(h, cn, template, search)
    s = bin_shift(template)
    ctr = ext[sr:sr + H + 2 * tr, sr:sr + W + 2 * tr]       # template support of every output pixel
    est = np.zeros((H, W, cn), np.int64)
    wsum = np.zeros((H, W), np.int64)
    k = template
    for dy in range(-sr, sr + 1):
        for dx in range(-sr, sr + 1):
            sh = ext[sr + dy:sr + dy + H + 2 * tr, sr + dx:sr + dx + W + 2 * tr]
            d = ((ctr - sh) ** 2).sum(-1)                   # [H+2tr, W+2tr]
            c = np.pad(d.cumsum(0).cumsum(1), ((1, 0), (1, 0)))
            dist = c[k:, k:] - c[:-k, k:] - c[k:, :-k] + c[:-k, :-k]
            w = lut[dist >> s]
            wsum += w
            est += w[..., None] * ext[b + dy:b + dy + H, b + dx:b + dx + W]
    assert est.max(initial=0) <= INT_MAX                     # the int accumulator OpenCV uses
    out = (est + (wsum // 2)[..., None]) // wsum[..., None]
    return np.clip(out, 0, 255).astype(np.uint8)


def nl_means_u8_naive(img: np.ndarray, h: float, template: int = 7, search: int = 21) -> np.ndarray:
    """Per-pixel loop form of the same invoker (small images only) — pins the vectorised form above."""
    H, W, cn = img.shape
    tr, sr = template // 2, search // 2
    lut = weight_lut(h, cn, template, search)
    s = bin_shift(template)
    x = img.astype(np.int64)

    def px(y, xx):
        return x[_reflect101(np.array([y]), H)[0], _reflect101(np.array([xx]), W)[0]]

    out = np.zeros_like(img)
    for y in range(H):
        for xx in range(W):
            ws, est = 0, np.zeros(cn, np.int64)
            for dy in range(-sr, sr + 1):
                for dx in range(-sr, sr + 1):
                    dist = 0
                    for ty in range(-tr, tr + 1):
                        for tx in range(-tr, tr + 1):
                            dist += int(((px(y + ty, xx + tx) - px(y + dy + ty, xx + dx + tx)) ** 2).sum())
                    w = int(lut[dist >> s])
                    ws += w
                    est += w * px(y + dy, xx + dx)
            out[y, xx] = np.clip((est + ws // 2) // ws, 0, 255)
    return out
