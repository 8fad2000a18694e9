"""Evaluation metrics — numpy/scipy/PIL restatement of the reference's `src/metrics.py`.

The reference imports cv2, scikit-image and torchvision (`src/metrics.py:11-22`) and exits when any
is missing; none of them is installed on the GPU image, so `scripts/evaluate_model.py --no-lpips
--no-fid` could not run there.  This module keeps the same surface (`load_image`,
`MetricsCalculator.calculate_{psnr,ssim,delta_e,all}`, `evaluate_task`, `print_results`) with the
arithmetic restated:

* PSNR  = skimage `peak_signal_noise_ratio(gt, pred, data_range=255)` (`src/metrics.py:82-87`)
* SSIM  = skimage `structural_similarity(gt, pred, data_range=255, channel_axis=2)` defaults:
  7x7 uniform window (scipy `uniform_filter`, reflect borders), sample covariance (NP/(NP-1)),
  K1 = 0.01, K2 = 0.03, mean over the map cropped by 3 px, mean over channels (`:89-95`)
* dE76  = mean Euclidean distance of skimage `rgb2lab` (D65, 2 deg) of pred/255 and gt/255 (`:115-148`)
* shape mismatch: pred resized to gt with cv2 `INTER_LINEAR` semantics (half-pixel centres,
  11-bit fixed-point weights, round-to-nearest) (`:84-85`)
* `load_image`: `cv2.imread` + BGR->RGB == PIL decode to RGB (`:40-46`)

PSNR / SSIM / rgb2lab are pinned against scikit-image 0.18.3 outputs committed under
`tests/golden/metrics.json` (tests/test_metrics.py).  The INTER_LINEAR resize and JPEG decode are
restatements without an oracle in this image (cv2 is absent): parity unpinned.  LPIPS and FID need
network-downloaded networks and stay unavailable, exactly as the reference behaves without
`lpips`/torchvision (`src/metrics.py:24-37`).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
from PIL import Image
from scipy.ndimage import uniform_filter

LPIPS_AVAILABLE = False
FID_AVAILABLE = False

# skimage.color: sRGB (D65) -> XYZ and the D65 / 2-degree white point
_XYZ_FROM_RGB = np.array([[0.412453, 0.357580, 0.180423],
                          [0.212671, 0.715160, 0.072169],
                          [0.019334, 0.119193, 0.950227]])
_WHITE_D65 = np.array([0.95047, 1.0, 1.08883])


def load_image(path: Path) -> np.ndarray:
    """Load image as RGB uint8 HWC (reference `src/metrics.py:40-46`)."""
    try:
        with Image.open(str(path)) as im:
            return np.array(im.convert("RGB"))
    except (OSError, ValueError):
        raise ValueError(f"Could not load image: {path}")


def resize_linear(img: np.ndarray, width: int, height: int) -> np.ndarray:
    """cv2.resize(img, (width, height)) with INTER_LINEAR for uint8 images."""
    H, W = img.shape[:2]
    if (H, W) == (height, width):
        return img.copy()

    def axis(n_out, n_in):
        scale = n_in / n_out
        f = (np.arange(n_out) + 0.5) * scale - 0.5
        i0 = np.floor(f).astype(np.int64)
        f = f - i0
        lo = i0 < 0
        f[lo], i0[lo] = 0.0, 0
        hi = i0 >= n_in - 1
        f[hi], i0[hi] = 0.0, n_in - 1
        w1 = np.rint(f * 2048).astype(np.int64)
        return i0, np.minimum(i0 + 1, n_in - 1), 2048 - w1, w1

    y0, y1, wy0, wy1 = axis(height, H)
    x0, x1, wx0, wx1 = axis(width, W)
    a = img.astype(np.int64)
    if a.ndim == 2:
        a = a[..., None]
    rows = a[:, x0] * wx0[None, :, None] + a[:, x1] * wx1[None, :, None]        # [H, width, C]
    out = rows[y0] * wy0[:, None, None] + rows[y1] * wy1[:, None, None]
    out = (out + (1 << 21)) >> 22
    out = np.clip(out, 0, 255).astype(np.uint8)
    return out[..., 0] if img.ndim == 2 else out


def psnr(gt: np.ndarray, pred: np.ndarray, data_range: float = 255.0) -> float:
    err = np.mean((gt.astype(np.float64) - pred.astype(np.float64)) ** 2)
    with np.errstate(divide="ignore"):
        return float(10 * np.log10((data_range ** 2) / err))


def _ssim_2d(X: np.ndarray, Y: np.ndarray, data_range: float, win: int = 7, K1: float = 0.01,
             K2: float = 0.03) -> float:
    X = X.astype(np.float64)
    Y = Y.astype(np.float64)
    NP = win * win
    cov_norm = NP / (NP - 1)
    ux = uniform_filter(X, size=win)
    uy = uniform_filter(Y, size=win)
    uxx = uniform_filter(X * X, size=win)
    uyy = uniform_filter(Y * Y, size=win)
    uxy = uniform_filter(X * Y, size=win)
    vx = cov_norm * (uxx - ux * ux)
    vy = cov_norm * (uyy - uy * uy)
    vxy = cov_norm * (uxy - ux * uy)
    C1 = (K1 * data_range) ** 2
    C2 = (K2 * data_range) ** 2
    A1, A2 = 2 * ux * uy + C1, 2 * vxy + C2
    B1, B2 = ux ** 2 + uy ** 2 + C1, vx + vy + C2
    S = (A1 * A2) / (B1 * B2)
    pad = (win - 1) // 2
    return float(S[pad:S.shape[0] - pad, pad:S.shape[1] - pad].mean())


def ssim(gt: np.ndarray, pred: np.ndarray, data_range: float = 255.0) -> float:
    if gt.shape != pred.shape:
        raise ValueError("Input images must have the same dimensions.")
    if gt.ndim == 2:
        return _ssim_2d(gt, pred, data_range)
    return float(np.mean([_ssim_2d(gt[..., c], pred[..., c], data_range) for c in range(gt.shape[2])]))


def rgb2lab(rgb: np.ndarray) -> np.ndarray:
    """skimage.color.rgb2lab for float RGB in [0, 1] (D65, 2-degree observer)."""
    arr = np.array(rgb, copy=True)
    mask = arr > 0.04045
    arr[mask] = np.power((arr[mask] + 0.055) / 1.055, 2.4)
    arr[~mask] /= 12.92
    xyz = arr @ _XYZ_FROM_RGB.T
    xyz = xyz / _WHITE_D65
    mask = xyz > 0.008856
    xyz[mask] = np.cbrt(xyz[mask])
    xyz[~mask] = 7.787 * xyz[~mask] + 16.0 / 116.0
    x, y, z = xyz[..., 0], xyz[..., 1], xyz[..., 2]
    return np.stack([116.0 * y - 16.0, 500.0 * (x - y), 200.0 * (y - z)], axis=-1)


class MetricsCalculator:
    """Per-image metrics (reference `src/metrics.py:57-209`).  LPIPS/FID: unavailable offline."""

    def __init__(self, use_lpips: bool = True, use_fid: bool = True, device: str = "cpu"):
        self.use_lpips = use_lpips and LPIPS_AVAILABLE
        self.use_fid = use_fid and FID_AVAILABLE
        self.device = device

    @staticmethod
    def _match(pred: np.ndarray, gt: np.ndarray) -> np.ndarray:
        return pred if pred.shape == gt.shape else resize_linear(pred, gt.shape[1], gt.shape[0])

    def calculate_psnr(self, pred: np.ndarray, gt: np.ndarray) -> float:
        return psnr(gt, self._match(pred, gt), data_range=255.0)

    def calculate_ssim(self, pred: np.ndarray, gt: np.ndarray) -> float:
        return ssim(gt, self._match(pred, gt), data_range=255.0)

    def calculate_lpips(self, pred: np.ndarray, gt: np.ndarray):
        return None

    def calculate_delta_e(self, pred: np.ndarray, gt: np.ndarray, use_delta_e2000: bool = False) -> float:
        pred = self._match(pred, gt)
        pl = rgb2lab(pred.astype(np.float32) / 255.0)
        gl = rgb2lab(gt.astype(np.float32) / 255.0)
        return float(np.mean(np.sqrt(np.sum((pl - gl) ** 2, axis=2))))

    def calculate_fid(self, pred_images, gt_images):
        return None

    def calculate_all(self, pred: np.ndarray, gt: np.ndarray) -> dict:
        out = {"psnr": self.calculate_psnr(pred, gt), "ssim": self.calculate_ssim(pred, gt)}
        if self.use_lpips:
            out["lpips"] = self.calculate_lpips(pred, gt)
        return out


_EXTS = {".jpg", ".jpeg", ".png"}


def evaluate_task(pred_dir: Path, gt_dir: Path, task_name: str = "denoise", use_lpips: bool = True,
                  use_fid: bool = True, device: str = "cpu") -> dict:
    """Match predictions to ground truth by file name (any of .jpg/.jpeg/.png) and aggregate
    mean/std/min/max/median per metric (reference `src/metrics.py:238-348`)."""
    pred_dir, gt_dir = Path(pred_dir), Path(gt_dir)
    calc = MetricsCalculator(use_lpips=use_lpips, use_fid=use_fid, device=device)
    pred_files = sorted(f for f in pred_dir.iterdir() if f.suffix.lower() in _EXTS)
    gt_names = {f.name for f in gt_dir.iterdir() if f.suffix.lower() in _EXTS}
    if len(pred_files) != len(gt_names):
        print(f"Warning: Mismatch - {len(pred_files)} predictions vs {len(gt_names)} ground truth")
    pairs = []
    for pf in pred_files:
        gf = gt_dir / pf.name
        if not gf.exists():
            for ext in (".jpg", ".jpeg", ".png"):
                alt = gt_dir / (pf.stem + ext)
                if alt.exists():
                    gf = alt
                    break
        if gf.exists():
            pairs.append((pf, gf))
    if not pairs:
        raise ValueError(f"No matching files found between {pred_dir} and {gt_dir}")
    all_metrics = {"psnr": [], "ssim": []}
    if use_lpips:
        all_metrics["lpips"] = []
    print(f"Evaluating {task_name}: {len(pairs)} image pairs...")
    for i, (pp, gp) in enumerate(pairs):
        try:
            for k, v in calc.calculate_all(load_image(pp), load_image(gp)).items():
                if v is not None:
                    all_metrics[k].append(v)
            if (i + 1) % 10 == 0:
                print(f"  Processed {i + 1}/{len(pairs)}")
        except Exception as e:  # the reference skips unreadable pairs
            print(f"Error processing {pp.name}: {e}")
    res = {"task": task_name, "num_samples": len(pairs), "metrics": {}}
    for k, vals in all_metrics.items():
        if vals:
            res["metrics"][k] = {"mean": np.mean(vals), "std": np.std(vals), "min": np.min(vals),
                                 "max": np.max(vals), "median": np.median(vals)}
    return res


def print_results(results: dict):
    print(f"\n{'=' * 60}")
    print(f"Evaluation Results: {results['task']}")
    print(f"{'=' * 60}")
    print(f"Number of samples: {results['num_samples']}")
    print("\nMetrics:")
    for name, st in results["metrics"].items():
        print(f"\n  {name.upper()}:")
        print(f"    Mean:   {st['mean']:.4f} ± {st['std']:.4f}")
        print(f"    Median: {st['median']:.4f}")
        print(f"    Range:  [{st['min']:.4f}, {st['max']:.4f}]")
    print(f"\n{'=' * 60}\n")
