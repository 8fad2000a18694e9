"""The reference's classical denoise fallback (`src/inference.py:500-522`) on the GPU: cv2.fastNlMeansDenoising /
fastNlMeansDenoisingColored (templateWindowSize 7, searchWindowSize 21; csrc/nlmeans.hip, C ABI `irx_nlm_weights`
/ `irx_nlmeans_u8`), cv2.bilateralFilter(9, 75, 75) and cv2.medianBlur(5) (csrc/filters.hip,
`irx_bilateral_tables` / `irx_bilateral_u8` / `irx_median_blur_u8`), and `denoise_opencv` composing them.

The invoker (integer patch distances, the weight table, the rounded integer average) is OpenCV's and exact
against `oracle/nlm_ref.py`.  The colour conversion of the Colored variant (COLOR_LBGR2Lab and back, 8-bit
Lab; the reference passes RGB bytes where cv2 expects BGR) is `classical`'s fp64 restatement, run on the GPU
(`irx_lab_convert_u8`) with the same bytes.  cv2 is absent from this image, so parity against cv2 itself is
unpinned.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Tuple

import numpy as np
import torch

from . import _lib as L

_LUT_CACHE: Dict[Tuple[float, int, int, int, str], torch.Tensor] = {}


def nlm_weights(h: float, cn: int, template: int = 7, search: int = 21) -> np.ndarray:
    """The invoker's weight table (almost_dist2weight), truncated at its first zero (host computation)."""
    n = C.c_int()
    L.call("irx_nlm_weights", float(h), cn, template, search, None, 0, C.byref(n))
    buf = (C.c_int * max(n.value, 1))()
    L.call("irx_nlm_weights", float(h), cn, template, search, buf, n.value, C.byref(n))
    return np.frombuffer(buf, dtype=np.int32, count=n.value).copy()


def _lut(h: float, cn: int, template: int, search: int, device) -> torch.Tensor:
    key = (float(np.float32(h)), cn, template, search, str(device))
    t = _LUT_CACHE.get(key)
    if t is None:
        t = torch.from_numpy(nlm_weights(h, cn, template, search)).to(device)
        _LUT_CACHE[key] = t
    return t


def _check(img: torch.Tensor) -> torch.Tensor:
    if img.dtype != torch.uint8 or not img.is_cuda:
        raise ValueError("expected a uint8 CUDA tensor [H, W, C] or [B, H, W, C]")
    return img.contiguous()


def denoise_group(src: torch.Tensor, dst: torch.Tensor, h: float, ch_off: int, cn: int, template: int = 7,
                  search: int = 21) -> None:
    """Denoise channels [ch_off, ch_off + cn) of `src` into the same channels of `dst` ([B, H, W, C] uint8)."""
    B, H, W, Cc = src.shape
    lut = _lut(h, cn, template, search, src.device)
    L.call("irx_nlmeans_u8", C.c_void_p(torch.cuda.current_stream().cuda_stream), C.c_void_p(src.data_ptr()),
           C.c_void_p(dst.data_ptr()), B, H, W, Cc, ch_off, cn, template, search, C.c_void_p(lut.data_ptr()),
           int(lut.numel()))


def fast_nl_means_denoising(src: torch.Tensor, h: float = 3.0, template_window_size: int = 7,
                            search_window_size: int = 21) -> torch.Tensor:
    """cv2.fastNlMeansDenoising on uint8 images with 1 or 2 channels (one h for the channel group)."""
    x = _check(src)
    single = x.dim() == 3
    if single:
        x = x.unsqueeze(0)
    if x.shape[-1] not in (1, 2):
        raise ValueError("fastNlMeansDenoising: 1 or 2 channels (colour images: fast_nl_means_denoising_colored)")
    out = torch.empty_like(x)
    denoise_group(x, out, h, 0, x.shape[-1], template_window_size, search_window_size)
    return out[0] if single else out


def fast_nl_means_denoising_lab(lab: torch.Tensor, h: float, h_color: float, template_window_size: int = 7,
                                search_window_size: int = 21) -> torch.Tensor:
    """The invoker half of cv2.fastNlMeansDenoisingColored on 8-bit Lab images [B, H, W, 3]: L with `h`, the
    (a, b) pair with `h_color` (denoising.cpp: mixChannels into l / ab, two fastNlMeansDenoising calls)."""
    x = _check(lab)
    if x.dim() != 4 or x.shape[-1] != 3:
        raise ValueError("expected Lab images [B, H, W, 3]")
    out = torch.empty_like(x)
    denoise_group(x, out, h, 0, 1, template_window_size, search_window_size)
    denoise_group(x, out, h_color, 1, 2, template_window_size, search_window_size)
    return out


def lab_convert(src: torch.Tensor, direction: int) -> torch.Tensor:
    """COLOR_LBGR2Lab (direction 0) / COLOR_Lab2LBGR (1) on uint8 [..., 3] CUDA tensors (fp64, exact vs classical)."""
    x = _check(src)
    if x.shape[-1] != 3:
        raise ValueError("expected 3-channel pixels")
    out = torch.empty_like(x)
    L.call("irx_lab_convert_u8", C.c_void_p(torch.cuda.current_stream().cuda_stream), C.c_void_p(x.data_ptr()),
           C.c_void_p(out.data_ptr()), x.numel() // 3, direction)
    return out


def fast_nl_means_denoising_colored(img, h: float = 3.0, h_color: float = 3.0, template_window_size: int = 7,
                                    search_window_size: int = 21, device: str = "cuda"):
    """cv2.fastNlMeansDenoisingColored(img, None, h, hColor, 7, 21) for uint8 [H, W, 3] or [B, H, W, 3] images:
    LBGR -> Lab, L with h, (a, b) with hColor, Lab -> LBGR, all on the GPU.  A CUDA tensor stays on the device;
    a numpy array is uploaded once and returned as numpy."""
    is_np = not isinstance(img, torch.Tensor)
    x = torch.from_numpy(np.ascontiguousarray(img, dtype=np.uint8)).to(device) if is_np else _check(img)
    single = x.dim() == 3
    if single:
        x = x.unsqueeze(0)
    lab = lab_convert(x, 0)
    den = fast_nl_means_denoising_lab(lab, h, h_color, template_window_size, search_window_size)
    out = lab_convert(den, 1)
    out = out[0] if single else out
    return out.cpu().numpy() if is_np else out


_BIL_CACHE: Dict[Tuple[int, float, float, str], tuple] = {}


def _bilateral_tables(d: int, sigma_color: float, sigma_space: float, device):
    key = (d, float(sigma_color), float(sigma_space), str(device))
    t = _BIL_CACHE.get(key)
    if t is None:
        maxk, radius = C.c_int(), C.c_int()
        L.call("irx_bilateral_tables", d, float(sigma_color), float(sigma_space), 3, None, None, None, 0,
               C.byref(maxk), C.byref(radius))
        cw = np.zeros(256 * 3, np.float32)
        sw = np.zeros(maxk.value, np.float32)
        dydx = np.zeros(2 * maxk.value, np.int32)
        L.call("irx_bilateral_tables", d, float(sigma_color), float(sigma_space), 3, C.c_void_p(cw.ctypes.data),
               C.c_void_p(sw.ctypes.data), C.c_void_p(dydx.ctypes.data), maxk.value, C.byref(maxk), C.byref(radius))
        t = (torch.from_numpy(cw).to(device), torch.from_numpy(sw).to(device), torch.from_numpy(dydx).to(device),
             maxk.value, radius.value)
        _BIL_CACHE[key] = t
    return t


def bilateral_filter(src: torch.Tensor, d: int = 9, sigma_color: float = 75.0, sigma_space: float = 75.0
                     ) -> torch.Tensor:
    """cv2.bilateralFilter on uint8 RGB/BGR images [H, W, 3] or [B, H, W, 3] (d = 9)."""
    x = _check(src)
    single = x.dim() == 3
    if single:
        x = x.unsqueeze(0)
    if x.shape[-1] != 3:
        raise ValueError("bilateralFilter: 3-channel images")
    cw, sw, dydx, maxk, radius = _bilateral_tables(d, sigma_color, sigma_space, x.device)
    out = torch.empty_like(x)
    B, H, W, _ = x.shape
    L.call("irx_bilateral_u8", C.c_void_p(torch.cuda.current_stream().cuda_stream), C.c_void_p(x.data_ptr()),
           C.c_void_p(out.data_ptr()), B, H, W, radius, C.c_void_p(sw.data_ptr()), C.c_void_p(dydx.data_ptr()),
           maxk, C.c_void_p(cw.data_ptr()))
    return out[0] if single else out


def median_blur(src: torch.Tensor, ksize: int = 5) -> torch.Tensor:
    """cv2.medianBlur(img, 5) on uint8 images [H, W, C] or [B, H, W, C], C <= 4."""
    x = _check(src)
    single = x.dim() == 3
    if single:
        x = x.unsqueeze(0)
    out = torch.empty_like(x)
    B, H, W, Cc = x.shape
    L.call("irx_median_blur_u8", C.c_void_p(torch.cuda.current_stream().cuda_stream), C.c_void_p(x.data_ptr()),
           C.c_void_p(out.data_ptr()), B, H, W, Cc, ksize)
    return out[0] if single else out


def denoise_opencv(image, strength: float, device: str = "cuda"):
    """RestorationPipeline._denoise_opencv (src/inference.py:500-522) with every step on the GPU: one upload,
    Lab conversion, NLM on L and ab, back to BGR, bilateral if strength > 0.6, median if > 0.8, one download."""
    from PIL import Image
    img = np.array(image.convert("RGB"))
    hs = float(np.clip(strength, 0.1, 1.0))
    h_value = hs * 10 if hs < 0.6 else 20          # luminance strength (src/inference.py:505-507)
    h_color = hs * 10 if hs < 0.6 else 20
    x = torch.from_numpy(img).to(device)
    den = fast_nl_means_denoising_colored(x, h_value, h_color, 7, 21)
    if strength > 0.6:
        den = bilateral_filter(den, 9, 75, 75)
    if strength > 0.8:
        den = median_blur(den, 5)
    return Image.fromarray(den.cpu().numpy())


def auto_mask(img: torch.Tensor):
    """_auto_mask_from_image (src/inference.py:805-840) on uint8 RGB CUDA images [H, W, 3] or [B, H, W, 3]:
    returns (masks uint8 [.., H, W] with 255 = damaged, keep bool per image = non-zero share >= 1 %)."""
    x = _check(img)
    single = x.dim() == 3
    if single:
        x = x.unsqueeze(0)
    B, H, W, _ = x.shape
    mask = torch.empty((B, H, W), dtype=torch.uint8, device=x.device)
    tmp = torch.empty_like(mask)
    counts = torch.empty(B, dtype=torch.int32, device=x.device)
    L.call("irx_auto_mask_u8", C.c_void_p(torch.cuda.current_stream().cuda_stream), C.c_void_p(x.data_ptr()), B, H,
           W, C.c_void_p(mask.data_ptr()), C.c_void_p(tmp.data_ptr()), C.c_void_p(counts.data_ptr()))
    keep = [int(c) / (H * W) >= 0.01 for c in counts.cpu().tolist()]
    return (mask[0], keep[0]) if single else (mask, keep)


_COLOR_TABLES: Dict[str, tuple] = {}


def colorize_lab(img: torch.Tensor) -> torch.Tensor:
    """_colorize_lab (src/inference.py:683-703) on uint8 RGB CUDA images [..., 3]; same bytes as
    classical.colorize_lab (the 256-entry tables come from its fp64 restatement)."""
    from . import classical
    x = _check(img)
    key = str(x.device)
    if key not in _COLOR_TABLES:
        lin = torch.from_numpy(classical.srgb_linear_lut()).to(x.device)
        cmap = torch.from_numpy(np.ascontiguousarray(classical.colorize_from_L(np.arange(256, dtype=np.uint8)))).to(
            x.device)
        _COLOR_TABLES[key] = (lin, cmap)
    lin, cmap = _COLOR_TABLES[key]
    out = torch.empty_like(x)
    L.call("irx_colorize_lab_u8", C.c_void_p(torch.cuda.current_stream().cuda_stream), C.c_void_p(x.data_ptr()),
           x.numel() // 3, C.c_void_p(lin.data_ptr()), C.c_void_p(cmap.data_ptr()), C.c_void_p(out.data_ptr()))
    return out
