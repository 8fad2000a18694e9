"""CPU tests of the drop-in `RestorationPipeline` host logic (reference src/inference.py): constructor
surface, fallback semantics when the diffusion engine cannot load (no GPU here), grey detection,
mask normalisation / auto-mask, `process` chaining, IrxError propagation, and the classical helpers."""
import logging

import numpy as np
import pytest
import torch
from PIL import Image

from image_restoration_and_enhancement_amd import classical as CL
from image_restoration_and_enhancement_amd import image_processor as ip
from image_restoration_and_enhancement_amd import inference as INF
from image_restoration_and_enhancement_amd._lib import IrxError


def rgb(h=24, w=32, seed=0):
    rng = np.random.default_rng(seed)
    return Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8))


def gray_rgb(h=24, w=32, seed=0):
    rng = np.random.default_rng(seed)
    g = rng.integers(40, 200, (h, w), dtype=np.uint8)
    return Image.fromarray(np.repeat(g[..., None], 3, axis=2))


def test_src_shim_surface():
    import src.inference as S
    import src.metrics as SM
    assert S.RestorationPipeline is INF.RestorationPipeline
    assert S.TASK_MODEL_DIRS == {"denoise": "outputs/models/denoising/best",
                                 "sr": "outputs/models/super_resolution/best",
                                 "colorize": "outputs/models/colorization/best",
                                 "inpaint": "outputs/models/inpainting/best"}
    assert callable(SM.evaluate_task) and callable(SM.print_results)


def test_constructor_attributes():
    p = INF.RestorationPipeline(device="cpu", seed=7)
    assert p.device == "cpu" and p.dtype == torch.float32 and p.seed == 7 and p.models == {}
    assert set(p.config) == {"denoise", "sr", "colorize", "inpaint"}
    assert p.prompts["denoise"] == "clean high quality photo, no noise, sharp details"
    p2 = INF.RestorationPipeline(device="cpu", config={"denoise": {"fine_tuned_dir": "nonexistent",
                                                                   "pretrained_id": "x/y"}})
    assert p2.config["denoise"]["fine_tuned_dir"] == "nonexistent" and "sr" in p2.config
    with pytest.raises(ValueError):
        INF.RestorationPipeline(device="cpu", config={"engine": {"dtype": "int8"}})
    p3 = INF.RestorationPipeline(device="cpu", config={"engine": {"dtype": "fp16"}})
    assert p3.engine_dtype == "fp16" and p3.dtype == torch.float32      # CPU host: fallbacks only
    # defaults: fp16 (the reference's GPU dtype, src/inference.py:57); a bf16 UNet gets an fp16 VAE
    assert INF.RestorationPipeline(device="cpu").engine_dtype == "fp16"
    p4 = INF.RestorationPipeline(device="cpu", config={"engine": {"dtype": "bf16"}})
    assert p4.engine_dtype == "bf16" and p4.vae_dtype == "fp16"
    p5 = INF.RestorationPipeline(device="cpu", config={"engine": {"dtype": "bf16", "vae_dtype": "bf16"}})
    assert p5.vae_dtype == "bf16"


def test_fallbacks_without_gpu(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)            # no outputs/models/* here -> FileNotFoundError -> fallback
    p = INF.RestorationPipeline(device="cpu")
    img = rgb(16, 20)
    out = p.super_resolve(img, scale=2)
    assert p.models["sr"] == "lanczos"
    assert np.array_equal(np.array(out), np.array(img.resize((40, 32), Image.LANCZOS)))
    assert p.inpaint(img, mask=Image.new("L", (20, 16), 255)) is img and p.models["inpaint"] is None
    col = p.colorize(gray_rgb(16, 16))
    assert p.models["colorize"] == "improved" and col.size == (16, 16) and col.mode == "RGB"
    den = p.denoise(rgb(12, 12), strength=0.3)
    assert p.models["denoise"] is None and den.size == (12, 12)


def test_colour_image_skips_colorize(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    p = INF.RestorationPipeline(device="cpu")
    img = rgb()
    assert INF.RestorationPipeline.is_color(img)
    assert p.colorize(img) is img
    assert not INF.RestorationPipeline.is_color(gray_rgb())
    g = INF.RestorationPipeline.gray_to_rgb(Image.fromarray(np.array(rgb())[..., 0]))
    assert np.array(g).shape[2] == 3


def test_process_chain_and_error_swallowing(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    p = INF.RestorationPipeline(device="cpu")
    img = rgb(8, 8)
    res = p.process(img, ["sr", "inpaint"], sr_scale=2, mask=Image.new("L", (16, 16), 255))
    assert res["original"] is img and res["super_resolved"].size == (16, 16)
    assert res["inpainted"] is res["super_resolved"] and res["final"] is res["inpainted"]

    def boom(*a, **k):
        raise RuntimeError("model failure")

    monkeypatch.setattr(p, "super_resolve", boom)
    res = p.process(img, ["sr"])           # per-task exceptions are logged and skipped
    assert res["final"] is img and "super_resolved" not in res


def test_missing_native_library_is_loud(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    p = INF.RestorationPipeline(device="cpu", config={"denoise": {"fine_tuned_dir": "x", "pretrained_id": "y",
                                                                  "weights": "random"}})

    def no_lib(*a, **k):
        raise IrxError("native library not built")

    monkeypatch.setattr(p, "_load_native", no_lib)
    with pytest.raises(IrxError):
        p.denoise(rgb())
    with pytest.raises(IrxError):
        p.process(rgb(), ["denoise"])


def test_normalize_mask_polarity_and_size():
    m = np.zeros((10, 10), np.uint8)
    m[:2, :2] = 255                         # 4 % white -> treated as inverted
    out = np.array(ip.normalize_mask(Image.fromarray(m), (10, 10)))
    assert out[0, 0] == 0 and out[5, 5] == 255
    m2 = np.zeros((10, 10), np.uint8)
    m2[:5] = 255
    out2 = ip.normalize_mask(Image.fromarray(m2), (20, 30))
    assert out2.size == (20, 30)
    assert np.array(out2)[0, 0] == 255


def test_mask_to_binary_threshold():
    m = Image.fromarray(np.array([[0, 127, 128, 255]], np.uint8))
    assert ip.mask_to_binary(m, 1, 4).tolist() == [[0.0, 0.0, 1.0, 1.0]]


def test_nearest_downsample_matches_torch():
    rng = np.random.default_rng(0)
    m = (rng.random((2, 37, 50)) > 0.5).astype(np.float32)
    ref = torch.nn.functional.interpolate(torch.from_numpy(m)[:, None], size=(5, 6))[:, 0].numpy()
    assert np.array_equal(ip.nearest_downsample(m, 5, 6), ref)


def test_auto_mask():
    a = np.full((40, 40, 3), 128, np.uint8)
    assert CL.auto_mask(Image.fromarray(a)) is None
    a[5:20, 5:20] = 10                       # dark damage, 14 % of the image
    m = CL.auto_mask(Image.fromarray(a))
    mm = np.array(m)
    assert mm[10, 10] == 255 and mm[30, 30] == 0
    assert (mm > 0).sum() == 15 * 15


def test_gray_fixed_point():
    px = np.array([[[255, 255, 255], [255, 0, 0], [0, 255, 0], [0, 0, 255], [0, 0, 0]]], np.uint8)
    assert CL.rgb_to_gray_u8(px).tolist() == [[255, 76, 150, 29, 0]]


def test_lab_round_trip():
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (16, 16, 3), dtype=np.uint8)
    back = CL.lab_u8_to_rgb(CL.rgb_to_lab_u8(a))
    d = np.abs(back.astype(int) - a.astype(int))
    assert d.mean() < 1.5 and d.max() <= 16        # 8-bit LAB quantisation (dark saturated colours)


def test_median_and_bilateral_shapes():
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, (9, 11, 3), dtype=np.uint8)
    med = CL.median5(a)
    assert med.shape == a.shape and med[4, 5, 0] == np.median(a[2:7, 3:8, 0])
    flat = np.full((9, 11, 3), 77, np.uint8)
    assert np.array_equal(CL.bilateral(flat), flat)


def test_nl_means_reduces_noise():
    rng = np.random.default_rng(2)
    clean = np.full((24, 24, 1), 120.0)
    noisy = np.clip(np.rint(clean + rng.normal(0, 8, clean.shape)), 0, 255).astype(np.uint8)
    out = CL.nl_means_u8(noisy, 10.0, 7, 11)
    assert np.abs(out - clean).mean() < 0.5 * np.abs(noisy - clean).mean()


def test_prediction_driver_layout(tmp_path):
    """scripts/generate_predictions.py keeps the reference's {task}/{split}/<name> layout (CPU: fallbacks)."""
    import subprocess
    import sys
    from pathlib import Path
    root = tmp_path / "pairs"
    rng = np.random.default_rng(3)
    for task in ("denoise", "sr_x4", "colorize", "inpaint"):
        d = root / task / "test" / "input"
        d.mkdir(parents=True)
        Image.fromarray(rng.integers(0, 256, (16, 16, 3), dtype=np.uint8)).save(d / "a.png")
    (root / "inpaint" / "test" / "mask").mkdir()
    Image.new("L", (16, 16), 255).save(root / "inpaint" / "test" / "mask" / "a.png")
    out = tmp_path / "pred"
    script = Path(__file__).resolve().parents[1] / "scripts" / "generate_predictions.py"
    r = subprocess.run([sys.executable, str(script), "--test_root", str(root), "--output_root", str(out)],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600,
                       env={**__import__("os").environ, "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 0, r.stderr[-2000:]
    assert Image.open(out / "denoise" / "test" / "a.png").size == (16, 16)
    assert Image.open(out / "sr_x4" / "test" / "a.png").size == (64, 64)
    assert (out / "colorize" / "test" / "a.png").exists() and (out / "inpaint" / "test" / "a.png").exists()


def test_restore_batch_strength_zero_and_fallback(tmp_path, monkeypatch):
    """restore_batch keeps strength=0.0 (not 'unset'), and a failing batched engine call falls back per image
    to the single-image entry point, as _denoise_sd does."""
    monkeypatch.chdir(tmp_path)
    p = INF.RestorationPipeline(device="cpu")
    img = rgb(12, 16, seed=3)
    got = p.restore_batch("denoise", [img], strength=0.0)[0]
    assert np.array_equal(np.array(got), np.array(p.denoise(img, strength=0.0)))

    def engine_fails(*a, **k):
        raise ValueError("strength too small: no denoising steps")

    monkeypatch.setattr(p, "load_denoise_model", lambda: None)
    p.models["denoise"] = INF.NativeSDModel(None, "img2img", "test")
    monkeypatch.setattr(p, "_img2img", engine_fails)
    out = p.restore_batch("denoise", [img, rgb(12, 16, seed=4)], strength=0.0)
    assert np.array_equal(np.array(out[0]), np.array(CL.denoise_opencv(img, 0.0)))
