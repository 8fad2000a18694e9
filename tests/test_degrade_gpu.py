"""GPU parity of the synthetic-degradation kernels (csrc/degrade.hip, through the C ABI) against the numpy
oracle (oracle/degrade_ref.py): bit-exact for the integer paths (noise with given draws, binomial blur,
cubic decimation, BGR2GRAY, stroke masks), within 1 level for the fp32 Lab L channel.  Parity against
cv2 itself is unpinned (OpenCV is absent from this image)."""
import random

import numpy as np
import pytest
import torch

from image_restoration_and_enhancement_amd import degrade as D
from oracle import degrade_ref as R

pytestmark = pytest.mark.gpu


def _img(shape, seed=0):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


def test_noise_bit_exact_with_reference_draws(device):
    img = _img((33, 47, 3))
    random.seed(1)
    np.random.seed(2)
    got = D.add_gaussian_noise(torch.from_numpy(img).to(device)).cpu().numpy()
    random.seed(1)
    np.random.seed(2)
    sigma = random.uniform(5, 8)
    ref = R.add_gaussian_noise(img, sigma, np.random.randn(*img.shape))
    assert np.array_equal(got, ref)


def test_noise_in_kernel_rng_distribution(device):
    img = torch.full((256, 256, 3), 128, dtype=torch.uint8, device=device)
    np.random.seed(3)
    a = D.add_gaussian_noise(img, (6, 6), exact_noise=False)
    np.random.seed(3)
    b = D.add_gaussian_noise(img, (6, 6), exact_noise=False)
    assert torch.equal(a, b)                           # reproducible from numpy's seed
    d = a.float() - 128       # uint8 truncation of 128 + 6z: mean -1/2, variance 36 + 1/12
    assert abs(d.mean().item() + 0.5) < 0.05 and abs(d.std().item() - (36 + 1 / 12) ** 0.5) < 0.1


@pytest.mark.parametrize("H,W,scale", [(64, 64, 4), (37, 50, 4), (30, 45, 3), (21, 17, 2), (8, 8, 4)])
def test_blur_and_cubic_down_bit_exact(device, H, W, scale):
    B = 4
    imgs = _img((B, H, W, 3), seed=H)
    ks = [1, 3, 5, 7]
    blur, lr = D.gaussian_blur_down(torch.from_numpy(imgs).to(device), ks, scale)
    for b in range(B):
        rb = R.gaussian_blur_u8(imgs[b], ks[b])
        assert np.array_equal(blur[b].cpu().numpy(), rb)
        assert np.array_equal(lr[b].cpu().numpy(), R.resize_cubic_down_u8(rb, scale))


def test_gray_modes(device):
    img = _img((70, 33, 3), seed=4)
    t = torch.from_numpy(img).to(device)
    assert np.array_equal(D.to_grayscale(t, "simple").cpu().numpy(), R.gray_simple_u8(img))
    assert np.array_equal(D.to_grayscale(t, "simple", rgb=True).cpu().numpy(), R.gray_simple_u8(img, rgb=True))
    lab = D.to_grayscale(t, "lab").cpu().numpy().astype(int)
    assert np.abs(lab - R.gray_lab_u8(img).astype(int)).max() <= 1
    every = np.stack(np.meshgrid(np.arange(256), np.arange(0, 256, 51), np.arange(0, 256, 85)), -1)
    every = every.reshape(-1, 3).astype(np.uint8)[None]
    lab = D.to_grayscale(torch.from_numpy(every).to(device), "lab").cpu().numpy().astype(int)
    assert np.abs(lab - R.gray_lab_u8(every).astype(int)).max() <= 1


def test_strokes_and_masked_input_bit_exact(device):
    H, W = 96, 128
    random.seed(7)
    per = [D.draw_free_form_strokes(H, W, (3, 7), (5, 20)), D.draw_free_form_strokes(H, W, (8, 15), (20, 40)), []]
    imgs = _img((3, H, W, 3), seed=5)
    mask, masked = D.rasterize_strokes(H, W, per, device, torch.from_numpy(imgs).to(device))
    for b in range(3):
        ref = R.stroke_mask(H, W, per[b])
        assert np.array_equal(mask[b].cpu().numpy(), ref)
        exp = imgs[b].copy()
        exp[ref == 255] = 0
        assert np.array_equal(masked[b].cpu().numpy(), exp)
    assert mask[2].sum().item() == 0


def test_make_pairs_batch(device):
    random.seed(0)
    np.random.seed(0)
    batch = torch.from_numpy(_img((3, 64, 48, 3), seed=9)).to(device)
    out = D.make_pairs(batch)
    assert out["denoise"].shape == batch.shape and out["sr"].shape == (3, 16, 12, 3)
    assert out["colorize"].shape == (3, 64, 48) and out["inpaint_mask"].shape == (3, 64, 48)
    m = out["inpaint_mask"] == 255
    assert (out["inpaint"][m] == 0).all() and torch.equal(out["inpaint"][~m], batch[~m])
