"""GPU parity of the fast non-local-means kernel (csrc/nlmeans.hip, through the C ABI) against the integer
oracle (oracle/nlm_ref.py, OpenCV's FastNlMeansDenoisingInvoker restated): bit-exact on every case — ragged and
tiny images (reflect-101 folding more than once), both channel-group widths, both compiled window sizes,
channel groups embedded in 3-channel pixels, batches.  Parity against cv2 itself is unpinned (OpenCV absent)."""
import numpy as np
import pytest
import torch
from PIL import Image

from image_restoration_and_enhancement_amd import _lib as L
from image_restoration_and_enhancement_amd import classical as CL
from image_restoration_and_enhancement_amd import nlmeans as N
from oracle import nlm_ref as R

pytestmark = pytest.mark.gpu


def _img(shape, seed=0):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


@pytest.mark.parametrize("shape", [(1, 7), (5, 3), (33, 40), (64, 32), (70, 45)])
@pytest.mark.parametrize("cn", [1, 2])
@pytest.mark.parametrize("h", [3.0, 20.0])
def test_nlm_small_window_bit_exact(device, shape, cn, h):
    img = _img((2, *shape, cn), seed=shape[0] * 7 + cn)
    got = N.fast_nl_means_denoising(torch.from_numpy(img).to(device), h, 3, 5).cpu().numpy()
    for b in range(2):
        assert np.array_equal(got[b], R.nl_means_u8(img[b], h, 3, 5)), b


@pytest.mark.parametrize("shape", [(13, 9), (37, 50), (96, 64)])
@pytest.mark.parametrize("cn", [1, 2])
def test_nlm_reference_window_bit_exact(device, shape, cn):
    img = _img((*shape, cn), seed=shape[1] + cn)
    got = N.fast_nl_means_denoising(torch.from_numpy(img).to(device), 20.0 if cn == 2 else 10.0).cpu().numpy()
    assert np.array_equal(got, R.nl_means_u8(img, 20.0 if cn == 2 else 10.0))


def test_nlm_lab_groups_in_three_channel_pixels(device):
    lab = _img((2, 45, 77, 3), seed=9)
    got = N.fast_nl_means_denoising_lab(torch.from_numpy(lab).to(device), 7.0, 12.0).cpu().numpy()
    for b in range(2):
        ref = np.concatenate([R.nl_means_u8(lab[b, ..., :1], 7.0), R.nl_means_u8(lab[b, ..., 1:], 12.0)], -1)
        assert np.array_equal(got[b], ref), b


def test_nlm_full_size_noisy_photo_like(device):
    """256x256 smooth image + noise (the regime where most weights are non-zero): exact vs the oracle and
    denoising, i.e. closer to the clean image than the input."""
    y, x = np.mgrid[0:256, 0:256]
    clean = np.stack([(x + y) / 2, 128 + 60 * np.sin(x / 20.0)], -1)
    noisy = np.clip(np.rint(clean + np.random.default_rng(3).normal(0, 10, clean.shape)), 0, 255).astype(np.uint8)
    got = N.fast_nl_means_denoising(torch.from_numpy(noisy).to(device), 20.0).cpu().numpy()
    assert np.array_equal(got, R.nl_means_u8(noisy, 20.0))
    assert np.abs(got - clean).mean() < 0.6 * np.abs(noisy - clean).mean()


def test_nlm_colored_matches_cpu_form(device):
    img = _img((40, 52, 3), seed=11)
    got = N.fast_nl_means_denoising_colored(img, 10.0, 10.0)
    assert np.array_equal(got, CL.fast_nl_means_denoising_colored(img, 10.0, 10.0))


def test_pipeline_classical_denoise_runs_gpu_nlm(device):
    from image_restoration_and_enhancement_amd.inference import RestorationPipeline
    img = Image.fromarray(_img((48, 40, 3), seed=12))
    p = RestorationPipeline.__new__(RestorationPipeline)
    p.device = "cuda"
    for strength in (0.3, 0.7, 0.9):
        got = np.array(p._denoise_opencv(img, strength))
        assert np.array_equal(got, np.array(CL.denoise_opencv(img, strength))), strength


def test_nlm_rejects_unsupported_windows_and_aliasing(device):
    x = torch.zeros((1, 16, 16, 1), dtype=torch.uint8, device=device)
    with pytest.raises(L.IrxError):
        N.fast_nl_means_denoising(x, 10.0, 5, 11)
    with pytest.raises(L.IrxError):
        N.denoise_group(x, x, 10.0, 0, 1)
    with pytest.raises(ValueError):
        N.fast_nl_means_denoising(torch.zeros((16, 16, 3), dtype=torch.uint8, device=device), 10.0)


@pytest.mark.parametrize("shape", [(1, 1), (3, 5), (8, 32), (37, 70), (130, 97)])
def test_bilateral_bit_exact(device, shape):
    from oracle import filters_ref as F
    img = _img((2, *shape, 3), seed=shape[1])
    got = N.bilateral_filter(torch.from_numpy(img).to(device), 9, 75, 75).cpu().numpy()
    for b in range(2):
        assert np.array_equal(got[b], F.bilateral_u8(img[b], 9, 75, 75)), b


def test_bilateral_other_sigmas(device):
    from oracle import filters_ref as F
    img = _img((64, 48, 3), seed=4)
    got = N.bilateral_filter(torch.from_numpy(img).to(device), 9, 20.0, 3.0).cpu().numpy()
    assert np.array_equal(got, F.bilateral_u8(img, 9, 20.0, 3.0))


@pytest.mark.parametrize("shape,c", [((1, 1), 3), ((4, 3), 1), ((33, 65), 3), ((40, 41), 4)])
def test_median_exact(device, shape, c):
    from oracle import filters_ref as F
    img = _img((2, *shape, c), seed=c + shape[0])
    got = N.median_blur(torch.from_numpy(img).to(device), 5).cpu().numpy()
    for b in range(2):
        assert np.array_equal(got[b], F.median5_u8(img[b])), b


@pytest.mark.parametrize("tmpl,search", [(3, 5), (7, 21)])
def test_nlm_strip8_variant_bit_exact(device, tmpl, search):
    img = _img((2, 45, 70, 1), seed=tmpl)
    L.call("irx_set_option", b"nlm_v2", 0)
    L.call("irx_set_option", b"nlm_strip", 8)
    try:
        got = N.fast_nl_means_denoising(torch.from_numpy(img).to(device), 12.0, tmpl, search).cpu().numpy()
    finally:
        L.call("irx_set_option", b"nlm_strip", 4)
        L.call("irx_set_option", b"nlm_v2", 1)
    for b in range(2):
        assert np.array_equal(got[b], R.nl_means_u8(img[b], 12.0, tmpl, search)), b


@pytest.mark.parametrize("tmpl,search", [(3, 5), (7, 21)])
@pytest.mark.parametrize("cn", [1, 2])
@pytest.mark.parametrize("shape", [(1, 7), (13, 9), (37, 130), (70, 45)])
def test_nlm_v1_register_window_bit_exact(device, tmpl, search, cn, shape):
    """The v1 kernel (per-thread register window, irx option nlm_v2 = 0); the default v2 runs everywhere else."""
    img = _img((2, *shape, cn), seed=tmpl + cn + shape[1])
    L.call("irx_set_option", b"nlm_v2", 0)
    try:
        got = N.fast_nl_means_denoising(torch.from_numpy(img).to(device), 15.0, tmpl, search).cpu().numpy()
    finally:
        L.call("irx_set_option", b"nlm_v2", 1)
    for b in range(2):
        assert np.array_equal(got[b], R.nl_means_u8(img[b], 15.0, tmpl, search)), b


@pytest.mark.parametrize("tmpl,search", [(3, 5), (7, 21)])
@pytest.mark.parametrize("cn", [1, 2])
def test_nlm_v2_dpp_centre_variant_bit_exact(device, tmpl, search, cn):
    img = _img((2, 37, 130, cn), seed=tmpl * cn)
    L.call("irx_set_option", b"nlm_v2", 2)
    try:
        got = N.fast_nl_means_denoising(torch.from_numpy(img).to(device), 15.0, tmpl, search).cpu().numpy()
    finally:
        L.call("irx_set_option", b"nlm_v2", 1)
    for b in range(2):
        assert np.array_equal(got[b], R.nl_means_u8(img[b], 15.0, tmpl, search)), b


def test_lab_conversion_exhaustive(device):
    """Every one of the 2^24 byte triplets, both directions, against classical's fp64 restatement."""
    v = np.arange(1 << 24, dtype=np.uint32)
    px = np.stack([v & 255, (v >> 8) & 255, v >> 16], -1).astype(np.uint8).reshape(4096, 4096, 3)
    t = torch.from_numpy(px).to(device)
    fwd = N.lab_convert(t, 0).cpu().numpy()
    bad = np.argwhere((fwd != CL.lbgr_to_lab_u8(px)).any(-1))
    assert len(bad) == 0, (len(bad), px[tuple(bad[0])])
    inv = N.lab_convert(t, 1).cpu().numpy()
    bad = np.argwhere((inv != CL.lab_u8_to_lbgr(px)).any(-1))
    assert len(bad) == 0, (len(bad), px[tuple(bad[0])])


def test_colored_device_tensor_path(device):
    img = _img((2, 40, 52, 3), seed=13)
    got = N.fast_nl_means_denoising_colored(torch.from_numpy(img).to(device), 10.0, 12.0).cpu().numpy()
    for b in range(2):
        assert np.array_equal(got[b], CL.fast_nl_means_denoising_colored(img[b], 10.0, 12.0))


def _damaged(shape, seed):
    rng = np.random.default_rng(seed)
    img = rng.integers(20, 240, shape, dtype=np.uint8)
    H, W = shape[-3], shape[-2]
    for _ in range(6):
        y, x = rng.integers(0, H), rng.integers(0, W)
        img[..., y:y + rng.integers(1, 9), x:x + rng.integers(1, 20), :] = rng.choice([0, 255])
    return img


@pytest.mark.parametrize("shape", [(1, 1), (3, 7), (37, 70), (64, 64), (97, 130)])
def test_auto_mask_exact(device, shape):
    from oracle import filters_ref as F
    img = _damaged((3, *shape, 3), seed=shape[1])
    masks, keep = N.auto_mask(torch.from_numpy(img).to(device))
    masks = masks.cpu().numpy()
    for b in range(3):
        m, k = F.auto_mask_u8(img[b])
        assert np.array_equal(masks[b], m) and keep[b] == k, b


def test_pipeline_auto_mask_runs_gpu(device):
    from image_restoration_and_enhancement_amd.inference import RestorationPipeline
    p = RestorationPipeline.__new__(RestorationPipeline)
    p.device = "cuda"
    for seed in (1, 2):
        img = Image.fromarray(_damaged((80, 96, 3), seed))
        got, ref = p._auto_mask_from_image(img), CL.auto_mask(img)
        assert (got is None) == (ref is None)
        if ref is not None:
            assert np.array_equal(np.array(got), np.array(ref))
    flat = Image.fromarray(np.full((40, 40, 3), 128, np.uint8))
    assert p._auto_mask_from_image(flat) is None


def test_colorize_exhaustive(device):
    """Every RGB triplet through the GPU colorize fallback against classical.colorize_lab's bytes."""
    v = np.arange(1 << 24, dtype=np.uint32)
    px = np.stack([v & 255, (v >> 8) & 255, v >> 16], -1).astype(np.uint8).reshape(4096, 4096, 3)
    got = N.colorize_lab(torch.from_numpy(px).to(device)).cpu().numpy()
    ref = CL.colorize_from_L(CL.rgb_to_lab_u8(px)[..., 0])
    bad = np.argwhere((got != ref).any(-1))
    assert len(bad) == 0, (len(bad), px[tuple(bad[0])])


def test_pipeline_colorize_fallback_runs_gpu(device):
    from image_restoration_and_enhancement_amd.inference import RestorationPipeline
    p = RestorationPipeline.__new__(RestorationPipeline)
    p.device = "cuda"
    img = Image.fromarray(_img((33, 47, 3), seed=17))
    assert np.array_equal(np.array(p._colorize_lab(img)), np.array(CL.colorize_lab(img)))


@pytest.mark.parametrize("strip", [2, 8, 16])
@pytest.mark.parametrize("cn", [1, 2])
def test_nlm_v2_strip_variants_bit_exact(device, strip, cn):
    img = _img((2, 70, 130, cn), seed=strip + cn)
    L.call("irx_set_option", b"nlm2_strip", strip)
    try:
        got = N.fast_nl_means_denoising(torch.from_numpy(img).to(device), 15.0).cpu().numpy()
    finally:
        L.call("irx_set_option", b"nlm2_strip", 4)
    for b in range(2):
        assert np.array_equal(got[b], R.nl_means_u8(img[b], 15.0)), b
