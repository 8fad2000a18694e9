"""GPU parity of every hand-written kernel (through the C ABI) against fp32 PyTorch-CPU references.

Tolerances (max |err| / max |ref|): fp32 path 1e-4 (exact-f32 MFMA / fp32 VALU, different
summation order only); bf16 path 2e-2, fp16 path 5e-3 (16-bit storage of inputs/outputs, fp32
accumulation) with the reference fed the same rounded inputs.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from tests import opref as O

pytestmark = pytest.mark.gpu

TOL = {torch.float32: 1e-4, torch.bfloat16: 2e-2, torch.float16: 5e-3}
DTS = [torch.float32, torch.bfloat16, torch.float16]
DT16 = [torch.bfloat16, torch.float16]


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


def _dev(x, dt, device):
    return x.to(dt).to(device).contiguous()


def _q(x, dt):      # what the device sees, back in fp32 for the CPU reference
    return x.to(dt).float()


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("case", [
    # (N, H, W, Cin, Cout, k, stride, pad)
    (2, 16, 16, 64, 64, 3, 1, 1),
    (1, 13, 9, 32, 40, 3, 1, 1),       # ragged spatial + N not a tile multiple
    (2, 17, 12, 64, 64, 3, 2, 1),      # UNet Downsample2D on odd size
    (1, 8, 8, 8, 320, 3, 1, 1),        # conv_in (4 channels padded to 8)
    (2, 8, 8, 320, 4, 3, 1, 1),        # conv_out (N = 4)
    (1, 12, 12, 96, 48, 1, 1, 0),      # 1x1 shortcut
    (1, 40, 24, 128, 256, 3, 1, 1),
])
def test_conv(device, dt, case):
    N, H, W, Ci, Co, k, s, p = case
    x = _r(N, Ci, H, W, seed=1)
    w = _r(Co, Ci, k, k, seed=2, scale=1 / math.sqrt(Ci * k * k))
    b = _r(Co, seed=3)
    got = O.conv2d(_dev(x.permute(0, 2, 3, 1), dt, device), w.to(dt).float(), b, stride=s, pad=(p, p))
    ref = F.conv2d(_q(x, dt), _q(w, dt), b, stride=s, padding=p).permute(0, 2, 3, 1)
    assert got.shape == ref.shape
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTS)
def test_conv_vae_downsample_asym_pad(device, dt):
    # F.pad(x, (0,1,0,1)) + 3x3 stride 2 pad 0 (AutoencoderKL Downsample2D, padding=0)
    x = _r(2, 64, 18, 14, seed=4)
    w = _r(64, 64, 3, 3, seed=5, scale=0.05)
    b = _r(64, seed=6)
    Ho, Wo = (18 + 1 - 3) // 2 + 1, (14 + 1 - 3) // 2 + 1
    got = O.conv2d(_dev(x.permute(0, 2, 3, 1), dt, device), w.to(dt).float(), b, stride=2, pad=(0, 0),
                   out_hw=(Ho, Wo))
    ref = F.conv2d(F.pad(_q(x, dt), (0, 1, 0, 1)), _q(w, dt), b, stride=2).permute(0, 2, 3, 1)
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("src_hw,dst_hw", [((8, 8), (16, 16)), ((6, 4), (11, 7)), ((5, 6), (10, 12))])
def test_conv_fused_upsample(device, dt, src_hw, dst_hw):
    # Upsample2D: nearest resize (x2 or to the skip size) fused into the following 3x3 conv
    x = _r(2, 32, *src_hw, seed=7)
    w = _r(48, 32, 3, 3, seed=8, scale=0.06)
    b = _r(48, seed=9)
    got = O.conv2d(_dev(x.permute(0, 2, 3, 1), dt, device), w.to(dt).float(), b, up_hw=dst_hw)
    up = F.interpolate(_q(x, dt), size=dst_hw, mode="nearest")
    ref = F.conv2d(up, _q(w, dt), b, padding=1).permute(0, 2, 3, 1)
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("k", [1, 3])
def test_conv_concat_rowadd_residual(device, dt, k):
    # up-block resnet: cat([h, skip]) read from two sources; + time-embedding row add; + residual
    N, H, W, C0, C1, Co = 2, 10, 9, 64, 32, 80
    x0, x1 = _r(N, C0, H, W, seed=10), _r(N, C1, H, W, seed=11)
    w = _r(Co, C0 + C1, k, k, seed=12, scale=0.05)
    b = _r(Co, seed=13)
    temb = _r(N, Co + 16, seed=14)             # padded row stride like the fused time_emb_proj output
    res = _r(N, H, W, Co, seed=15)
    p = k // 2
    got = O.conv2d(_dev(x0.permute(0, 2, 3, 1), dt, device), w.to(dt).float(), b, pad=(p, p),
                   x1=_dev(x1.permute(0, 2, 3, 1), dt, device), rowadd=temb.to(device).contiguous(),
                   residual=_dev(res, dt, device))
    ref = F.conv2d(torch.cat([_q(x0, dt), _q(x1, dt)], 1), _q(w, dt), b, padding=p)
    ref = ref + temb[:, :Co, None, None]
    ref = ref.permute(0, 2, 3, 1) + _q(res, dt)
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("M,N,K", [(4096, 320, 320), (77, 2304, 768), (300, 2560, 320), (16, 1280, 320),
                                   (1024, 640, 2560), (5, 24, 8)])
def test_gemm(device, dt, M, N, K):
    A = _r(M, K, seed=20)
    Bw = _r(N, K, seed=21, scale=1 / math.sqrt(K))
    bias = _r(N, seed=22)
    got = O.gemm(_dev(A, dt, device), _dev(Bw, dt, device), bias=bias.to(device))
    ref = _q(A, dt) @ _q(Bw, dt).T + bias
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("act", [1, 2, 3])
def test_gemm_act_residual_f32out(device, dt, act):
    M, N, K = 200, 96, 64
    A, Bw, bias, res = _r(M, K, seed=23), _r(N, K, seed=24, scale=0.2), _r(N, seed=25), _r(M, N, seed=26)
    got = O.gemm(_dev(A, dt, device), _dev(Bw, dt, device), bias=bias.to(device), act=act,
                 residual=_dev(res, dt, device), out_f32=True, alpha=0.5)
    y = 0.5 * (_q(A, dt) @ _q(Bw, dt).T) + bias
    y = {1: F.silu, 2: F.gelu, 3: lambda v: v * torch.sigmoid(1.702 * v)}[act](y)
    ref = y + _q(res, dt)
    assert got.dtype == torch.float32
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTS)
def test_gemm_batched(device, dt):
    b, M, N, K = 3, 130, 70, 64
    A, Bw = _r(b, M, K, seed=27), _r(b, N, K, seed=28, scale=0.2)
    got = O.gemm(_dev(A, dt, device), _dev(Bw, dt, device), batch=b, out_f32=True)
    ref = torch.bmm(_q(A, dt), _q(Bw, dt).transpose(1, 2))
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("C0,C1,H,W,silu,eps", [(320, 0, 16, 16, True, 1e-5), (1280, 640, 8, 8, True, 1e-5),
                                                (128, 0, 33, 20, False, 1e-6), (640, 0, 7, 5, False, 1e-6),
                                                (2560, 0, 4, 4, True, 1e-5)])
def test_group_norm(device, dt, C0, C1, H, W, silu, eps, N=2):
    x0 = _r(N, C0, H, W, seed=30) * 3 + 1.5        # offset mean: exercises the variance path
    x1 = _r(N, C1, H, W, seed=31) if C1 else None
    g, b = 1 + 0.1 * _r(C0 + C1, seed=32), 0.1 * _r(C0 + C1, seed=33)
    got = O.group_norm(_dev(x0.permute(0, 2, 3, 1), dt, device), g.to(device), b.to(device), eps, silu=silu,
                       x1=_dev(x1.permute(0, 2, 3, 1), dt, device) if C1 else None)
    xin = torch.cat([_q(x0, dt)] + ([_q(x1, dt)] if C1 else []), 1)
    ref = F.group_norm(xin, 32, g, b, eps)
    ref = (F.silu(ref) if silu else ref).permute(0, 2, 3, 1)
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("N,C0,C1,H,W", [(16, 2560, 0, 8, 8), (16, 1280, 1280, 8, 8), (16, 1280, 640, 16, 16),
                                         (16, 320, 0, 64, 64), (3, 128, 0, 96, 80), (16, 960, 0, 5, 3)])
def test_group_norm_unet_shapes(device, N, C0, C1, H, W):
    """Batch-16 UNet level shapes: channel slabs (C >= 2048), multi-chunk images, tiny images."""
    test_group_norm(device, torch.bfloat16, C0, C1, H, W, True, 1e-5, N=N)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("rows,Cc", [(4096, 320), (154, 768), (64, 1280), (3, 640)])
def test_layer_norm(device, dt, rows, Cc):
    x = _r(rows, Cc, seed=40) * 2 + 0.5
    g, b = 1 + 0.1 * _r(Cc, seed=41), 0.1 * _r(Cc, seed=42)
    got = O.layer_norm(_dev(x, dt, device), g.to(device), b.to(device), 1e-5)
    ref = F.layer_norm(_q(x, dt), (Cc,), g, b, 1e-5)
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("B,Lq,Lk,C,heads,causal", [
    (2, 256, 256, 320, 8, False),     # d = 40 self-attention
    (2, 200, 77, 320, 8, False),      # cross-attention, ragged Lq, Lk = 77
    (1, 100, 100, 640, 8, False),     # d = 80
    (2, 64, 77, 1280, 8, False),      # d = 160 cross
    (1, 300, 300, 1280, 8, False),    # d = 160 self
    (2, 77, 77, 768, 12, True),       # CLIP causal, d = 64
])
def test_attention(device, dt, B, Lq, Lk, C, heads, causal):
    q, k, v = _r(B, Lq, C, seed=50), _r(B, Lk, C, seed=51), _r(B, Lk, C, seed=52)
    got = O.attention(_dev(q, dt, device), _dev(k, dt, device), _dev(v, dt, device), heads, causal)
    ref = O.ref_attention(_q(q, dt), _q(k, dt), _q(v, dt), heads, causal)
    assert O.rel_err(got, ref) < TOL[dt] * (1 if dt == torch.float32 else 2)


@pytest.mark.parametrize("dt", DTS)
def test_attention_fused_qkv_strides(device, dt):
    # q|k|v packed in one [B, L, 3C] buffer (the engine's fused projection)
    B, Lq, C, heads = 2, 130, 640, 8
    qkv = _dev(_r(B, Lq, 3 * C, seed=53), dt, device)
    got = O.attention(qkv[:, :, :C], qkv[:, :, C:2 * C], qkv[:, :, 2 * C:], heads)
    c = qkv.float().cpu()
    ref = O.ref_attention(c[:, :, :C], c[:, :, C:2 * C], c[:, :, 2 * C:], heads)
    assert O.rel_err(got, ref) < TOL[dt] * (1 if dt == torch.float32 else 2)


@pytest.mark.parametrize("dt", DTS)
def test_attention_softmax_spike(device, dt):
    # a key whose score dwarfs the rest, arriving in a late tile: forces the online-softmax rescale
    B, L, C, heads = 1, 256, 320, 8
    q, k, v = _r(B, L, C, seed=54), _r(B, L, C, seed=55), _r(B, L, C, seed=56)
    k[:, 200] = q[:, 3] * 4.0
    got = O.attention(_dev(q, dt, device), _dev(k, dt, device), _dev(v, dt, device), heads)
    ref = O.ref_attention(_q(q, dt), _q(k, dt), _q(v, dt), heads)
    assert O.rel_err(got, ref) < TOL[dt] * (1 if dt == torch.float32 else 2)


@pytest.mark.parametrize("dt", DTS)
def test_geglu(device, dt):
    x = _r(300, 2 * 1280, seed=60)
    got = O.geglu(_dev(x, dt, device))
    h, g = _q(x, dt).chunk(2, dim=-1)
    ref = h * F.gelu(g)
    assert O.rel_err(got, ref) < TOL[dt]


# ------------------------------------------------------------------ large-tile (8-wave LDS-DMA) path
@pytest.fixture(params=[(1, 0, 0), (1, 1, 0), (1, 2, 0), (1, 0, 1), (0, 0, 0)],
                ids=["two_stage", "ring32", "ring64", "small4w", "4wave"])
def tiles(request):
    from image_restoration_and_enhancement_amd import _lib as L
    L.call("irx_set_option", b"large_tiles", request.param[0])
    L.call("irx_set_option", b"gemm_deep", request.param[1])
    L.call("irx_set_option", b"gemm_small", request.param[2])
    yield request.param
    L.call("irx_set_option", b"large_tiles", 1)
    L.call("irx_set_option", b"gemm_deep", 0)
    L.call("irx_set_option", b"gemm_small", 0)


@pytest.mark.parametrize("case", [
    # (N, Hin, Win, C0, C1, Cout, k, stride, pad, up_hw)
    (2, 64, 64, 320, 0, 320, 3, 1, 1, None),        # level-0 resnet conv  -> 128x320 tile
    (4, 32, 32, 1280, 640, 640, 3, 1, 1, None),     # up-block concat conv -> 128x320 tile
    (4, 16, 16, 1280, 0, 1280, 3, 1, 1, (32, 32)),  # Upsample2D conv      -> 256x256 tile
    (2, 63, 41, 256, 0, 512, 3, 2, 1, None),        # odd sizes, stride 2  -> 256x256 tile
    (3, 40, 40, 128, 128, 128, 1, 1, 0, None),      # 1x1 concat shortcut  -> 256x128 tile
    (2, 48, 48, 96, 32, 128, 3, 1, 1, None),        # channels % 32 only   -> ring path only (BK 32)
    (1, 16, 16, 1280, 1280, 1280, 3, 1, 1, None),   # long K, few tiles    -> split-K
])
@pytest.mark.parametrize("dt", DT16)
def test_conv_large(device, tiles, case, dt):
    N, H, W, C0, C1, Co, k, s, p, up = case
    x0 = _r(N, C0, H, W, seed=70)
    x1 = _r(N, C1, H, W, seed=71) if C1 else None
    w = _r(Co, C0 + C1, k, k, seed=72, scale=1 / math.sqrt((C0 + C1) * k * k))
    b = _r(Co, seed=73)
    res = None
    got = O.conv2d(_dev(x0.permute(0, 2, 3, 1), dt, device), w.to(dt).float(), b, stride=s, pad=(p, p),
                   x1=_dev(x1.permute(0, 2, 3, 1), dt, device) if C1 else None, up_hw=up)
    xin = torch.cat([_q(x0, dt)] + ([_q(x1, dt)] if C1 else []), 1)
    if up is not None:
        xin = F.interpolate(xin, size=up, mode="nearest")
    ref = F.conv2d(xin, _q(w, dt), b, stride=s, padding=p).permute(0, 2, 3, 1)
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("M,N,K,res,f32", [(8192, 2560, 320, False, False), (4096, 320, 1280, True, False),
                                           (5000, 640, 640, True, True), (4096, 512, 512, False, False),
                                           (6144, 384, 128, False, True)])
@pytest.mark.parametrize("dt", DT16)
def test_gemm_large(device, tiles, M, N, K, res, f32, dt):
    A = _r(M, K, seed=74)
    Bw = _r(N, K, seed=75, scale=1 / math.sqrt(K))
    bias = _r(N, seed=76)
    R = _r(M, N, seed=77) if res else None
    got = O.gemm(_dev(A, dt, device), _dev(Bw, dt, device), bias=bias.to(device),
                 residual=_dev(R, dt, device) if res else None, out_f32=f32)
    ref = _q(A, dt) @ _q(Bw, dt).T + bias + (_q(R, dt) if res else 0)
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("M,C", [(8192, 320), (4096, 640)])
def test_gemm_geglu_fused(device, M, C, dt):
    """ff.net.0.proj + GEGLU in one kernel (GEGLU64 weight order) vs Linear -> chunk -> h * gelu(g)."""
    from image_restoration_and_enhancement_amd import _lib as L
    from image_restoration_and_enhancement_amd.engine import geglu64_order
    A = _r(M, C, seed=80)
    Wt = _r(8 * C, C, seed=81, scale=1 / math.sqrt(C))
    bias = _r(8 * C, seed=82)
    perm = geglu64_order(8 * C)
    out = torch.empty(M, 4 * C, dtype=dt, device=device)
    a_d, w_d, b_d = _dev(A, dt, device), _dev(Wt[perm], dt, device), bias[perm].to(device).contiguous()
    L.call("irx_op_gemm_geglu", O.S(), O.DT[dt], M, 8 * C, C, O.P(a_d), O.P(w_d), O.P(b_d), O.P(out))
    pr = _q(A, dt) @ _q(Wt, dt).T + bias
    h, g = pr.chunk(2, dim=-1)
    assert O.rel_err(out, h * F.gelu(g)) < TOL[dt]


def test_gemm_large_batched(device, tiles):
    dt = torch.bfloat16
    b, M, N, K = 2, 4096, 256, 512
    A, Bw = _r(b, M, K, seed=78), _r(b, N, K, seed=79, scale=0.05)
    got = O.gemm(_dev(A, dt, device), _dev(Bw, dt, device), batch=b, out_f32=True)
    ref = torch.bmm(_q(A, dt), _q(Bw, dt).transpose(1, 2))
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("inkernel", [0, 1])
@pytest.mark.parametrize("M,N,K", [(4096, 1280, 1280), (1024, 1280, 2560), (4096, 640, 5120)])
def test_gemm_splitk_modes(device, inkernel, M, N, K):
    """Split-K shapes (few output tiles, long K) with the in-kernel last-arriver reduction and with the
    separate reduce kernel; bias + residual run in whichever epilogue finishes the tile."""
    from image_restoration_and_enhancement_amd import _lib as L
    dt = torch.bfloat16
    A = _r(M, K, seed=90)
    Bw = _r(N, K, seed=91, scale=1 / math.sqrt(K))
    bias, R = _r(N, seed=92), _r(M, N, seed=93)
    L.call("irx_set_option", b"splitk_inkernel", inkernel)
    try:
        for _ in range(2):   # second call: the arrival tickets must have been reset
            got = O.gemm(_dev(A, dt, device), _dev(Bw, dt, device), bias=bias.to(device), residual=_dev(R, dt, device))
            ref = _q(A, dt) @ _q(Bw, dt).T + bias + _q(R, dt)
            assert O.rel_err(got, ref) < TOL[dt]
    finally:
        L.call("irx_set_option", b"splitk_inkernel", 1)


# ------------------------------------------------------------------ halo conv tiles (whole image rows)
@pytest.fixture
def halo_forced():
    from image_restoration_and_enhancement_amd import _lib as L
    L.call("irx_set_option", b"conv_halo", 2)
    yield
    L.call("irx_set_option", b"conv_halo", 1)


@pytest.mark.parametrize("case", [
    # (N, H, W, C0, C1, Cout, rowadd+residual)
    (2, 64, 64, 320, 0, 320, False),    # UNet level-0 resnet conv, BN 160
    (1, 64, 64, 640, 320, 320, True),   # up-block concat conv + time-embedding row add + residual
    (1, 32, 32, 640, 0, 640, False),    # W 32: 8-row tiles
    (2, 16, 32, 128, 64, 160, True),    # W 32, 8-row tiles, concat
    (1, 8, 32, 64, 0, 160, False),      # W 32 over 8-row images: one tile per image
    (1, 8, 16, 64, 0, 160, False),      # W 16 needs 16-row images: falls back to the im2col walk
    (1, 16, 16, 64, 64, 160, False),    # W 16: one tile per image
])
@pytest.mark.parametrize("dt", DT16)
def test_conv_halo(device, halo_forced, case, dt):
    N, H, W, C0, C1, Co, extra = case
    x0 = _r(N, C0, H, W, seed=80)
    x1 = _r(N, C1, H, W, seed=81) if C1 else None
    w = _r(Co, C0 + C1, 3, 3, seed=82, scale=1 / math.sqrt((C0 + C1) * 9))
    b = _r(Co, seed=83)
    temb = _r(N, Co, seed=84) if extra else None
    res = _r(N, H, W, Co, seed=85) if extra else None
    got = O.conv2d(_dev(x0.permute(0, 2, 3, 1), dt, device), w.to(dt).float(), b,
                   x1=_dev(x1.permute(0, 2, 3, 1), dt, device) if C1 else None,
                   rowadd=temb.to(device).contiguous() if extra else None,
                   residual=_dev(res, dt, device) if extra else None)
    xin = torch.cat([_q(x0, dt)] + ([_q(x1, dt)] if C1 else []), 1)
    ref = F.conv2d(xin, _q(w, dt), b, padding=1)
    if extra:
        ref = ref + temb[:, :, None, None]
    ref = ref.permute(0, 2, 3, 1)
    if extra:
        ref = ref + _q(res, dt)
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("case", [
    # (N, H, W, C0, C1, Cout, rowadd+residual, forced): the UNet resnet shapes that take the fused path at
    # batch 16, and small forced-halo shapes (concat seam inside a group, W 16 / 32 / 64)
    (2, 64, 64, 320, 0, 320, False, False),
    (1, 64, 64, 640, 320, 320, True, False),   # up-block concat (groups of 30 straddle the seam) + temb + residual
    (1, 32, 32, 1280, 640, 640, True, False),
    (2, 16, 16, 1280, 0, 1280, True, False),   # 16x16 level: two K splits
    (2, 16, 32, 128, 64, 160, True, True),
    (1, 16, 16, 64, 64, 160, False, True),
])
@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("silu", [True, False])
def test_gn_conv3_fused_bit_exact(device, case, dt, silu):
    """GroupNorm(+SiLU) folded into the halo conv == group_norm op then conv op, bit for bit (same per-channel
    scale / shift, same gn_act, same rounding of the normalised operand); and both within tolerance of the
    fp32 CPU reference."""
    from image_restoration_and_enhancement_amd import _lib as L
    N, H, W, C0, C1, Co, extra, forced = case
    L.call("irx_set_option", b"gn_fuse", 1)     # (off by default: measured slower)
    if forced:
        L.call("irx_set_option", b"conv_halo", 2)
    try:
        x0 = _r(N, H, W, C0, seed=90, scale=2.0) + 0.7
        x1 = _r(N, H, W, C1, seed=91) - 0.3 if C1 else None
        g = _r(C0 + C1, seed=92) * 0.2 + 1.0
        bt = _r(C0 + C1, seed=93) * 0.1
        w = _r(Co, C0 + C1, 3, 3, seed=94, scale=1 / math.sqrt((C0 + C1) * 9))
        b = _r(Co, seed=95)
        temb = _r(N, Co, seed=96).to(device).contiguous() if extra else None
        res = _dev(_r(N, H, W, Co, seed=97), dt, device) if extra else None
        d0 = _dev(x0, dt, device)
        d1 = _dev(x1, dt, device) if C1 else None
        gd, bd = g.to(device).contiguous(), bt.to(device).contiguous()
        assert O.gn_conv3(d0, gd, bd, 1e-5, w, b, x1=d1, silu=silu, query=True)
        got = O.gn_conv3(d0, gd, bd, 1e-5, w, b, x1=d1, silu=silu, rowadd=temb, residual=res)
        n = O.group_norm(d0, gd, bd, 1e-5, 32, silu, x1=d1)
        ref_dev = O.conv2d(n, w.to(dt).float(), b, rowadd=temb, residual=res)   # the same halo walk, unfused
        torch.cuda.synchronize()
        assert torch.equal(got, ref_dev)
        xin = torch.cat([_q(x0, dt)] + ([_q(x1, dt)] if C1 else []), 3).permute(0, 3, 1, 2)
        nr = F.group_norm(xin, 32, g, bt, 1e-5)
        nr = _q(F.silu(nr) if silu else nr, dt)
        ref = F.conv2d(nr, _q(w, dt), b, padding=1)
        if extra:
            ref = ref + temb.cpu()[:, :, None, None]
        ref = ref.permute(0, 2, 3, 1)
        if extra:
            ref = ref + res.cpu().float()
        assert O.rel_err(got, ref) < TOL[dt]
    finally:
        L.call("irx_set_option", b"conv_halo", 1)
        L.call("irx_set_option", b"gn_fuse", 0)


def test_gn_conv3_not_fusable_is_refused(device):
    """Shapes off the halo path (the 8x8 level: rows narrower than 16 pixels) report fused = 0 and the launch
    fails loudly (the models fall back to a normalised copy + plain conv)."""
    from image_restoration_and_enhancement_amd import _lib as L
    dt = torch.bfloat16
    x = _dev(_r(2, 8, 8, 1280, seed=98), dt, device)
    g = torch.ones(1280, device=device)
    w = _r(1280, 1280, 3, 3, seed=99, scale=0.01)
    L.call("irx_set_option", b"gn_fuse", 1)
    try:
        assert not O.gn_conv3(x, g, g, 1e-5, w, None, query=True)
        with pytest.raises(L.IrxError):
            O.gn_conv3(x, g, g, 1e-5, w, None)
    finally:
        L.call("irx_set_option", b"gn_fuse", 0)


@pytest.mark.parametrize("case", [
    # (N, H, W, C0, C1, Cout, rowadd+residual): the UNet's 16x16-level convs, whose 128 halo tiles take two
    # K splits (whole 64-channel slabs, in-kernel reduction)
    (2, 16, 16, 1280, 0, 1280, True),
    (1, 16, 16, 1280, 1280, 1280, True),   # up-block concat
    (3, 16, 16, 640, 0, 1280, False),      # down2 resnet 0 conv1 (10 slabs)
])
@pytest.mark.parametrize("dt", DT16)
def test_conv_halo_split_k(device, case, dt):
    N, H, W, C0, C1, Co, extra = case
    x0 = _r(N, C0, H, W, seed=180)
    x1 = _r(N, C1, H, W, seed=181) if C1 else None
    w = _r(Co, C0 + C1, 3, 3, seed=182, scale=1 / math.sqrt((C0 + C1) * 9))
    b = _r(Co, seed=183)
    temb = _r(N, Co, seed=184) if extra else None
    res = _r(N, H, W, Co, seed=185) if extra else None
    got = O.conv2d(_dev(x0.permute(0, 2, 3, 1), dt, device), w.to(dt).float(), b,
                   x1=_dev(x1.permute(0, 2, 3, 1), dt, device) if C1 else None,
                   rowadd=temb.to(device).contiguous() if extra else None,
                   residual=_dev(res, dt, device) if extra else None)
    xin = torch.cat([_q(x0, dt)] + ([_q(x1, dt)] if C1 else []), 1)
    ref = F.conv2d(xin, _q(w, dt), b, padding=1)
    if extra:
        ref = ref + temb[:, :, None, None]
    ref = ref.permute(0, 2, 3, 1)
    if extra:
        ref = ref + _q(res, dt)
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("case", [
    # (N, H, W, C0, C1, Cout, forced): W 64 / 32 / 16, concat seams, the K-split 16x16 level (two in-kernel
    # reduced splits), batch-16 production shapes; `forced` = halo tiles although the grid is small
    (16, 64, 64, 320, 0, 320, False),
    (4, 64, 64, 640, 320, 320, False),
    (16, 32, 32, 640, 0, 640, False),
    (2, 16, 32, 128, 64, 160, True),
    (16, 16, 16, 1280, 1280, 1280, False),
    (1, 16, 16, 64, 64, 160, True),
])
@pytest.mark.parametrize("dt", DT16)
def test_conv_halo_pipelined_bit_exact(device, case, dt):
    """The software-pipelined halo main loop (option halo_pipe, default) issues the same MFMAs into every
    accumulator in the same order as the round-2 loop: outputs are identical bit for bit."""
    from image_restoration_and_enhancement_amd import _lib as L
    N, H, W, C0, C1, Co, forced = case
    x0 = _dev(_r(N, H, W, C0, seed=280), dt, device)
    x1 = _dev(_r(N, H, W, C1, seed=281), dt, device) if C1 else None
    w = _r(Co, C0 + C1, 3, 3, seed=282, scale=1 / math.sqrt((C0 + C1) * 9))
    b = _r(Co, seed=283)
    temb = _r(N, Co, seed=284).to(device).contiguous()
    res = _dev(_r(N, H, W, Co, seed=285), dt, device)
    L.call("irx_set_option", b"conv_halo", 2 if forced else 1)
    try:
        outs = []
        for pipe in (0, 1):
            L.call("irx_set_option", b"halo_pipe", pipe)
            outs.append(O.conv2d(x0, w.to(dt).float(), b, x1=x1, rowadd=temb, residual=res))
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1])
    finally:
        L.call("irx_set_option", b"halo_pipe", 1)
        L.call("irx_set_option", b"conv_halo", 1)


@pytest.mark.parametrize("M,N,K,res,conv", [
    (65536, 320, 320, True, None),        # K = 320 projections (256x320 tiles, BK 32)
    (16384, 640, 640, True, None),        # 32x32 level (128x320 / split-K)
    (4096, 1280, 1280, False, None),      # 16x16 level (128x128 tiles, BK 64, split-K)
    (1000, 256, 512, False, None),        # ragged M
    (65536, 1280, 320, False, "geglu"),   # GEGLU epilogue (256x256, BK 32)
    (16384, 5120, 640, False, None),      # 32x32-level FF projection shape (256x256 tiles)
    (4096, 2560, 1280, False, "geglu"),   # 16x16-level GEGLU (256x256, K = 1280)
    (0, 640, 0, False, (16, 16, 16, 1280, 640)),   # im2col conv: 16x16 level, 1280 -> 640
    (0, 320, 0, False, (8, 32, 32, 640, 320)),     # im2col conv: upsample-free 32x32, 640 -> 320 (1x1 shortcut)
])
@pytest.mark.parametrize("dt", DT16)
def test_gemm_pingpong_bit_exact(device, M, N, K, res, conv, dt):
    """The ping-pong main loops (option gemm_pp: 2 = the lean dense form on 256x256 tiles, the default; 1 = every tile)
    issue every accumulator's MFMAs in the round-2 order (32-deep K sub-steps, ascending; the same split-K
    boundaries): outputs identical bit for bit to the two-stage loop (0)."""
    from image_restoration_and_enhancement_amd import _lib as L
    from image_restoration_and_enhancement_amd.engine import geglu64_order
    outs = []
    try:
        for pp in (0, 1, 2):
            L.call("irx_set_option", b"gemm_pp", pp)
            if conv == "geglu":
                C = K
                A = _dev(_r(M, C, seed=300), dt, device)
                W = _r(8 * C, C, seed=301, scale=1 / math.sqrt(C))[geglu64_order(8 * C)]
                b = _r(8 * C, seed=302)
                out = torch.empty(M, 4 * C, dtype=dt, device=device)
                L.call("irx_op_gemm_geglu", O.S(), O.DT[dt], M, 8 * C, C, O.P(A), O.P(_dev(W, dt, device)),
                       O.P(b.to(device).contiguous()), O.P(out))
                outs.append(out)
            elif conv is not None:
                n, h, w, ci, co = conv
                x = _dev(_r(n, h, w, ci, seed=303), dt, device)
                k = 3 if h <= 16 else 1
                wt = _r(co, ci, k, k, seed=304, scale=1 / math.sqrt(ci * k * k))
                outs.append(O.conv2d(x, wt.to(dt).float(), _r(co, seed=305), pad=(k // 2, k // 2)))
            else:
                A = _dev(_r(M, K, seed=306), dt, device)
                Bw = _dev(_r(N, K, seed=307, scale=1 / math.sqrt(K)), dt, device)
                r = _dev(_r(M, N, seed=308), dt, device) if res else None
                outs.append(O.gemm(A, Bw, bias=_r(N, seed=309).to(device).contiguous(), residual=r))
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1])
        assert torch.equal(outs[0], outs[2])
    finally:
        L.call("irx_set_option", b"gemm_pp", 2)


@pytest.mark.parametrize("B,L", [(2, 256), (1, 333), (2, 1024), (1, 77)])
@pytest.mark.parametrize("dt", DT16)
def test_attention_d512_flash(device, dt, B, L):
    """The VAE mid-block's single d = 512 head through the wide flash kernel (attnw): ragged lengths, fused
    q|k|v rows (row stride 3C), vs a PyTorch fp32 softmax attention on the same rounded inputs."""
    C = 512
    qkv = _r(B, L, 3 * C, seed=190) * 0.5
    d = _dev(qkv, dt, device)
    got = O.attention(d[..., :C], d[..., C:2 * C], d[..., 2 * C:], 1)
    q, k, v = (_q(qkv[..., i * C:(i + 1) * C], dt) for i in range(3))
    ref = torch.softmax(q @ k.transpose(1, 2) / math.sqrt(C), -1) @ v
    assert O.rel_err(got, ref) < TOL[dt] * 2


def test_gemm_splitk_two_streams(device):
    """Two streams running in-kernel split-K GEMMs concurrently (the arrival tickets were one
    process-global array): each stream's results equal a single-stream run bit for bit."""
    from image_restoration_and_enhancement_amd import _lib as L
    dt = torch.bfloat16
    shapes = [(4096, 1280, 1280), (1024, 1280, 2560)]
    ins = [(_dev(_r(M, K, seed=94 + i), dt, device), _dev(_r(N, K, seed=96 + i, scale=1 / math.sqrt(K)), dt, device))
           for i, (M, N, K) in enumerate(shapes)]
    L.call("irx_set_option", b"splitk_inkernel", 1)
    want = [O.gemm(a, b) for a, b in ins]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [[], []]
    for _ in range(8):
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                outs[i].append(O.gemm(*ins[i]))
    torch.cuda.synchronize()
    for i in range(2):
        for o in outs[i]:
            assert torch.equal(o, want[i])


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("B,Lq,Lk,C,heads", [(2, 256, 256, 320, 8), (1, 333, 190, 640, 8), (2, 130, 77, 1280, 8)])
def test_attention_v3_vs_v2_and_head_major(device, dt, B, Lq, Lk, C, heads):
    """attn3 with heads laid out [b][h][L][d] (head strides) equals the interleaved layout bit for bit, and
    (bf16) agrees with the round-1 kernel within the bf16 bound."""
    from image_restoration_and_enhancement_amd import _lib as L
    d = C // heads
    q, k, v = _r(B, Lq, C, seed=63), _r(B, Lk, C, seed=64), _r(B, Lk, C, seed=65)
    qd, kd, vd = _dev(q, dt, device), _dev(k, dt, device), _dev(v, dt, device)
    got = O.attention(qd, kd, vd, heads)
    hm = [x.view(B, x.shape[1], heads, d).transpose(1, 2).contiguous() for x in (qd, kd, vd)]
    o = torch.empty(B, heads, Lq, d, dtype=dt, device=device)
    L.call("irx_op_attention_hm", O.S(), O.DT[dt], B, heads, Lq, Lk, d, O.P(hm[0]), O.P(hm[1]), O.P(hm[2]),
           O.P(o), 1.0 / math.sqrt(d))
    assert torch.equal(o.transpose(1, 2).reshape(B, Lq, C), got)
    ref = O.ref_attention(_q(q, dt), _q(k, dt), _q(v, dt), heads)
    assert O.rel_err(got, ref) < 2 * TOL[dt]


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("B,Lq,Lk,C", [(16, 4096, 77, 320), (16, 3600, 77, 320), (16, 4000, 128, 320),
                                       (16, 2048, 20, 640), (32, 1024, 77, 1280)])
def test_attention_resident_kv(device, dt, B, Lq, Lk, C):
    """Cross-attention with K/V resident in LDS (Lk <= 128; qrep query groups per block, some blocks' last
    groups entirely past Lq) equals the streamed attn3 kernel (irx_set_option("attn_qrep", 0)) bit for bit."""
    from image_restoration_and_enhancement_amd import _lib as L
    q, k, v = _r(B, Lq, C, seed=66), _r(B, Lk, C, seed=67), _r(B, Lk, C, seed=68)
    qd, kd, vd = _dev(q, dt, device), _dev(k, dt, device), _dev(v, dt, device)
    got = O.attention(qd, kd, vd, 8)
    L.call("irx_set_option", b"attn_qrep", 0)
    try:
        want = O.attention(qd, kd, vd, 8)
    finally:
        L.call("irx_set_option", b"attn_qrep", 1)
    assert torch.equal(got, want)
    ref = O.ref_attention(_q(q[:2], dt), _q(k[:2], dt), _q(v[:2], dt), 8)
    assert O.rel_err(got[:2], ref) < 2 * TOL[dt]


def _with_sk(v, fn):
    # v = 3: every K = 320 shape on gemm_sk (the default takes only the GEGLU projection there)
    from image_restoration_and_enhancement_amd import _lib as L
    L.call("irx_set_option", b"gemm_sk", v)
    try:
        out = fn()
        torch.cuda.synchronize()
        return out
    finally:
        L.call("irx_set_option", b"gemm_sk", 1)


@pytest.mark.parametrize("M,N,res", [(5000, 320, True), (65536, 960, False), (777, 640, True), (64, 320, False),
                                     (16384, 2560, False),
                                     # M = 1 (mod the tile): a last tile with a single valid row
                                     (1025, 320, True), (4097, 960, False)])
@pytest.mark.parametrize("dt", DT16)
def test_gemm_sk(device, M, N, res, dt):
    """K = 320 streaming kernel (gemm_sk.hip: B slice in registers, A ring, lane-local epilogue) vs fp32, and
    bit for bit vs the large-tile kernel (same MFMA, same k order, same epilogue arithmetic)."""
    K = 320
    A = _r(M, K, seed=90)
    Bw = _r(N, K, seed=91, scale=1 / math.sqrt(K))
    bias = _r(N, seed=92)
    R = _r(M, N, seed=93) if res else None
    a_d, b_d, r_d = _dev(A, dt, device), _dev(Bw, dt, device), (_dev(R, dt, device) if res else None)
    run = lambda: O.gemm(a_d, b_d, bias=bias.to(device), residual=r_d, guard_rows=8)       # noqa: E731
    sk, lt = _with_sk(3, run), _with_sk(0, run)
    ref = _q(A, dt) @ _q(Bw, dt).T + bias + (_q(R, dt) if res else 0)
    assert O.rel_err(sk, ref) < TOL[dt]
    _same_as_large_tile(sk, lt, dt)


def _same_as_large_tile(sk, lt, dt):
    # bit for bit in both dtypes: the two kernels' MFMA products are operand-order symmetric (scripts/
    # mfma_swap_check.hip: 0 of 2^20 elements differ, f16 and bf16) and every fp32 -> fp16 conversion goes through
    # f16_src (irx_common.h), so hipcc cannot fuse an epilogue FMA into a single-rounding v_fma_mixlo_f16 at some
    # call sites and not others — the round-3 fp16 residual mismatch
    assert torch.equal(sk, lt)


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("M", [8192, 1000, 1025])
def test_gemm_sk_geglu(device, M, dt):
    """GEGLU feed-forward projection at K = 320 on the streaming kernel: vs fp32 and bit for bit vs the
    large-tile kernel's fused GEGLU epilogue."""
    from image_restoration_and_enhancement_amd import _lib as L
    from image_restoration_and_enhancement_amd.engine import geglu64_order
    C = 320
    A = _r(M, C, seed=94)
    Wt = _r(8 * C, C, seed=95, scale=1 / math.sqrt(C))
    bias = _r(8 * C, seed=96)
    perm = geglu64_order(8 * C)
    a_d, w_d, b_d = _dev(A, dt, device), _dev(Wt[perm], dt, device), bias[perm].to(device).contiguous()

    def run():
        buf = torch.full((M + 8, 4 * C), 1234.0, dtype=dt, device=device)   # 8 guard rows: no write past M
        L.call("irx_op_gemm_geglu", O.S(), O.DT[dt], M, 8 * C, C, O.P(a_d), O.P(w_d), O.P(b_d), O.P(buf))
        torch.cuda.synchronize()
        assert bool((buf[M:] == 1234.0).all()), "GEGLU GEMM wrote past its last output row"
        return buf[:M]
    sk = _with_sk(1, run)
    pr = _q(A, dt) @ _q(Wt, dt).T + bias
    h, g = pr.chunk(2, dim=-1)
    assert O.rel_err(sk, h * F.gelu(g)) < TOL[dt]
    _same_as_large_tile(sk, _with_sk(0, run), dt)


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("B,Lq,Lk", [(2, 1024, 1024), (1, 333, 190), (1, 64, 129), (2, 4096, 4096)])
def test_attention_prefetch_d40_bit_exact(device, dt, B, Lq, Lk):
    """attn3 with whole-tile K / V fragment prefetch (option attn_pf) issues the same MFMAs on the same operands in the
    same order as the default kernel — only the LDS reads move — so the outputs are identical bit for bit."""
    from image_restoration_and_enhancement_amd import _lib as L
    C, heads = 320, 8
    q, k, v = _r(B, Lq, C, seed=73) * 2, _r(B, Lk, C, seed=74) * 2, _r(B, Lk, C, seed=75)
    qd, kd, vd = _dev(q, dt, device), _dev(k, dt, device), _dev(v, dt, device)
    with L.option(attn_pf=1, attn_q2=0):
        got = O.attention(qd, kd, vd, heads)
    with L.option(attn_pf=0, attn_q2=0):
        base = O.attention(qd, kd, vd, heads)
    torch.cuda.synchronize()
    assert torch.equal(got, base)


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("B,Lq,Lk", [(2, 256, 256), (1, 64, 64), (2, 256, 77), (1, 64, 77), (1, 333, 190), (1, 100, 128)])
def test_attention_prefetch_d160_bit_exact(device, dt, B, Lq, Lk):
    """d = 160 (the UNet's 16x16 / 8x8 levels, one wave per SIMD) with the whole-tile fragment prefetch (option
    attn_pf160), streamed (Lk > 128) and resident K/V (Lk <= 128, the 77 text tokens): the same MFMAs on the same
    operands in the same order as without it — identical bit for bit."""
    from image_restoration_and_enhancement_amd import _lib as L
    C, heads = 1280, 8
    q, k, v = _r(B, Lq, C, seed=79) * 2, _r(B, Lk, C, seed=80) * 2, _r(B, Lk, C, seed=81)
    qd, kd, vd = _dev(q, dt, device), _dev(k, dt, device), _dev(v, dt, device)
    with L.option(attn_pf160=1):
        got = O.attention(qd, kd, vd, heads)
    with L.option(attn_pf160=0):
        base = O.attention(qd, kd, vd, heads)
    torch.cuda.synchronize()
    assert torch.equal(got, base)
    assert O.rel_err(got, O.ref_attention(_q(q, dt), _q(k, dt), _q(v, dt), heads, False)) < TOL[dt] * 2


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("B,Lq,Lk", [(2, 1024, 1024), (1, 333, 190), (1, 64, 129), (2, 130, 300)])
def test_attention_prefetch_d80_bit_exact(device, dt, B, Lq, Lk):
    """d = 80 self-attention (the UNet's 32x32 level) with the whole-tile fragment prefetch at 2 waves / SIMD (option
    attn_pf80, default 2): the same MFMAs on the same operands in the same order as the kernel without it."""
    from image_restoration_and_enhancement_amd import _lib as L
    C, heads = 640, 8
    q, k, v = _r(B, Lq, C, seed=82) * 2, _r(B, Lk, C, seed=83) * 2, _r(B, Lk, C, seed=84)
    qd, kd, vd = _dev(q, dt, device), _dev(k, dt, device), _dev(v, dt, device)
    with L.option(attn_pf80=2):
        got = O.attention(qd, kd, vd, heads)
    with L.option(attn_pf80=0):
        base = O.attention(qd, kd, vd, heads)
    torch.cuda.synchronize()
    assert torch.equal(got, base)
    assert O.rel_err(got, O.ref_attention(_q(q, dt), _q(k, dt), _q(v, dt), heads, False)) < TOL[dt] * 2


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("B,Lq,Lk", [(2, 1024, 1024), (1, 333, 190), (1, 64, 129), (2, 4096, 4096)])
def test_attention_two_query_groups_d40_bit_exact(device, dt, B, Lq, Lk):
    """attn3q (option attn_q2: two 32-query groups per wave sharing every K / V^T fragment read) runs each group's
    arithmetic exactly as attn3 does (same MFMA order per accumulator, the deferred-max decision over the group's own
    queries): identical outputs bit for bit, ragged query and key counts included."""
    from image_restoration_and_enhancement_amd import _lib as L
    C, heads = 320, 8
    q, k, v = _r(B, Lq, C, seed=76) * 2, _r(B, Lk, C, seed=77) * 2, _r(B, Lk, C, seed=78)
    qd, kd, vd = _dev(q, dt, device), _dev(k, dt, device), _dev(v, dt, device)
    with L.option(attn_q2=1):
        got = O.attention(qd, kd, vd, heads)
    with L.option(attn_q2=0, attn_pf=0):
        base = O.attention(qd, kd, vd, heads)
    torch.cuda.synchronize()
    assert torch.equal(got, base)


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("N,H,W,C0,C1,Co,res", [
    (2, 64, 64, 320, 1280, 320, True),     # proj_out ∘ ff.net.2 at 64^2 (the ff chain, + residual)
    (2, 32, 32, 640, 2560, 640, True),     # ... at 32^2
    (4, 16, 16, 1280, 5120, 1280, True),   # ... at 16^2 (split-K)
    (2, 32, 32, 1280, 640, 640, False),    # up-block resnet shortcut over the skip concat
    (2, 64, 64, 640, 0, 320, False),       # single-source 1x1
    (3, 7, 9, 320, 1280, 320, True),       # ragged rows (M = 189: a partial tile)
])
def test_conv1x1_two_source_dense(device, dt, N, H, W, C0, C1, Co, res):
    """1x1 convs over a channel concat as a dense GEMM with a second A source from K = C0 (option conv1x1_dense,
    default; conv1x1_as_dense) vs PyTorch fp32 on the same rounded operands, and vs the im2col conv path (option
    off): the same per-output K order, so equal up to a different split choice."""
    from image_restoration_and_enhancement_amd import _lib as L
    x0 = _r(N, C0, H, W, seed=90)
    x1 = _r(N, C1, H, W, seed=91) if C1 else None
    w = _r(Co, C0 + C1, 1, 1, seed=92, scale=1 / math.sqrt(C0 + C1))
    b = _r(Co, seed=93)
    r = _r(N, H, W, Co, seed=94) if res else None
    d0 = _dev(x0.permute(0, 2, 3, 1), dt, device)
    d1 = _dev(x1.permute(0, 2, 3, 1), dt, device) if C1 else None
    dr = _dev(r, dt, device) if res else None
    outs = []
    for v in (1, 0):
        with L.option(conv1x1_dense=v):
            outs.append(O.conv2d(d0, w.to(dt).float(), b, pad=(0, 0), x1=d1, residual=dr))
    torch.cuda.synchronize()
    xin = torch.cat([_q(x0, dt)] + ([_q(x1, dt)] if C1 else []), 1)
    ref = F.conv2d(xin, _q(w, dt), b).permute(0, 2, 3, 1)
    if res:
        ref = ref + _q(r, dt)
    assert torch.isfinite(outs[0].float()).all()
    assert O.rel_err(outs[0], ref) < TOL[dt]
    assert O.rel_err(outs[0], outs[1].float()) < 2e-3


# ------------------------------------------------------------------ strip halo tiles (8 rows x 32 columns)
@pytest.mark.parametrize("case", [
    # (N, H, W, C0, C1, Cout, rowadd+residual): the VAE's widths (BN 128) at W > 64, the 768^2 UNet's 96-wide
    # level (BN 160), a concat, ragged strip counts (W 96 / 160), BN 128 on whole-row tiles (W 64)
    (1, 16, 128, 128, 0, 128, True),
    (2, 8, 256, 256, 0, 256, False),
    (1, 8, 512, 128, 0, 128, True),
    (1, 16, 96, 320, 0, 320, True),
    (1, 8, 160, 64, 64, 128, True),
    (1, 24, 64, 512, 0, 512, True),
])
@pytest.mark.parametrize("dt", DT16)
def test_conv_halo_strip(device, halo_forced, case, dt):
    """Strip halo tiles (HALO == 5, option halo_strip) and the 128-wide halo tiles vs the fp32 CPU conv: the
    neighbouring columns of every strip, the image's left / right / top / bottom zero padding, the epilogue's
    row -> NHWC pixel mapping for the store, the residual and the row add."""
    N, H, W, C0, C1, Co, extra = case
    x0 = _r(N, C0, H, W, seed=380)
    x1 = _r(N, C1, H, W, seed=381) if C1 else None
    w = _r(Co, C0 + C1, 3, 3, seed=382, scale=1 / math.sqrt((C0 + C1) * 9))
    b = _r(Co, seed=383)
    temb = _r(N, Co, seed=384) if extra else None
    res = _r(N, H, W, Co, seed=385) if extra else None
    got = O.conv2d(_dev(x0.permute(0, 2, 3, 1), dt, device), w.to(dt).float(), b,
                   x1=_dev(x1.permute(0, 2, 3, 1), dt, device) if C1 else None,
                   rowadd=temb.to(device).contiguous() if extra else None,
                   residual=_dev(res, dt, device) if extra else None)
    xin = torch.cat([_q(x0, dt)] + ([_q(x1, dt)] if C1 else []), 1)
    ref = F.conv2d(xin, _q(w, dt), b, padding=1)
    if extra:
        ref = ref + temb[:, :, None, None]
    ref = ref.permute(0, 2, 3, 1)
    if extra:
        ref = ref + _q(res, dt)
    assert O.rel_err(got, ref) < TOL[dt]
    # every pixel, not only the norm: the strip seams and the image border are where a mapping slip would show
    err = (got.float().cpu() - ref).abs().amax(dim=-1)
    assert float(err.max()) < 0.05 * float(ref.abs().max()), err.argmax()


@pytest.mark.parametrize("case", [
    # (N, H, W, C0, C1, Cout): whole-row halo shapes also run as strips (halo_strip 2): same MFMAs per accumulator
    (2, 64, 64, 320, 0, 320),
    (1, 32, 64, 128, 0, 128),
    (2, 16, 32, 128, 64, 160),
    (16, 32, 32, 640, 0, 640),
])
@pytest.mark.parametrize("dt", DT16)
def test_conv_halo_strip_equals_rows_bit_exact(device, case, dt):
    """The strip tiles accumulate every output over the same (slab, tap, sub-step) order as the whole-row tiles, so
    at W <= 64 forcing strips (option halo_strip 2) reproduces the row tiles bit for bit, residual and row add
    included: the strip halo (neighbouring columns, zero borders) and the row mapping are exact."""
    from image_restoration_and_enhancement_amd import _lib as L
    N, H, W, C0, C1, Co = case
    x0 = _dev(_r(N, H, W, C0, seed=480), dt, device)
    x1 = _dev(_r(N, H, W, C1, seed=481), dt, device) if C1 else None
    w = _r(Co, C0 + C1, 3, 3, seed=482, scale=1 / math.sqrt((C0 + C1) * 9))
    b = _r(Co, seed=483)
    temb = _r(N, Co, seed=484).to(device).contiguous()
    res = _dev(_r(N, H, W, Co, seed=485), dt, device)
    L.call("irx_set_option", b"conv_halo", 2)
    try:
        outs = []
        for strip in (1, 2):
            L.call("irx_set_option", b"halo_strip", strip)
            outs.append(O.conv2d(x0, w.to(dt).float(), b, x1=x1, rowadd=temb, residual=res))
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1])
    finally:
        L.call("irx_set_option", b"halo_strip", 1)
        L.call("irx_set_option", b"conv_halo", 1)


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("N,H,W,C0,C1,Co", [
    (16, 64, 64, 320, 1280, 320),     # proj_out o ff.net.2 at 64^2, batch 16: 256 x 320 tiles
    (16, 32, 32, 640, 2560, 640),     # ... at 32^2: 128 x 320 tiles
    (16, 16, 16, 1280, 5120, 1280),   # ... at 16^2: 128 x 320 tiles, two in-kernel K splits
    (2, 32, 32, 640, 2560, 640),
])
def test_chain_pingpong_bit_exact(device, dt, N, H, W, C0, C1, Co):
    """The two-source 1x1 chains on the lean dense ping-pong loop (option gemm_pp_chain, default) run the same 32-deep
    MFMA steps in the same K order into every accumulator as the two-stage loop: identical outputs, residual and the
    second A source's switch at K = C0 included."""
    from image_restoration_and_enhancement_amd import _lib as L
    d0 = _dev(_r(N, H, W, C0, seed=190), dt, device)
    d1 = _dev(_r(N, H, W, C1, seed=191), dt, device)
    w = _r(Co, C0 + C1, 1, 1, seed=192, scale=1 / math.sqrt(C0 + C1))
    b = _r(Co, seed=193)
    dr = _dev(_r(N, H, W, Co, seed=194), dt, device)
    outs = []
    for v in (1, 0):
        with L.option(gemm_pp_chain=v):
            outs.append(O.conv2d(d0, w.to(dt).float(), b, pad=(0, 0), x1=d1, residual=dr))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("case", [
    # (N, C0, C1, Cout, rowadd+residual): the UNet's 8x8-level convs (four images per halo tile, K splits + the
    # reduce kernel), a partial last tile (N % 4 != 0), the up-block concat
    (16, 1280, 0, 1280, True),
    (5, 1280, 0, 1280, False),
    (3, 1280, 1280, 1280, True),
    (16, 640, 640, 1280, True),
])
@pytest.mark.parametrize("dt", DT16)
def test_conv_halo_8x8_images(device, case, dt):
    """3x3 convs over 8x8 images on four-image halo tiles (HALO == 8, option halo_mi): each image's halo block with its
    own zero pad rows, split-K partials reduced by the separate kernel; vs the fp32 CPU conv, and vs the im2col walk
    (halo_mi 0) within the reassociation of a different K order."""
    from image_restoration_and_enhancement_amd import _lib as L
    N, C0, C1, Co, extra = case
    x0 = _r(N, C0, 8, 8, seed=580)
    x1 = _r(N, C1, 8, 8, seed=581) if C1 else None
    w = _r(Co, C0 + C1, 3, 3, seed=582, scale=1 / math.sqrt((C0 + C1) * 9))
    b = _r(Co, seed=583)
    temb = _r(N, Co, seed=584) if extra else None
    res = _r(N, 8, 8, Co, seed=585) if extra else None
    args = dict(x1=_dev(x1.permute(0, 2, 3, 1), dt, device) if C1 else None,
                rowadd=temb.to(device).contiguous() if extra else None,
                residual=_dev(res, dt, device) if extra else None)
    d0 = _dev(x0.permute(0, 2, 3, 1), dt, device)
    got = O.conv2d(d0, w.to(dt).float(), b, **args)
    with L.option(halo_mi=0):
        walk = O.conv2d(d0, w.to(dt).float(), b, **args)
    xin = torch.cat([_q(x0, dt)] + ([_q(x1, dt)] if C1 else []), 1)
    ref = F.conv2d(xin, _q(w, dt), b, padding=1)
    if extra:
        ref = ref + temb[:, :, None, None]
    ref = ref.permute(0, 2, 3, 1)
    if extra:
        ref = ref + _q(res, dt)
    assert O.rel_err(got, ref) < TOL[dt]
    # (two K orders, each rounded once to the 16-bit output: about one bf16 ulp apart on some elements)
    assert O.rel_err(got, walk.float()) < (8e-3 if dt == torch.bfloat16 else 2e-3)
    err = (got.float().cpu() - ref).abs().amax(dim=-1)   # every pixel: image seams and pad rows
    assert float(err.max()) < 0.05 * float(ref.abs().max()), err.argmax()


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("M,N,K,act,res", [
    (154, 768, 3072, 0, True),    # CLIP fc2 (+ residual): 8 K splits
    (16, 1280, 1280, 1, False),   # time embedding linear_2 (+ SiLU): 4 K splits
    (154, 768, 768, 0, True),     # K < 1024: no split (the plain 4-wave kernel)
])
def test_small_m_splitk(device, dt, M, N, K, act, res):
    """Small-M, long-K GEMMs on the 4-wave kernel in K splits + the split-K reduce kernel (option small_splitk):
    vs PyTorch fp32 on the same rounded operands, vs the unsplit kernel within fp32 reassociation, and batch-invariant
    (the split depends on N and K only: the first rows of an M-row call equal a 6-row call bit for bit)."""
    from image_restoration_and_enhancement_amd import _lib as L
    A = _r(M, K, seed=700)
    Bw = _r(N, K, seed=701, scale=1 / math.sqrt(K))
    bias, R = _r(N, seed=702), _r(M, N, seed=703)
    dA, dB = _dev(A, dt, device), _dev(Bw, dt, device)
    dR = _dev(R, dt, device) if res else None
    got = O.gemm(dA, dB, bias=bias.to(device), act=act, residual=dR)
    with L.option(small_splitk=0):
        plain = O.gemm(dA, dB, bias=bias.to(device), act=act, residual=dR)
    six = O.gemm(dA[:6].contiguous(), dB, bias=bias.to(device), act=act, residual=dR[:6].contiguous() if res else None)
    torch.cuda.synchronize()
    ref = _q(A, dt) @ _q(Bw, dt).T + bias
    if act == 1:
        ref = F.silu(ref)
    if res:
        ref = ref + _q(R, dt)
    assert O.rel_err(got, ref) < TOL[dt]
    assert O.rel_err(got, plain.float()) < (8e-3 if dt == torch.bfloat16 else 2e-3)
    assert torch.equal(got[:6], six)
