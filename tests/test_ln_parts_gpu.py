"""LayerNorm statistics from the producer's epilogue (VERDICT r3 "next" #1b; GemmArgs::ln_out / ln_part).

The diffusers BasicTransformerBlock the reference runs (src/inference.py:486 -> UNet2DConditionModel ->
Transformer2DModel) normalises its residual stream h three times (norm1 / norm2 / norm3) right after a projection
wrote it (proj_in, attn1.to_out + h, attn2.to_out + h).  The 16-bit engines fold each LayerNorm into the following
projection (ln_fold); with ln_parts the projection that writes h also emits, per row and 320-column group, the
(mean, M2) of the values it stored, and the folded consumer merges them — no statistics pass over h.

Checked here through the C ABI (irx_op_gemm_ln_out / irx_op_gemm_ln_fold):
  * the producer's outputs are bit-identical with and without the emission, and its partials equal the fp64
    two-pass statistics of the stored rows (|d mean| <= 1e-5 of the row's max |x|, M2 relative 5e-5: the epilogue
    makes one fp32 pass of sums shifted by the row's first value);
  * the folded consumer fed the partials matches PyTorch fp32 LayerNorm + projection within the dtype bound, and
    the consumer fed the same statistics as (rstd, rstd * mean) rows within one ulp of its output;
  * GEGLU consumers (K = 320 streaming kernel, K = 640 large tiles with two partials per row);
  * the folded fp16 GEGLU projection is batch invariant at the op level (rows of 16 images vs 1 + 15 / 3 + 13 /
    7 + 9, with the 8x8-level row count of 64 per image — the shape of the round-3 fp16 divergence, whose cause was
    hipcc fusing the epilogue FMA and the fp16 conversion into v_fma_mixlo_f16 at some unrolled sites only).
"""
import math

import pytest
import torch
import torch.nn.functional as F

from image_restoration_and_enhancement_amd import _lib as L
from image_restoration_and_enhancement_amd.engine import geglu64_order
from tests import opref as O

pytestmark = pytest.mark.gpu

DT16 = [torch.bfloat16, torch.float16]
TOL = {torch.bfloat16: 2e-2, torch.float16: 5e-3}
ULP = {torch.bfloat16: 2.0 ** -7, torch.float16: 2.0 ** -10}


def _r(*shape, seed=0, scale=1.0, shift=0.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale + shift


def _dev(x, dt, device):
    return x.to(dt).to(device).contiguous()


def produce(A, W, bias, R, dt, device, final_rs=False):
    M, K = A.shape
    N = W.shape[0]
    C = torch.empty(M, N, dtype=dt, device=device)
    parts = torch.full((M, N // 320, 2), float("nan"), dtype=torch.float32, device=device)
    L.call("irx_op_gemm_ln_out", O.S(), O.DT[dt], M, N, K, O.P(A), O.P(W), O.P(bias), O.P(R), O.P(C), O.P(parts),
           int(final_rs), 1e-5)
    return C, parts


def two_pass(x):   # fp64 (mean, M2) per 320-column group
    g = x.double().view(x.shape[0], -1, 320)
    mean = g.mean(-1)
    return mean, ((g - mean[..., None]) ** 2).sum(-1)


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("M,C,res", [(8192, 320, False), (8192, 320, True), (16384, 640, True), (16384, 640, False)])
def test_ln_out_partials(device, dt, M, C, res):
    A = _dev(_r(M, C, seed=1), dt, device)
    W = _dev(_r(C, C, seed=2, scale=1 / math.sqrt(C)), dt, device)
    bias = _r(C, seed=3, scale=0.5).to(device)
    R = _dev(_r(M, C, seed=4, shift=0.7), dt, device) if res else None
    out, parts = produce(A, W, bias, R, dt, device)
    plain = O.gemm(A, W, bias=bias, residual=R)
    torch.cuda.synchronize()
    assert torch.equal(out, plain)                      # the emission does not change what is stored
    mean, m2 = two_pass(out.float())
    scale = out.float().abs().amax(-1, keepdim=True).double()
    assert torch.isfinite(parts).all()
    assert float(((parts[..., 0].double() - mean).abs() / scale).max()) < 1e-5
    assert float(((parts[..., 1].double() - m2).abs() / m2).max()) < 5e-5     # (one shifted fp32 pass)


def _ln_fold_operands(C, N, seed, geglu):
    W = _r(N, C, seed=seed, scale=1 / math.sqrt(C))
    b = _r(N, seed=seed + 1, scale=0.3)
    gamma = _r(C, seed=seed + 2, scale=0.2, shift=1.0)
    beta = _r(C, seed=seed + 3, scale=0.1)
    return W, b, gamma, beta


def _fold(W, b, gamma, beta, dt, device, geglu):
    perm = geglu64_order(W.shape[0]) if geglu else torch.arange(W.shape[0])
    Wg = (W * gamma)[perm].to(dt)                       # W diag(gamma) as stored
    u = Wg.double().sum(1).float()                      # row sums of the stored matrix
    v = (W.double() @ beta.double() + b.double()).float()[perm]
    return Wg.to(device).contiguous(), u.to(device).contiguous(), v.to(device).contiguous()


def fold_gemm(x, Wg, u, v, dt, device, rs=None, parts=None, T=0, geglu=False):
    M, K = x.shape
    N = Wg.shape[0]
    out = torch.empty(M, N // 2 if geglu else N, dtype=dt, device=device)
    L.call("irx_op_gemm_ln_fold", O.S(), O.DT[dt], M, N, K, O.P(x), O.P(Wg), O.P(u), O.P(v), O.P(rs), O.P(parts),
           T, int(geglu), O.P(out))
    return out


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("N,geglu", [(960, False), (320, False), (2560, True)])
def test_ln_fold_from_producer_rs(device, dt, N, geglu):
    """The engine's form at C = 320: the producer writes each row's final (rstd, rstd * mean) (final_rs), the folded
    consumer takes it as its ln_rs — matching the statistics of the stored rows (fp64) and PyTorch LayerNorm +
    projection."""
    M, C = 8192, 320
    A = _dev(_r(M, C, seed=40), dt, device)
    Wp = _dev(_r(C, C, seed=41, scale=1 / math.sqrt(C)), dt, device)
    h, rs = produce(A, Wp, _r(C, seed=42).to(device), _dev(_r(M, C, seed=43, shift=0.5), dt, device), dt, device,
                    final_rs=True)
    rs = rs.view(M, 2).contiguous()
    hd = h.double()
    mean = hd.mean(-1)
    rstd = torch.rsqrt(((hd - mean[:, None]) ** 2).mean(-1) + 1e-5)
    assert float(((rs[:, 0].double() - rstd).abs() / rstd).max()) < 2e-5
    assert float(((rs[:, 1].double() - rstd * mean).abs() / (rstd * hd.abs().amax(-1))).max()) < 2e-5
    W, b, gamma, beta = _ln_fold_operands(C, N, 44, geglu)
    Wg, u, v = _fold(W, b, gamma, beta, dt, device, geglu)
    got = fold_gemm(h, Wg, u, v, dt, device, rs=rs, geglu=geglu)
    torch.cuda.synchronize()
    ref = F.layer_norm(h.float().cpu(), (C,), gamma, beta, 1e-5) @ W.t() + b
    if geglu:
        hv, gt = ref.chunk(2, dim=-1)
        ref = hv * F.gelu(gt)
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("M,C,N,geglu", [(8192, 320, 960, False), (8192, 320, 2560, True), (16384, 640, 640, False),
                                          (16384, 640, 5120, True), (16384, 640, 1920, False)])
def test_ln_fold_from_partials(device, dt, M, C, N, geglu):
    # producer: h = A Wp^T + bp + R (the residual stream), then LN(h) -> projection from its partials
    A = _dev(_r(M, C, seed=10), dt, device)
    Wp = _dev(_r(C, C, seed=11, scale=1 / math.sqrt(C)), dt, device)
    h, parts = produce(A, Wp, _r(C, seed=12).to(device), _dev(_r(M, C, seed=13, shift=0.5), dt, device), dt, device)
    W, b, gamma, beta = _ln_fold_operands(C, N, 20, geglu)
    Wg, u, v = _fold(W, b, gamma, beta, dt, device, geglu)
    got = fold_gemm(h, Wg, u, v, dt, device, parts=parts, T=C // 320, geglu=geglu)
    # the same statistics handed over as rows (rstd, rstd * mean), computed in fp32 from the partials the way
    # the epilogue merges them
    pm, pq = parts[..., 0].double(), parts[..., 1].double()
    mean = pm.mean(-1)
    m2 = (pq + 320.0 * (pm - mean[:, None]) ** 2).sum(-1)
    rstd = torch.rsqrt(m2 / C + 1e-5)
    mean, rstd = mean.float(), rstd.float()
    rs = torch.stack([rstd, rstd * mean], -1).contiguous()
    via_rs = fold_gemm(h, Wg, u, v, dt, device, rs=rs, geglu=geglu)
    torch.cuda.synchronize()
    d = (got.float() - via_rs.float()).abs() / via_rs.float().abs().clamp_min(1.0)
    assert float(d.max()) <= 2 * ULP[dt], float(d.max())
    # fp32 reference: LayerNorm(h) W^T + b (GEGLU: h * gelu(g))
    hf = h.float().cpu()
    ref = F.layer_norm(hf, (C,), gamma, beta, 1e-5) @ W.t() + b
    if geglu:
        hv, gt = ref.chunk(2, dim=-1)
        ref = hv * F.gelu(gt)
    assert O.rel_err(got, ref) < TOL[dt]


@pytest.mark.parametrize("split", [1, 3, 7])
def test_ln_fold_geglu_fp16_batch_invariant(device, split):
    """The folded GEGLU projection at the 8x8 level (K = 1280, 64 rows per image, 256-row tiles), fp16: rows of 16
    images as one call vs the first `split` images + the rest (op_imgs set like the engine), bit for bit."""
    dt, C, N, hw = torch.float16, 1280, 10240, 64
    M = 16 * hw
    x = _dev(_r(M, C, seed=30, shift=0.3), dt, device)
    W, b, gamma, beta = _ln_fold_operands(C, N, 31, True)
    Wg, u, v = _fold(W, b, gamma, beta, dt, device, True)
    xf = x.float()
    mean = xf.mean(-1)
    rstd = torch.rsqrt(((xf - mean[:, None]) ** 2).mean(-1) + 1e-5)
    rs = torch.stack([rstd, rstd * mean], -1).contiguous()
    with L.option(op_imgs=16):
        whole = fold_gemm(x, Wg, u, v, dt, device, rs=rs, geglu=True)
    c = split * hw
    with L.option(op_imgs=split):
        p1 = fold_gemm(x[:c].contiguous(), Wg, u, v, dt, device, rs=rs[:c].contiguous(), geglu=True)
    with L.option(op_imgs=16 - split):
        p2 = fold_gemm(x[c:].contiguous(), Wg, u, v, dt, device, rs=rs[c:].contiguous(), geglu=True)
    torch.cuda.synchronize()
    diff = (whole.float() - torch.cat([p1, p2]).float()).abs().view(16, hw, -1).amax(dim=(1, 2))
    assert torch.isfinite(whole).all()
    assert int((diff > 0).sum()) == 0, diff.tolist()


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_unet_ln_parts_vs_stats_pass(device, dtype):
    """The folded UNet with the producers' partials (ln_parts, default) vs the statistics pass (ln_parts 0): the same
    LayerNorm up to the summation order of its statistics."""
    from tests import models_common as MC
    from image_restoration_and_enhancement_amd.engine import UNet
    pc, sd = MC.state_dicts("denoise")
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    u = UNet(pc.unet, dtype, device)
    u.load_state_dict(sd["unet"])
    g = torch.Generator().manual_seed(5)
    B, h, w = 2, 32, 32
    x = torch.randn(B, 4, h, w, generator=g)
    ctx = torch.randn(B, 77, 768, generator=g)
    xin = torch.zeros(B, h, w, u.cin_pad)
    xin[..., :4] = x.permute(0, 2, 3, 1)
    kv = u.prepare_context(ctx.to(tdt).to(device).contiguous())
    outs = []
    for v in (1, 0):
        with L.option(ln_parts=v):
            outs.append(u.forward(xin.to(tdt).to(device).contiguous(), torch.full((B,), 481.0, device=device), kv,
                                  77).float().cpu())
    rel = float((outs[0] - outs[1]).norm() / outs[1].norm())
    print(f"\nln_parts vs stats pass ({dtype}): rel L2 {rel:.2e}")
    assert torch.isfinite(outs[0]).all()
    assert rel < (1e-2 if dtype == "bf16" else 3e-3), rel
