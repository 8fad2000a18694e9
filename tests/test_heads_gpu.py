"""The models' output heads: GroupNorm -> SiLU -> 3x3 conv to a few channels in one kernel (gn_conv_narrow.hip; the
UNet's conv_norm_out -> conv_out, the VAE encoder's and decoder's, as diffusers runs them under src/inference.py:486)
and the UNet input padded to one 64-channel slab in the 16-bit engines (conv_in on the large-tile conv path).

Checked through the C ABI (irx_op_gn_conv_narrow) against PyTorch fp32 GroupNorm + SiLU (rounded to the storage type,
as the engine's GroupNorm output is) + conv2d with the 16-bit weights, and at the model level: the UNet / VAE with the
fused heads (option gn_narrow, default) vs the GroupNorm pass + conv path.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from image_restoration_and_enhancement_amd import _lib as L
from tests import opref as O

pytestmark = pytest.mark.gpu

DT16 = [torch.bfloat16, torch.float16]
TOL = {torch.bfloat16: 1.5e-2, torch.float16: 3e-3}


def _r(*shape, seed=0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed))


def narrow(x, gamma, beta, w, bias, groups, eps, out_f32, ldo, dt, device):
    n, h, wd, c = x.shape
    cout = w.shape[0]
    xd = x.to(dt).to(device).contiguous()
    wd_ = w.permute(0, 2, 3, 1).to(dt).to(device).contiguous()            # [cout][3][3][c]
    out = torch.full((n, h, wd, ldo), float("nan"), dtype=torch.float32 if out_f32 else dt, device=device)
    ws = torch.empty(L.load().irx_op_gn_conv3_ws_bytes(n, h * wd, groups, c), dtype=torch.uint8, device=device)
    # (device copies held in locals until the launch is queued: a temporary's block could be reused by the next copy)
    gd, bd, bsd = (t.float().to(device).contiguous() for t in (gamma, beta, bias))
    L.call("irx_op_gn_conv_narrow", O.S(), O.DT[dt], O.P(xd), n, h, wd, c, groups, eps, O.P(gd), O.P(bd), 1, O.P(wd_),
           O.P(bsd), cout, O.P(out), ldo, int(out_f32), O.P(ws))
    torch.cuda.synchronize()
    return out


def reference(x, gamma, beta, w, bias, groups, eps, dt):
    xq = x.to(dt).float().permute(0, 3, 1, 2)
    g = F.silu(F.group_norm(xq, groups, gamma, beta, eps)).to(dt).float()
    return F.conv2d(g, w.to(dt).float(), bias, padding=1).permute(0, 2, 3, 1)


@pytest.mark.parametrize("dt", DT16)
@pytest.mark.parametrize("n,h,w,c,cout,out_f32,ldo", [
    (4, 64, 64, 320, 4, True, 4),      # UNet conv_out (eps prediction, fp32)
    (2, 32, 32, 512, 8, False, 8),     # VAE encoder conv_out (moments)
    (1, 96, 80, 128, 3, False, 4),     # VAE decoder conv_out (RGB padded to 4), W not a multiple of 64
    (3, 7, 5, 320, 4, True, 4),        # odd latent
])
def test_gn_conv_narrow_vs_fp32(device, dt, n, h, w, c, cout, out_f32, ldo):
    x = _r(n, h, w, c, seed=1) * 1.5 + 0.3
    gamma, beta = 1.0 + 0.2 * _r(c, seed=2), 0.1 * _r(c, seed=3)
    wt = _r(cout, c, 3, 3, seed=4) / math.sqrt(9 * c)
    bias = 0.1 * _r(cout, seed=5)
    got = narrow(x, gamma, beta, wt, bias, 32, 1e-5, out_f32, ldo, dt, device)
    torch.cuda.synchronize()
    ref = reference(x, gamma, beta, wt, bias, 32, 1e-5, dt)
    assert torch.isfinite(got[..., :cout]).all()
    if ldo > cout:    # padding channels of the output rows are not written
        assert torch.isnan(got[..., cout:].float()).all()
    assert O.rel_err(got[..., :cout], ref) < TOL[dt]


def test_gn_conv_narrow_refuses_unaligned_channels(device):
    x = _r(1, 8, 8, 96)
    with pytest.raises(L.IrxError):
        narrow(x, torch.ones(96), torch.zeros(96), _r(4, 96, 3, 3), torch.zeros(4), 32, 1e-5, True, 4,
               torch.bfloat16, device)


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_unet_heads_fused_vs_unfused(device, dtype):
    """UNet at 64x64 latents: the fused output head and the 64-channel conv_in path vs the GroupNorm pass + conv
    (option gn_narrow 0) — the same arithmetic up to the conv's accumulation order."""
    from tests import models_common as MC
    from image_restoration_and_enhancement_amd.engine import UNet
    pc, sd = MC.state_dicts("denoise")
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    unet = UNet(pc.unet, dtype, device)
    unet.load_state_dict(sd["unet"])
    assert unet.cin_pad == 64
    g = torch.Generator().manual_seed(9)
    xin = torch.zeros(2, 64, 64, unet.cin_pad)
    xin[..., :4] = torch.randn(2, 64, 64, 4, generator=g)
    kv = unet.prepare_context(torch.randn(2, 77, 768, generator=g).to(tdt).to(device).contiguous())
    outs = []
    for v in (1, 0):
        with L.option(gn_narrow=v):
            outs.append(unet.forward(xin.to(tdt).to(device).contiguous(), torch.full((2,), 481.0, device=device),
                                     kv, 77).float().cpu())
    rel = float((outs[0] - outs[1]).norm() / outs[1].norm())
    print(f"\nUNet heads fused vs unfused ({dtype}): rel L2 {rel:.2e}")
    assert torch.isfinite(outs[0]).all()
    assert rel < (2e-3 if dtype == "bf16" else 5e-4), rel


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_vae_heads_fused_vs_unfused(device, dtype):
    from tests import models_common as MC
    from image_restoration_and_enhancement_amd.engine import VAE
    pc, sd = MC.state_dicts("denoise")
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    vae = VAE(pc.vae, dtype, device)
    vae.load_state_dict(sd["vae"])
    g = torch.Generator().manual_seed(10)
    img = torch.zeros(2, 128, 128, 8)
    img[..., :3] = torch.rand(2, 128, 128, 3, generator=g) * 2 - 1
    img = img.to(tdt).to(device).contiguous()
    z = vae.encode(img).contiguous()          # one decoder input for both arms (isolates the decoder's head)
    res = []
    for v in (1, 0):
        with L.option(gn_narrow=v):
            m = vae.encode(img).float().cpu()
            d = vae.decode(z).float().cpu()
        res.append((m, d))
    for k in range(2):
        rel = float((res[0][k] - res[1][k]).norm() / res[1][k].norm())
        assert torch.isfinite(res[0][k]).all()
        assert rel < (1e-2 if dtype == "bf16" else 2e-3), (k, rel)


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("res", [64, 40])
def test_unet_up2_vs_resize_conv(device, dtype, res):
    """The UNet's nearest-2x upsamplers as four per-parity 2x2 convs (option up2, default) vs the resize conv
    (up2 0): the same real arithmetic (tests/test_ln_fold_host.py::test_conv_up2_parity_identity), the folded
    weights rounded once to 16 bit.  res 40: latent sides not divisible by 8 (5x5 -> 10x10 -> 20x20 -> 40x40)."""
    from tests import models_common as MC
    from image_restoration_and_enhancement_amd.engine import UNet
    pc, sd = MC.state_dicts("denoise")
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    unet = UNet(pc.unet, dtype, device)
    unet.load_state_dict(sd["unet"])
    g = torch.Generator().manual_seed(11)
    xin = torch.zeros(2, res, res, unet.cin_pad)
    xin[..., :4] = torch.randn(2, res, res, 4, generator=g)
    xin = xin.to(tdt).to(device).contiguous()
    kv = unet.prepare_context(torch.randn(2, 77, 768, generator=g).to(tdt).to(device).contiguous())
    outs = []
    for v in (1, 0):
        with L.option(up2=v):
            outs.append(unet.forward(xin, torch.full((2,), 481.0, device=device), kv, 77).float().cpu())
    rel = float((outs[0] - outs[1]).norm() / outs[1].norm())
    print(f"\nUNet up2 vs resize conv ({dtype}, {res}x{res}): rel L2 {rel:.2e}")
    assert torch.isfinite(outs[0]).all()
    assert rel < (2e-2 if dtype == "bf16" else 4e-3), rel


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_vae_decoder_up2_vs_resize_conv(device, dtype):
    from tests import models_common as MC
    from image_restoration_and_enhancement_amd.engine import VAE
    pc, sd = MC.state_dicts("denoise")
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    vae = VAE(pc.vae, dtype, device)
    vae.load_state_dict(sd["vae"])
    g = torch.Generator().manual_seed(12)
    z = torch.zeros(2, 16, 16, 8)
    z[..., :4] = torch.randn(2, 16, 16, 4, generator=g)
    z = z.to(tdt).to(device).contiguous()
    outs = []
    for v in (1, 0):
        with L.option(up2=v):
            outs.append(vae.decode(z).float().cpu())
    rel = float((outs[0] - outs[1]).norm() / outs[1].norm())
    print(f"\nVAE decoder up2 vs resize conv ({dtype}): rel L2 {rel:.2e}")
    assert torch.isfinite(outs[0]).all()
    assert rel < (3e-2 if dtype == "bf16" else 5e-3), rel


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("res", [64, 40])
def test_unet_head_major_operands_bit_exact(device, dtype, res):
    """q|k|v written head-major by the projection epilogue (option attn_hm, default; the segment-major coalesced
    store walk of gemm2's store pass) vs row-major operands: the same values in another layout, read by the same
    attention arithmetic — the UNet output is identical bit for bit.  res 40: 5x5 .. 40x40 levels (tiles that the
    segment walk refuses: rows of one tile spanning two images fall back to the per-chunk c_off stores)."""
    from tests import models_common as MC
    from image_restoration_and_enhancement_amd.engine import UNet
    pc, sd = MC.state_dicts("denoise")
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    unet = UNet(pc.unet, dtype, device)
    unet.load_state_dict(sd["unet"])
    g = torch.Generator().manual_seed(13)
    xin = torch.zeros(2, res, res, unet.cin_pad)
    xin[..., :4] = torch.randn(2, res, res, 4, generator=g)
    xin = xin.to(tdt).to(device).contiguous()
    kv = unet.prepare_context(torch.randn(2, 77, 768, generator=g).to(tdt).to(device).contiguous())
    outs = []
    for v in (1, 0):
        with L.option(attn_hm=v):
            outs.append(unet.forward(xin, torch.full((2,), 481.0, device=device), kv, 77).float().cpu())
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("res", [64, 40])
def test_unet_fused_small_level_groupnorm_bit_exact(device, dtype, res):
    """GroupNorm at the small levels (HW <= 256: 16^2 / 8^2 at res 64, 10^2 / 5^2 at res 40) as one finalize + apply
    launch (gn_fa_kernel, option gn_fa, default) vs gn_finalize_parts + gn_apply: the same fold (gn_parts_fold), the
    same scale / shift and the same per-element op — identical UNet output bit for bit."""
    from tests import models_common as MC
    from image_restoration_and_enhancement_amd.engine import UNet
    pc, sd = MC.state_dicts("denoise")
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    unet = UNet(pc.unet, dtype, device)
    unet.load_state_dict(sd["unet"])
    g = torch.Generator().manual_seed(14)
    xin = torch.zeros(2, res, res, unet.cin_pad)
    xin[..., :4] = torch.randn(2, res, res, 4, generator=g)
    xin = xin.to(tdt).to(device).contiguous()
    kv = unet.prepare_context(torch.randn(2, 77, 768, generator=g).to(tdt).to(device).contiguous())
    outs = []
    # 1: small levels only; 1 << 30: every level (pixel slices above HW 256, XCD-grouped), over the widest / the
    # narrowest channel span per block; 1024: up to 32^2
    for v, wide in ((0, 1), (1, 1), (1 << 30, 1), (1 << 30, 0), (1024, 1)):
        with L.option(gn_fa=v, gn_fa_wide=wide):
            outs.append(unet.forward(xin, torch.full((2,), 481.0, device=device), kv, 77).float().cpu())
    assert torch.isfinite(outs[0]).all()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_vae_fused_groupnorm_slices_bit_exact(device, dtype):
    """The VAE's GroupNorms from producer partials (64^2 .. 128^2 levels here, N = 1 and 2) as one sliced finalize +
    apply launch (gn_fa 1 << 30) vs gn_finalize_parts + gn_apply (gn_fa 0): identical encoder and decoder outputs."""
    from tests import models_common as MC
    from image_restoration_and_enhancement_amd.engine import VAE
    pc, sd = MC.state_dicts("denoise")
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    vae = VAE(pc.vae, dtype, device)
    vae.load_state_dict(sd["vae"])
    g = torch.Generator().manual_seed(15)
    for n in (1, 2):
        img = torch.zeros(n, 128, 128, 8)
        img[..., :3] = torch.rand(n, 128, 128, 3, generator=g) * 2 - 1
        img = img.to(tdt).to(device).contiguous()
        res = []
        for v in (0, 1 << 30):
            with L.option(gn_fa=v):
                z = vae.encode(img).contiguous()
                res.append((z.float().cpu(), vae.decode(z).float().cpu()))
        for k in range(2):
            assert torch.isfinite(res[1][k]).all()
            assert torch.equal(res[1][k], res[0][k]), (n, k)


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_unet_reduce_kernel_groupnorm_partials(device, dtype):
    """The 8x8-level split-K convs' GroupNorm partials from the reduce kernel (splitk_reduce_gn_kernel, option
    gn_red_parts, default) vs a statistics pass over the stored output (gn_stats3 + gn_finalize3): the same statistics
    up to fp64 summation order, whose last-bit differences flip 16-bit roundings that the UNet then carries (measured
    rel L2 5.8e-3 bf16, 1.0e-3 fp16); and each matches its own gn_fa-off form bit for bit (the fold is shared)."""
    from tests import models_common as MC
    from image_restoration_and_enhancement_amd.engine import UNet
    pc, sd = MC.state_dicts("denoise")
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    unet = UNet(pc.unet, dtype, device)
    unet.load_state_dict(sd["unet"])
    g = torch.Generator().manual_seed(16)
    xin = torch.zeros(2, 64, 64, unet.cin_pad)
    xin[..., :4] = torch.randn(2, 64, 64, 4, generator=g)
    xin = xin.to(tdt).to(device).contiguous()
    kv = unet.prepare_context(torch.randn(2, 77, 768, generator=g).to(tdt).to(device).contiguous())
    t = torch.full((2,), 481.0, device=device)
    outs = {}
    for red in (1, 0):
        for fa in (4096, 0):
            with L.option(gn_red_parts=red, gn_fa=fa):
                outs[(red, fa)] = unet.forward(xin, t, kv, 77).float().cpu()
    for red in (1, 0):
        assert torch.isfinite(outs[(red, 4096)]).all()
        assert torch.equal(outs[(red, 4096)], outs[(red, 0)])
    a, b = outs[(1, 4096)], outs[(0, 4096)]
    rel = float((a - b).norm() / b.norm())
    print(f"\nreduce-kernel GroupNorm partials vs stats pass ({dtype}): rel L2 {rel:.2e}")
    assert rel < (1e-2 if dtype == "bf16" else 2e-3), rel


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_halo_up2_vs_im2col_up2(device, dtype):
    """The upsamplers' per-parity 2x2 convs on 4-tap halo tiles (option halo_up2, default: row tiles at low-resolution
    widths 16 / 32 / 64, strip tiles at 128) vs the same convs on the im2col walk: the same products, summed slab-major
    instead of tap-major, so the outputs agree to fp32 reassociation.  VAE decoder from 32x32 latents (up2 at
    32 -> 64 and 64 -> 128 on row tiles, 128 -> 256 on strips) and the UNet at 64x64 (16 -> 32, 32 -> 64)."""
    from tests import models_common as MC
    from image_restoration_and_enhancement_amd.engine import UNet, VAE
    pc, sd = MC.state_dicts("denoise")
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    g = torch.Generator().manual_seed(13)
    vae = VAE(pc.vae, dtype, device)
    vae.load_state_dict(sd["vae"])
    z = torch.zeros(2, 32, 32, 8)
    z[..., :4] = torch.randn(2, 32, 32, 4, generator=g)
    z = z.to(tdt).to(device).contiguous()
    outs = []
    for v in (1, 0):
        with L.option(halo_up2=v):
            outs.append(vae.decode(z).float().cpu())
    rel_vae = float((outs[0] - outs[1]).norm() / outs[1].norm())
    unet = UNet(pc.unet, dtype, device)
    unet.load_state_dict(sd["unet"])
    xin = torch.zeros(2, 64, 64, unet.cin_pad)
    xin[..., :4] = torch.randn(2, 64, 64, 4, generator=g)
    xin = xin.to(tdt).to(device).contiguous()
    kv = unet.prepare_context(torch.randn(2, 77, 768, generator=g).to(tdt).to(device).contiguous())
    uo = []
    for v in (1, 0):
        with L.option(halo_up2=v):
            uo.append(unet.forward(xin, torch.full((2,), 481.0, device=device), kv, 77).float().cpu())
    rel_unet = float((uo[0] - uo[1]).norm() / uo[1].norm())
    print(f"\nhalo up2 vs im2col up2 ({dtype}): VAE rel L2 {rel_vae:.2e}, UNet rel L2 {rel_unet:.2e}")
    assert torch.isfinite(outs[0]).all() and torch.isfinite(uo[0]).all()
    # (the bars of the up2-vs-resize tests above; measured round 6: VAE 1.5e-2 / 1.9e-3, UNet 7.9e-3 / 9.9e-4 for
    # bf16 / fp16 — the 8x ratio of the two types' rounding, i.e. reassociation, not a mapping error)
    assert rel_vae < (3e-2 if dtype == "bf16" else 5e-3), rel_vae
    assert rel_unet < (2e-2 if dtype == "bf16" else 4e-3), rel_unet
