"""LayerNorm folded into the transformer projections (16-bit UNets, option ln_fold; GemmArgs::ln_rs, VERDICT r2
item 3): the folded UNet against the unfolded one and against the CPU oracle, at shapes that take the folded
epilogue (32x32 latents: large tiles, in-kernel split-K at the 8x8 level) and at odd shapes whose projections
fall back to the affine-free LayerNorm + folded weights (7x5 latents).  Tolerances: relative L2 vs the fp32
oracle as the unfolded engine's test_unet (4e-2 bf16 / 1e-2 fp16); folded vs unfolded < 1.5e-2 / 5e-3."""
import pytest
import torch

from image_restoration_and_enhancement_amd import _lib as L
from image_restoration_and_enhancement_amd.engine import UNet
from oracle import sd_ref
from tests import models_common as MC

pytestmark = pytest.mark.gpu


def _unet(pc, sd, dtype, device, fold):
    L.call("irx_set_option", b"ln_fold", int(fold))
    try:
        u = UNet(pc.unet, dtype, device)
    finally:
        L.call("irx_set_option", b"ln_fold", 1)
    u.load_state_dict(sd["unet"])
    return u


def _run(u, x, ctx, t, tdt, device):
    B, _, h, w = x.shape
    xin = torch.zeros(B, h, w, u.cin_pad)
    xin[..., :4] = x.permute(0, 2, 3, 1)
    kv = u.prepare_context(ctx.to(tdt).to(device).contiguous())
    return u.forward(xin.to(tdt).to(device).contiguous(), torch.full((B,), float(t), device=device), kv, 77)


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("h,w,B", [(32, 32, 4), (7, 5, 2)])
def test_unet_ln_fold(device, dtype, h, w, B):
    pc, sd = MC.state_dicts("denoise")
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, 4, h, w, generator=g)
    ctx = torch.randn(B, 77, 768, generator=g)
    folded = _run(_unet(pc, sd, dtype, device, True), x, ctx, 481, tdt, device).float().cpu()
    plain = _run(_unet(pc, sd, dtype, device, False), x, ctx, 481, tdt, device).float().cpu()
    with torch.no_grad():
        ref = sd_ref.unet_forward(sd["unet"], pc.unet, x, torch.tensor(481), ctx).permute(0, 2, 3, 1)
    rel = lambda a, b: float((a - b).norm() / b.norm())
    tol_ref, tol_ab = (4e-2, 1.5e-2) if dtype == "bf16" else (1e-2, 5e-3)
    assert rel(folded, ref) < tol_ref, rel(folded, ref)
    assert rel(folded, plain) < tol_ab, rel(folded, plain)
    print(f"\nln_fold {dtype} {h}x{w}: vs oracle {rel(folded, ref):.3e} (unfolded {rel(plain, ref):.3e}), "
          f"folded vs unfolded {rel(folded, plain):.3e}")
