"""CPU test of the LayerNorm fold the 16-bit UNets pack (include/irx.h IRX_LAYOUT_VEC_LN_U / _LN_V; GemmArgs::ln_rs):
for every folded projection, the packed (W * gamma, u, v) reproduce LN(x) W^T + b as
    rstd * (x W'^T) - rstd * mean * u + v
on random rows — the identity the GEMM epilogue applies (no GPU: manifest + packer only).  The fp32 engine packs
no fold."""
import numpy as np
import pytest
import torch

from image_restoration_and_enhancement_amd import _lib as L
from image_restoration_and_enhancement_amd import weights as W
from image_restoration_and_enhancement_amd.configs import UNetConfig
from image_restoration_and_enhancement_amd.engine import UNet, TORCH_DT


def _small_cfg():
    c = UNetConfig()
    c.block_out_channels = [64, 128]
    c.down_attn = [True, False]
    c.up_attn = [False, True]
    c.layers_per_block = 1
    c.cross_attention_dim = 64
    return c


def _entries(m, blob):
    out = {}
    for p in m.manifest():
        t = blob[p.offset:p.offset + p.nbytes].view(TORCH_DT[p.dtype]).float().reshape(p.shape)
        out[(p.name, p.layout)] = (p, t)
    return out


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_ln_fold_identity(dtype):
    cfg = _small_cfg()
    m = UNet(cfg, dtype, "cpu")
    sd = W.random_state_dict("unet", cfg, 3)
    e = _entries(m, m.pack(sd))
    folded = [k for k, (p, _) in e.items() if k[1] in (L.IRX_LAYOUT_MAT, L.IRX_LAYOUT_MAT_GEGLU64) and p.aux]
    assert len(folded) == 3 * 4          # (qkv, attn2.to_q, ff.net.0.proj) x 4 transformers (down, mid, 2 up)
    g = torch.Generator().manual_seed(0)
    for name, lay in folded:
        p, wq = e[(name, lay)]
        u = e[(name, L.IRX_LAYOUT_VEC_LN_U)][1]
        pv, v = e[(name, L.IRX_LAYOUT_VEC_LN_V)]
        C = wq.shape[1]
        x = torch.randn(7, C, generator=g, dtype=torch.float64) * 3 + 1.5
        mean, var = x.mean(1, keepdim=True), x.var(1, unbiased=False, keepdim=True)
        rstd = 1 / torch.sqrt(var + 1e-5)
        got = rstd * (x @ wq.double().T) - rstd * mean * u.double() + v.double()
        # reference: LN with the diffusers weights, the unfused packing of W (re-order, row scale), + bias
        gamma = sd[p.aux].double()
        beta_name, bias_spec = pv.aux.split(";")
        ln = (x - mean) * rstd * gamma + sd[beta_name].double()
        parts = [sd[n].double().reshape(sd[n].shape[0], -1) for n in name.split("|")]
        w = torch.cat(parts)
        if lay == L.IRX_LAYOUT_MAT_GEGLU64:
            from image_restoration_and_enhancement_amd.engine import geglu64_order
            w = w[geglu64_order(w.shape[0])]
        if p.scale_rows:
            w[:p.scale_rows] *= p.row_scale
        ref = ln @ w.T
        if bias_spec:
            b = torch.cat([sd[n].double().reshape(-1) for n in bias_spec.split("|")])
            if lay == L.IRX_LAYOUT_MAT_GEGLU64:
                from image_restoration_and_enhancement_amd.engine import geglu64_order
                b = b[geglu64_order(b.numel())]
            ref = ref + b
        tol = 2e-2 if dtype == "bf16" else 3e-3      # the 16-bit rounding of W * gamma
        assert float((got - ref).norm() / ref.norm()) < tol, name


def test_fp32_engine_packs_no_fold():
    m = UNet(_small_cfg(), "fp32", "cpu")
    assert not any(p.aux or p.layout in (L.IRX_LAYOUT_VEC_LN_U, L.IRX_LAYOUT_VEC_LN_V) for p in m.manifest())


def test_ln_fold_option_off_packs_plain(monkeypatch):
    L.call("irx_set_option", b"ln_fold", 0)
    try:
        m = UNet(_small_cfg(), "bf16", "cpu")
        assert not any(p.aux and p.layout != L.IRX_LAYOUT_VEC_CHAIN for p in m.manifest())
    finally:
        L.call("irx_set_option", b"ln_fold", 1)


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_ff2_proj_out_chain_identity(dtype):
    """IRX_LAYOUT_MAT_CHAIN / VEC_CHAIN (include/irx.h): one GEMM over the concat (h | g) equals diffusers'
    proj_out(h + ff.net.2(g)) — the transformer's last two layers with the residual add between them."""
    cfg = _small_cfg()
    m = UNet(cfg, dtype, "cpu")
    sd = W.random_state_dict("unet", cfg, 5)
    e = _entries(m, m.pack(sd))
    chains = [k for k in e if k[1] == L.IRX_LAYOUT_MAT_CHAIN]
    assert len(chains) == 4                      # one per transformer (down, mid, 2 up)
    g = torch.Generator().manual_seed(1)
    for name, _ in chains:
        wc = e[(name, L.IRX_LAYOUT_MAT_CHAIN)][1].double()
        pb, bc = e[(name, L.IRX_LAYOUT_VEC_CHAIN)]
        po, ff2 = name.split("|")
        C = sd[po].shape[0]
        wpo, wff2 = sd[po].double().reshape(C, -1), sd[ff2].double().reshape(C, -1)
        a_name, b_name = pb.aux.split(";")
        h = torch.randn(9, C, generator=g, dtype=torch.float64)
        gg = torch.randn(9, 4 * C, generator=g, dtype=torch.float64)
        ref = (h + gg @ wff2.T + sd[b_name].double()) @ wpo.T + sd[a_name].double()
        got = torch.cat([h, gg], 1) @ wc.T + bc.double()
        tol = 2e-2 if dtype == "bf16" else 3e-3    # the 16-bit rounding of [W_po | W_po W_ff2]
        assert float((got - ref).norm() / ref.norm()) < tol, name


def test_fp32_engine_packs_no_chain():
    m = UNet(_small_cfg(), "fp32", "cpu")
    assert not any(p.layout in (L.IRX_LAYOUT_MAT_CHAIN, L.IRX_LAYOUT_VEC_CHAIN) for p in m.manifest())


def test_conv_up2_parity_identity():
    """IRX_LAYOUT_CONV_UP2 (include/irx.h): nearest-2x upsample then conv3x3 (pad 1) == the four per-parity 2x2 convs
    of the low-resolution input (pad (1 - a, 1 - b)) with the folded weights, interleaved — exactly, in fp64."""
    import torch.nn.functional as F
    from image_restoration_and_enhancement_amd.engine import conv_up2
    g = torch.Generator().manual_seed(3)
    co, ci, H, Wd = 5, 6, 7, 9
    w = torch.randn(co, ci, 3, 3, generator=g, dtype=torch.float64)
    x = torch.randn(2, ci, H, Wd, generator=g, dtype=torch.float64)
    ref = F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest"), w, padding=1)
    w2 = conv_up2(w).reshape(4, co, 2, 2, ci).permute(0, 1, 4, 2, 3)     # [parity][Cout][Cin][2][2]
    out = torch.empty_like(ref)
    for a in range(2):
        for b in range(2):
            xp = F.pad(x, (1 - b, b, 1 - a, a))              # (left, right, top, bottom): window rows y-1+a .. y+a
            out[:, :, a::2, b::2] = F.conv2d(xp, w2[2 * a + b])
    assert torch.allclose(out, ref, rtol=0, atol=1e-12)
