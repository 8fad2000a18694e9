"""CPU fp32 restatement of the SD-1.5 modules the reference runs through diffusers.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  NCHW layout, exactly the
tensor algebra of diffusers 0.35.2 and
transformers' CLIPTextModel:

* `unet_forward`  — UNet2DConditionModel.forward for the config in
  `outputs/models/denoising/best/unet/config.json:5-67` (called by the reference at
  `src/inference.py:486, :566, :664, :758` through the diffusers pipelines).
* `vae_encode_moments` / `vae_decode` — AutoencoderKL (`.../best/vae/config.json:5-37`).
* `clip_text_forward` — CLIPTextModel (`.../best/text_encoder/config.json:10-23`).

Weights are a dict in diffusers / transformers naming (`W[name]`), so the same
state dict drives this oracle and the HIP engine.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
W_t = Dict[str, Tensor]


# --------------------------------------------------------------------------- building blocks
def resnet_block(W: W_t, p: str, x: Tensor, temb: Optional[Tensor], eps: float, groups: int = 32) -> Tensor:
    """diffusers ResnetBlock2D (resnet_time_scale_shift='default', output_scale_factor=1)."""
    h = F.group_norm(x, groups, W[p + "norm1.weight"], W[p + "norm1.bias"], eps)
    h = F.silu(h)
    h = F.conv2d(h, W[p + "conv1.weight"], W[p + "conv1.bias"], padding=1)
    if temb is not None:
        t = F.linear(F.silu(temb), W[p + "time_emb_proj.weight"], W[p + "time_emb_proj.bias"])
        h = h + t[:, :, None, None]
    h = F.group_norm(h, groups, W[p + "norm2.weight"], W[p + "norm2.bias"], eps)
    h = F.silu(h)
    h = F.conv2d(h, W[p + "conv2.weight"], W[p + "conv2.bias"], padding=1)
    if (p + "conv_shortcut.weight") in W:
        x = F.conv2d(x, W[p + "conv_shortcut.weight"], W[p + "conv_shortcut.bias"])
    return (x + h) / 1.0


def attention(q: Tensor, k: Tensor, v: Tensor, heads: int, causal: bool = False) -> Tensor:
    """Multi-head scaled-dot-product attention on (B, L, C) tensors (SDPA semantics)."""
    B, Lq, C = q.shape
    Lk = k.shape[1]
    d = C // heads
    q = q.view(B, Lq, heads, d).transpose(1, 2)
    k = k.view(B, Lk, heads, d).transpose(1, 2)
    v = v.view(B, Lk, heads, d).transpose(1, 2)
    s = torch.matmul(q, k.transpose(-1, -2)) * (1.0 / math.sqrt(d))
    if causal:
        mask = torch.full((Lq, Lk), float("-inf")).triu(1)
        s = s + mask
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, v)
    return o.transpose(1, 2).reshape(B, Lq, C)


def attn_block(W: W_t, p: str, x: Tensor, ctx: Optional[Tensor], heads: int) -> Tensor:
    """diffusers Attention (AttnProcessor2_0) for the UNet: q/k/v without bias, to_out with bias."""
    src = x if ctx is None else ctx
    q = F.linear(x, W[p + "to_q.weight"])
    k = F.linear(src, W[p + "to_k.weight"])
    v = F.linear(src, W[p + "to_v.weight"])
    o = attention(q, k, v, heads)
    return F.linear(o, W[p + "to_out.0.weight"], W[p + "to_out.0.bias"])


def transformer2d(W: W_t, p: str, x: Tensor, ctx: Tensor, heads: int, groups: int = 32) -> Tensor:
    """diffusers Transformer2DModel, use_linear_projection=False, one BasicTransformerBlock."""
    B, C, H, Wd = x.shape
    res = x
    h = F.group_norm(x, groups, W[p + "norm.weight"], W[p + "norm.bias"], 1e-6)
    h = F.conv2d(h, W[p + "proj_in.weight"], W[p + "proj_in.bias"])
    h = h.permute(0, 2, 3, 1).reshape(B, H * Wd, C)
    b = p + "transformer_blocks.0."
    n = F.layer_norm(h, (C,), W[b + "norm1.weight"], W[b + "norm1.bias"], 1e-5)
    h = attn_block(W, b + "attn1.", n, None, heads) + h
    n = F.layer_norm(h, (C,), W[b + "norm2.weight"], W[b + "norm2.bias"], 1e-5)
    h = attn_block(W, b + "attn2.", n, ctx, heads) + h
    n = F.layer_norm(h, (C,), W[b + "norm3.weight"], W[b + "norm3.bias"], 1e-5)
    pr = F.linear(n, W[b + "ff.net.0.proj.weight"], W[b + "ff.net.0.proj.bias"])
    hh, gate = pr.chunk(2, dim=-1)
    ff = hh * F.gelu(gate)
    h = F.linear(ff, W[b + "ff.net.2.weight"], W[b + "ff.net.2.bias"]) + h
    h = h.reshape(B, H, Wd, C).permute(0, 3, 1, 2).contiguous()
    h = F.conv2d(h, W[p + "proj_out.weight"], W[p + "proj_out.bias"])
    return h + res


def timestep_embedding(t: Tensor, dim: int, flip_sin_to_cos: bool = True, shift: float = 0.0) -> Tensor:
    """diffusers get_timestep_embedding (max_period 10000, scale 1)."""
    half = dim // 2
    exponent = -math.log(10000) * torch.arange(0, half, dtype=torch.float32)
    exponent = exponent / (half - shift)
    emb = torch.exp(exponent)
    emb = t[:, None].float() * emb[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


def _up_plan(cfg) -> List[dict]:
    rev = list(reversed(cfg.block_out_channels))
    out_ch = rev[0]
    plan = []
    n = len(rev)
    for i in range(n):
        prev = out_ch
        out_ch = rev[i]
        plan.append({"n": cfg.layers_per_block + 1, "attn": cfg.up_attn[i], "upsample": i < n - 1})
    return plan


def unet_forward(W: W_t, cfg, x: Tensor, t: Tensor, ctx: Tensor) -> Tensor:
    """UNet2DConditionModel.forward (SD-1.5).  x: (B, Cin, h, w); t: (B,) or scalar; ctx: (B, 77, 768)."""
    B = x.shape[0]
    heads = cfg.attention_heads
    eps = cfg.norm_eps
    G = cfg.norm_num_groups
    nup = len(cfg.block_out_channels) - 1
    fwd_up_size = any(s % (2 ** nup) != 0 for s in x.shape[-2:])
    if t.dim() == 0:
        t = t[None]
    t = t.expand(B)
    temb = timestep_embedding(t, cfg.block_out_channels[0], cfg.flip_sin_to_cos, cfg.freq_shift)
    temb = F.linear(temb, W["time_embedding.linear_1.weight"], W["time_embedding.linear_1.bias"])
    temb = F.silu(temb)
    temb = F.linear(temb, W["time_embedding.linear_2.weight"], W["time_embedding.linear_2.bias"])

    h = F.conv2d(x, W["conv_in.weight"], W["conv_in.bias"], padding=1)
    skips = [h]
    for i in range(len(cfg.block_out_channels)):
        for j in range(cfg.layers_per_block):
            h = resnet_block(W, f"down_blocks.{i}.resnets.{j}.", h, temb, eps, G)
            if cfg.down_attn[i]:
                h = transformer2d(W, f"down_blocks.{i}.attentions.{j}.", h, ctx, heads, G)
            skips.append(h)
        if i < len(cfg.block_out_channels) - 1:
            p = f"down_blocks.{i}.downsamplers.0.conv."
            h = F.conv2d(h, W[p + "weight"], W[p + "bias"], stride=2, padding=1)
            skips.append(h)
    h = resnet_block(W, "mid_block.resnets.0.", h, temb, eps, G)
    h = transformer2d(W, "mid_block.attentions.0.", h, ctx, heads, G)
    h = resnet_block(W, "mid_block.resnets.1.", h, temb, eps, G)
    for i, blk in enumerate(_up_plan(cfg)):
        n = blk["n"]
        res = skips[-n:]
        skips = skips[:-n]
        up_size = skips[-1].shape[2:] if (fwd_up_size and skips) else None
        for j in range(n):
            r = res[-1]
            res = res[:-1]
            h = torch.cat([h, r], dim=1)
            h = resnet_block(W, f"up_blocks.{i}.resnets.{j}.", h, temb, eps, G)
            if blk["attn"]:
                h = transformer2d(W, f"up_blocks.{i}.attentions.{j}.", h, ctx, heads, G)
        if blk["upsample"]:
            if up_size is None:
                h = F.interpolate(h, scale_factor=2.0, mode="nearest")
            else:
                h = F.interpolate(h, size=up_size, mode="nearest")
            p = f"up_blocks.{i}.upsamplers.0.conv."
            h = F.conv2d(h, W[p + "weight"], W[p + "bias"], padding=1)
    h = F.group_norm(h, G, W["conv_norm_out.weight"], W["conv_norm_out.bias"], eps)
    h = F.silu(h)
    return F.conv2d(h, W["conv_out.weight"], W["conv_out.bias"], padding=1)


# --------------------------------------------------------------------------- VAE
def vae_attn(W: W_t, p: str, x: Tensor, eps: float, groups: int = 32) -> Tensor:
    """diffusers Attention in UNetMidBlock2D of AutoencoderKL (1 head, group_norm, residual)."""
    B, C, H, Wd = x.shape
    res = x
    h = x.view(B, C, H * Wd).transpose(1, 2)
    h = F.group_norm(h.transpose(1, 2), groups, W[p + "group_norm.weight"], W[p + "group_norm.bias"], eps).transpose(1, 2)
    q = F.linear(h, W[p + "to_q.weight"], W[p + "to_q.bias"])
    k = F.linear(h, W[p + "to_k.weight"], W[p + "to_k.bias"])
    v = F.linear(h, W[p + "to_v.weight"], W[p + "to_v.bias"])
    o = attention(q, k, v, 1)
    o = F.linear(o, W[p + "to_out.0.weight"], W[p + "to_out.0.bias"])
    o = o.transpose(-1, -2).reshape(B, C, H, Wd)
    return (o + res) / 1.0


def vae_encode_moments(W: W_t, cfg, x: Tensor) -> Tensor:
    """AutoencoderKL.encode up to the (mean, logvar) moments (after quant_conv)."""
    eps = cfg.norm_eps
    G = cfg.norm_num_groups
    h = F.conv2d(x, W["encoder.conv_in.weight"], W["encoder.conv_in.bias"], padding=1)
    nb = len(cfg.block_out_channels)
    for i in range(nb):
        for j in range(cfg.layers_per_block):
            h = resnet_block(W, f"encoder.down_blocks.{i}.resnets.{j}.", h, None, eps, G)
        if i < nb - 1:
            h = F.pad(h, (0, 1, 0, 1), mode="constant", value=0)
            p = f"encoder.down_blocks.{i}.downsamplers.0.conv."
            h = F.conv2d(h, W[p + "weight"], W[p + "bias"], stride=2, padding=0)
    h = resnet_block(W, "encoder.mid_block.resnets.0.", h, None, eps, G)
    h = vae_attn(W, "encoder.mid_block.attentions.0.", h, eps, G)
    h = resnet_block(W, "encoder.mid_block.resnets.1.", h, None, eps, G)
    h = F.group_norm(h, G, W["encoder.conv_norm_out.weight"], W["encoder.conv_norm_out.bias"], eps)
    h = F.silu(h)
    h = F.conv2d(h, W["encoder.conv_out.weight"], W["encoder.conv_out.bias"], padding=1)
    return F.conv2d(h, W["quant_conv.weight"], W["quant_conv.bias"])


def latent_sample(moments: Tensor, noise: Tensor) -> Tensor:
    """DiagonalGaussianDistribution(moments).sample(generator) with the drawn noise supplied."""
    mean, logvar = torch.chunk(moments, 2, dim=1)
    logvar = torch.clamp(logvar, -30.0, 20.0)
    std = torch.exp(0.5 * logvar)
    return mean + std * noise


def vae_decode(W: W_t, cfg, z: Tensor) -> Tensor:
    """AutoencoderKL.decode (post_quant_conv + Decoder)."""
    eps = cfg.norm_eps
    G = cfg.norm_num_groups
    z = F.conv2d(z, W["post_quant_conv.weight"], W["post_quant_conv.bias"])
    h = F.conv2d(z, W["decoder.conv_in.weight"], W["decoder.conv_in.bias"], padding=1)
    h = resnet_block(W, "decoder.mid_block.resnets.0.", h, None, eps, G)
    h = vae_attn(W, "decoder.mid_block.attentions.0.", h, eps, G)
    h = resnet_block(W, "decoder.mid_block.resnets.1.", h, None, eps, G)
    nb = len(cfg.block_out_channels)
    for i in range(nb):
        for j in range(cfg.layers_per_block + 1):
            h = resnet_block(W, f"decoder.up_blocks.{i}.resnets.{j}.", h, None, eps, G)
        if i < nb - 1:
            h = F.interpolate(h, scale_factor=2.0, mode="nearest")
            p = f"decoder.up_blocks.{i}.upsamplers.0.conv."
            h = F.conv2d(h, W[p + "weight"], W[p + "bias"], padding=1)
    h = F.group_norm(h, G, W["decoder.conv_norm_out.weight"], W["decoder.conv_norm_out.bias"], eps)
    h = F.silu(h)
    return F.conv2d(h, W["decoder.conv_out.weight"], W["decoder.conv_out.bias"], padding=1)


# --------------------------------------------------------------------------- CLIP text encoder
def clip_text_forward(W: W_t, cfg, ids: Tensor) -> Tensor:
    """transformers CLIPTextModel(...).last_hidden_state for (B, 77) int64 ids (causal, no padding mask)."""
    p = "text_model."
    B, L = ids.shape
    d = cfg.hidden_size
    heads = cfg.num_attention_heads
    h = W[p + "embeddings.token_embedding.weight"][ids] + W[p + "embeddings.position_embedding.weight"][:L][None]
    for i in range(cfg.num_hidden_layers):
        b = f"{p}encoder.layers.{i}."
        r = h
        x = F.layer_norm(h, (d,), W[b + "layer_norm1.weight"], W[b + "layer_norm1.bias"], cfg.layer_norm_eps)
        q = F.linear(x, W[b + "self_attn.q_proj.weight"], W[b + "self_attn.q_proj.bias"])
        k = F.linear(x, W[b + "self_attn.k_proj.weight"], W[b + "self_attn.k_proj.bias"])
        v = F.linear(x, W[b + "self_attn.v_proj.weight"], W[b + "self_attn.v_proj.bias"])
        o = attention(q, k, v, heads, causal=True)
        h = r + F.linear(o, W[b + "self_attn.out_proj.weight"], W[b + "self_attn.out_proj.bias"])
        r = h
        x = F.layer_norm(h, (d,), W[b + "layer_norm2.weight"], W[b + "layer_norm2.bias"], cfg.layer_norm_eps)
        x = F.linear(x, W[b + "mlp.fc1.weight"], W[b + "mlp.fc1.bias"])
        x = x * torch.sigmoid(1.702 * x) if cfg.hidden_act == "quick_gelu" else F.gelu(x)
        h = r + F.linear(x, W[b + "mlp.fc2.weight"], W[b + "mlp.fc2.bias"])
    return F.layer_norm(h, (d,), W[p + "final_layer_norm.weight"], W[p + "final_layer_norm.bias"], cfg.layer_norm_eps)
