"""Parameter inventories, seeded random initialisation and local safetensors loading.

The reference loads every component with diffusers/transformers `from_pretrained`
(`src/inference.py:162-172`, `:437-442`). No weights ship with it
(`.gitignore:26-29`), so the engine supports two sources that produce the same
name -> tensor dictionary in the diffusers / transformers naming and layout:

* `random_state_dict(kind, cfg, seed)` — deterministic, per-parameter seeded
  weights with PyTorch's default Conv/Linear bounds (U(-1/sqrt(fan_in), +)).
  Used for parity tests and benchmarks (same shapes as SD-1.5).
* `load_component_dir(dir)` — reads `diffusion_pytorch_model.safetensors` /
  `model.safetensors` from a local `best/` component directory (the layout
  `save_pretrained` writes, e.g. `outputs/models/denoising/best/unet/`).

`*_param_specs(cfg)` enumerate (name, shape) pairs; the native engine publishes
its own manifest and `engine.py` checks every manifest entry against these.
"""
from __future__ import annotations

import zlib
from pathlib import Path
from typing import Dict, Iterator, List, Tuple

import torch

from .configs import UNetConfig, VAEConfig, CLIPConfig

Spec = Tuple[str, Tuple[int, ...]]


# --------------------------------------------------------------------------- inventories
def _resnet_specs(p: str, cin: int, cout: int, temb: int | None) -> Iterator[Spec]:
    yield p + "norm1.weight", (cin,)
    yield p + "norm1.bias", (cin,)
    yield p + "conv1.weight", (cout, cin, 3, 3)
    yield p + "conv1.bias", (cout,)
    if temb:
        yield p + "time_emb_proj.weight", (cout, temb)
        yield p + "time_emb_proj.bias", (cout,)
    yield p + "norm2.weight", (cout,)
    yield p + "norm2.bias", (cout,)
    yield p + "conv2.weight", (cout, cout, 3, 3)
    yield p + "conv2.bias", (cout,)
    if cin != cout:
        yield p + "conv_shortcut.weight", (cout, cin, 1, 1)
        yield p + "conv_shortcut.bias", (cout,)


def _transformer_specs(p: str, c: int, ctx: int) -> Iterator[Spec]:
    yield p + "norm.weight", (c,)
    yield p + "norm.bias", (c,)
    yield p + "proj_in.weight", (c, c, 1, 1)
    yield p + "proj_in.bias", (c,)
    b = p + "transformer_blocks.0."
    for n in ("norm1", "norm2", "norm3"):
        yield b + n + ".weight", (c,)
        yield b + n + ".bias", (c,)
    for a, kv in (("attn1", c), ("attn2", ctx)):
        yield b + a + ".to_q.weight", (c, c)
        yield b + a + ".to_k.weight", (c, kv)
        yield b + a + ".to_v.weight", (c, kv)
        yield b + a + ".to_out.0.weight", (c, c)
        yield b + a + ".to_out.0.bias", (c,)
    yield b + "ff.net.0.proj.weight", (8 * c, c)
    yield b + "ff.net.0.proj.bias", (8 * c,)
    yield b + "ff.net.2.weight", (c, 4 * c)
    yield b + "ff.net.2.bias", (c,)
    yield p + "proj_out.weight", (c, c, 1, 1)
    yield p + "proj_out.bias", (c,)


def unet_up_plan(cfg: UNetConfig) -> List[dict]:
    """diffusers UNet2DConditionModel up-block channel bookkeeping (restated)."""
    rev = list(reversed(cfg.block_out_channels))
    out_ch = rev[0]
    plan = []
    n = len(rev)
    for i in range(n):
        prev = out_ch
        out_ch = rev[i]
        in_ch = rev[min(i + 1, n - 1)]
        res = []
        for j in range(cfg.layers_per_block + 1):
            skip = in_ch if j == cfg.layers_per_block else out_ch
            rin = prev if j == 0 else out_ch
            res.append((rin, skip, out_ch))
        plan.append({"resnets": res, "attn": cfg.up_attn[i], "upsample": i < n - 1, "ch": out_ch})
    return plan


def unet_param_specs(cfg: UNetConfig) -> List[Spec]:
    s: List[Spec] = []
    bo = cfg.block_out_channels
    temb = bo[0] * 4
    s += [("conv_in.weight", (bo[0], cfg.in_channels, 3, 3)), ("conv_in.bias", (bo[0],))]
    s += [("time_embedding.linear_1.weight", (temb, bo[0])), ("time_embedding.linear_1.bias", (temb,)),
          ("time_embedding.linear_2.weight", (temb, temb)), ("time_embedding.linear_2.bias", (temb,))]
    cout = bo[0]
    for i, ch in enumerate(bo):
        cin, cout = cout, ch
        for j in range(cfg.layers_per_block):
            s += _resnet_specs(f"down_blocks.{i}.resnets.{j}.", cin if j == 0 else cout, cout, temb)
            if cfg.down_attn[i]:
                s += _transformer_specs(f"down_blocks.{i}.attentions.{j}.", cout, cfg.cross_attention_dim)
        if i < len(bo) - 1:
            s += [(f"down_blocks.{i}.downsamplers.0.conv.weight", (cout, cout, 3, 3)),
                  (f"down_blocks.{i}.downsamplers.0.conv.bias", (cout,))]
    c = bo[-1]
    s += _resnet_specs("mid_block.resnets.0.", c, c, temb)
    s += _transformer_specs("mid_block.attentions.0.", c, cfg.cross_attention_dim)
    s += _resnet_specs("mid_block.resnets.1.", c, c, temb)
    for i, blk in enumerate(unet_up_plan(cfg)):
        for j, (rin, skip, oc) in enumerate(blk["resnets"]):
            s += _resnet_specs(f"up_blocks.{i}.resnets.{j}.", rin + skip, oc, temb)
            if blk["attn"]:
                s += _transformer_specs(f"up_blocks.{i}.attentions.{j}.", oc, cfg.cross_attention_dim)
        if blk["upsample"]:
            s += [(f"up_blocks.{i}.upsamplers.0.conv.weight", (blk["ch"], blk["ch"], 3, 3)),
                  (f"up_blocks.{i}.upsamplers.0.conv.bias", (blk["ch"],))]
    s += [("conv_norm_out.weight", (bo[0],)), ("conv_norm_out.bias", (bo[0],)),
          ("conv_out.weight", (cfg.out_channels, bo[0], 3, 3)), ("conv_out.bias", (cfg.out_channels,))]
    return s


def _vae_attn_specs(p: str, c: int) -> Iterator[Spec]:
    yield p + "group_norm.weight", (c,)
    yield p + "group_norm.bias", (c,)
    for n in ("to_q", "to_k", "to_v", "to_out.0"):
        yield p + n + ".weight", (c, c)
        yield p + n + ".bias", (c,)


def vae_param_specs(cfg: VAEConfig) -> List[Spec]:
    s: List[Spec] = []
    bo = cfg.block_out_channels
    L = cfg.latent_channels
    s += [("encoder.conv_in.weight", (bo[0], cfg.in_channels, 3, 3)), ("encoder.conv_in.bias", (bo[0],))]
    cout = bo[0]
    for i, ch in enumerate(bo):
        cin, cout = cout, ch
        for j in range(cfg.layers_per_block):
            s += _resnet_specs(f"encoder.down_blocks.{i}.resnets.{j}.", cin if j == 0 else cout, cout, None)
        if i < len(bo) - 1:
            s += [(f"encoder.down_blocks.{i}.downsamplers.0.conv.weight", (cout, cout, 3, 3)),
                  (f"encoder.down_blocks.{i}.downsamplers.0.conv.bias", (cout,))]
    c = bo[-1]
    s += _resnet_specs("encoder.mid_block.resnets.0.", c, c, None)
    s += _vae_attn_specs("encoder.mid_block.attentions.0.", c)
    s += _resnet_specs("encoder.mid_block.resnets.1.", c, c, None)
    s += [("encoder.conv_norm_out.weight", (c,)), ("encoder.conv_norm_out.bias", (c,)),
          ("encoder.conv_out.weight", (2 * L, c, 3, 3)), ("encoder.conv_out.bias", (2 * L,))]
    s += [("quant_conv.weight", (2 * L, 2 * L, 1, 1)), ("quant_conv.bias", (2 * L,)),
          ("post_quant_conv.weight", (L, L, 1, 1)), ("post_quant_conv.bias", (L,))]
    s += [("decoder.conv_in.weight", (c, L, 3, 3)), ("decoder.conv_in.bias", (c,))]
    s += _resnet_specs("decoder.mid_block.resnets.0.", c, c, None)
    s += _vae_attn_specs("decoder.mid_block.attentions.0.", c)
    s += _resnet_specs("decoder.mid_block.resnets.1.", c, c, None)
    rev = list(reversed(bo))
    out_ch = rev[0]
    for i, ch in enumerate(rev):
        prev, out_ch = out_ch, ch
        for j in range(cfg.layers_per_block + 1):
            s += _resnet_specs(f"decoder.up_blocks.{i}.resnets.{j}.", prev if j == 0 else out_ch, out_ch, None)
        if i < len(rev) - 1:
            s += [(f"decoder.up_blocks.{i}.upsamplers.0.conv.weight", (out_ch, out_ch, 3, 3)),
                  (f"decoder.up_blocks.{i}.upsamplers.0.conv.bias", (out_ch,))]
    s += [("decoder.conv_norm_out.weight", (bo[0],)), ("decoder.conv_norm_out.bias", (bo[0],)),
          ("decoder.conv_out.weight", (cfg.out_channels, bo[0], 3, 3)),
          ("decoder.conv_out.bias", (cfg.out_channels,))]
    return s


def clip_param_specs(cfg: CLIPConfig) -> List[Spec]:
    d, f = cfg.hidden_size, cfg.intermediate_size
    p = "text_model."
    s: List[Spec] = [(p + "embeddings.token_embedding.weight", (cfg.vocab_size, d)),
                     (p + "embeddings.position_embedding.weight", (cfg.max_position_embeddings, d))]
    for i in range(cfg.num_hidden_layers):
        b = f"{p}encoder.layers.{i}."
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            s += [(b + f"self_attn.{n}.weight", (d, d)), (b + f"self_attn.{n}.bias", (d,))]
        s += [(b + "layer_norm1.weight", (d,)), (b + "layer_norm1.bias", (d,)),
              (b + "mlp.fc1.weight", (f, d)), (b + "mlp.fc1.bias", (f,)),
              (b + "mlp.fc2.weight", (d, f)), (b + "mlp.fc2.bias", (d,)),
              (b + "layer_norm2.weight", (d,)), (b + "layer_norm2.bias", (d,))]
    s += [(p + "final_layer_norm.weight", (d,)), (p + "final_layer_norm.bias", (d,))]
    return s


def param_specs(kind: str, cfg) -> List[Spec]:
    return {"unet": unet_param_specs, "vae": vae_param_specs, "clip": clip_param_specs}[kind](cfg)


# --------------------------------------------------------------------------- random init
def _is_norm(name: str) -> bool:
    # GroupNorm / LayerNorm modules: norm, norm1..3, conv_norm_out, group_norm, layer_norm*, final_layer_norm
    leaf = name.rsplit(".", 2)[-2] if name.count(".") >= 1 else name
    return "norm" in leaf


def random_param(name: str, shape: Tuple[int, ...], fan_in: int, seed: int) -> torch.Tensor:
    """One parameter, seeded by (seed, name) so it is independent of enumeration order."""
    g = torch.Generator().manual_seed((seed * 1000003 + zlib.crc32(name.encode())) & 0x7FFFFFFFFFFF)
    if "embedding" in name:
        return torch.randn(shape, generator=g) * 0.02
    u = torch.rand(shape, generator=g) * 2.0 - 1.0
    if _is_norm(name):
        # GroupNorm/LayerNorm affine: near identity, but not exactly, so parity tests see it.
        return (1.0 + 0.1 * u) if name.endswith(".weight") else 0.1 * u
    return u * (1.0 / fan_in ** 0.5)


def random_state_dict(kind: str, cfg, seed: int = 0) -> Dict[str, torch.Tensor]:
    specs = param_specs(kind, cfg)
    fan: Dict[str, int] = {}
    for n, sh in specs:
        if n.endswith(".weight") and len(sh) >= 2:
            f = 1
            for x in sh[1:]:
                f *= x
            fan[n[: -len("weight")]] = f
    out = {}
    for n, sh in specs:
        base = n.rsplit(".", 1)[0] + "."
        out[n] = random_param(n, sh, fan.get(base, sh[0] if sh else 1), seed)
    return out


# --------------------------------------------------------------------------- local files
_LEGACY_VAE_ATTN = {"query.": "to_q.", "key.": "to_k.", "value.": "to_v.", "proj_attn.": "to_out.0."}


_WEIGHT_NAMES = ("diffusion_pytorch_model", "model")


def component_weight_files(path: str | Path, variant: str | None = None) -> list:
    """The safetensors file(s) diffusers / transformers `from_pretrained(..., use_safetensors=True,
    variant=variant)` would read from one component directory: `<name>[.<variant>].safetensors`, or the
    shards its `<name>[.<variant>].safetensors.index.json` lists.  Other files (`.fp16` / `.non_ema` variants
    next to the plain file) are ignored unless that variant is asked for."""
    import json

    p = Path(path)
    suffix = f".{variant}.safetensors" if variant else ".safetensors"
    for name in _WEIGHT_NAMES:
        f = p / (name + suffix)
        if f.exists():
            return [f]
        idx = p / (name + suffix + ".index.json")
        if idx.exists():
            shards = sorted(set(json.loads(idx.read_text())["weight_map"].values()))
            return [p / s for s in shards]
    found = sorted(x.name for x in p.glob("*.safetensors"))
    raise FileNotFoundError(f"no {'|'.join(_WEIGHT_NAMES)}{suffix} (or its .index.json) under {p}"
                            + (f"; found {found}" if found else ""))


def load_component_dir(path: str | Path, variant: str | None = None) -> Dict[str, torch.Tensor]:
    """Read one saved component directory's weights (safetensors only: no pickle loading), chosen as
    diffusers chooses them (component_weight_files)."""
    from safetensors.torch import load_file

    sd: Dict[str, torch.Tensor] = {}
    for f in component_weight_files(path, variant):
        sd.update(load_file(str(f)))
    out = {}
    for k, v in sd.items():
        for old, new in _LEGACY_VAE_ATTN.items():
            if ".attentions." in k and old in k:
                k = k.replace(old, new)
        out[k] = v.float()
    return out


def check_state_dict(kind: str, cfg, sd: Dict[str, torch.Tensor]) -> None:
    missing = []
    for n, sh in param_specs(kind, cfg):
        t = sd.get(n)
        if t is None:
            missing.append(n)
            continue
        if tuple(t.shape) != tuple(sh):
            if t.numel() == int(torch.tensor(sh).prod()):
                sd[n] = t.reshape(sh)        # e.g. legacy 1x1-conv attention weights
            else:
                raise ValueError(f"{kind}:{n} has shape {tuple(t.shape)}, expected {sh}")
    if missing:
        raise KeyError(f"{kind}: {len(missing)} parameters missing, e.g. {missing[:3]}")
