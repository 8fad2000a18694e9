"""Host side of the native engine: model handles, weight packing, workspaces.

`NativeModel` wraps one `irx_model` (UNet / VAE / CLIP) created from a config, packs a
diffusers/transformers state dict into the device weight blob the native manifest describes,
and calls the model entry points with PyTorch-ROCm tensors used purely as device buffers.
This replaces the reference's `pipe_class.from_pretrained(...).to("cuda")`
(`src/inference.py:162-176`).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

from . import _lib as L
from .configs import UNetConfig, VAEConfig, CLIPConfig

DTYPES = {"fp32": L.IRX_F32, "float32": L.IRX_F32, "bf16": L.IRX_BF16, "bfloat16": L.IRX_BF16,
          "fp16": L.IRX_F16, "float16": L.IRX_F16, "half": L.IRX_F16}
TORCH_DT = {L.IRX_F32: torch.float32, L.IRX_BF16: torch.bfloat16, L.IRX_F16: torch.float16}


def dtype_code(dtype) -> int:
    if isinstance(dtype, int):
        return dtype
    if isinstance(dtype, torch.dtype):
        return {torch.float32: L.IRX_F32, torch.bfloat16: L.IRX_BF16, torch.float16: L.IRX_F16}[dtype]
    return DTYPES[str(dtype)]


def model_config(kind: int, cfg) -> L.ModelConfig:
    c = L.ModelConfig()
    if kind == L.IRX_MODEL_UNET:
        assert isinstance(cfg, UNetConfig)
        c.in_channels, c.out_channels = cfg.in_channels, cfg.out_channels
        c.n_blocks = len(cfg.block_out_channels)
        for i, v in enumerate(cfg.block_out_channels):
            c.block_out_channels[i] = v
        for i, v in enumerate(cfg.down_attn):
            c.down_attn[i] = int(v)
        for i, v in enumerate(cfg.up_attn):
            c.up_attn[i] = int(v)
        c.layers_per_block = cfg.layers_per_block
        c.heads = cfg.attention_heads
        c.cross_attention_dim = cfg.cross_attention_dim
        c.norm_groups = cfg.norm_num_groups
        c.norm_eps = cfg.norm_eps
        c.flip_sin_to_cos = int(cfg.flip_sin_to_cos)
        c.freq_shift = float(cfg.freq_shift)
    elif kind == L.IRX_MODEL_VAE:
        assert isinstance(cfg, VAEConfig)
        c.in_channels, c.out_channels, c.latent_channels = cfg.in_channels, cfg.out_channels, cfg.latent_channels
        c.n_blocks = len(cfg.block_out_channels)
        for i, v in enumerate(cfg.block_out_channels):
            c.block_out_channels[i] = v
        c.layers_per_block = cfg.layers_per_block
        c.norm_groups = cfg.norm_num_groups
        c.norm_eps = cfg.norm_eps
        c.heads = 1
    else:
        assert isinstance(cfg, CLIPConfig)
        c.vocab_size, c.hidden_size, c.intermediate_size = cfg.vocab_size, cfg.hidden_size, cfg.intermediate_size
        c.num_layers, c.max_positions = cfg.num_hidden_layers, cfg.max_position_embeddings
        c.heads = cfg.num_attention_heads
        c.layer_norm_eps = cfg.layer_norm_eps
        c.quick_gelu = int(cfg.hidden_act == "quick_gelu")
    return c


@dataclass
class ParamSpec:
    name: str
    layout: int
    dtype: int
    shape: Tuple[int, ...]
    offset: int
    nbytes: int
    row_scale: float = 1.0
    scale_rows: int = 0
    aux: str = ""


def geglu64_order(n: int) -> torch.Tensor:
    """Source row of each packed row for the GEGLU64 layout ([values; gates] -> (64 v, 64 g) pairs)."""
    r = torch.arange(n)
    return (r // 128) * 64 + r % 64 + (r % 128 >= 64).long() * (n // 2)


def _convert(t: torch.Tensor, layout: int) -> torch.Tensor:
    t = t.detach().float()
    if layout == L.IRX_LAYOUT_VEC:
        return t.reshape(-1)
    if layout == L.IRX_LAYOUT_MAT:
        return t.reshape(t.shape[0], -1)
    if layout == L.IRX_LAYOUT_VEC_GEGLU64:
        return t.reshape(-1)[geglu64_order(t.numel())]
    if layout == L.IRX_LAYOUT_MAT_GEGLU64:
        return t.reshape(t.shape[0], -1)[geglu64_order(t.shape[0])]
    if layout == L.IRX_LAYOUT_CONV:
        return t.permute(0, 2, 3, 1)          # OIHW -> O,KH,KW,I
    return t


UP2_TAPS = {(0, 0): (0,), (0, 1): (1, 2), (1, 0): (0, 1), (1, 1): (2,)}   # R(a, i): include/irx.h IRX_LAYOUT_CONV_UP2


def conv_up2(w: torch.Tensor) -> torch.Tensor:
    """OIHW 3x3 weights of a nearest-2x upsampler's conv -> [4 Cout, 2, 2, Cin] per-parity 2x2 weights (fp64 sums)."""
    w = w.double()
    out = torch.zeros(4, w.shape[0], 2, 2, w.shape[1], dtype=torch.float64)
    for a in range(2):
        for b in range(2):
            for i in range(2):
                for j in range(2):
                    for ky in UP2_TAPS[(a, i)]:
                        for kx in UP2_TAPS[(b, j)]:
                            out[2 * a + b, :, i, j, :] += w[:, :, ky, kx]
    return out.reshape(4 * w.shape[0], 2, 2, w.shape[1])


def _pad_to(t: torch.Tensor, shape: Tuple[int, ...]) -> torch.Tensor:
    if tuple(t.shape) == tuple(shape):
        return t
    if t.dim() != len(shape) or any(a > b for a, b in zip(t.shape, shape)):
        raise ValueError(f"cannot pad {tuple(t.shape)} to {shape}")
    pads = []
    for a, b in zip(reversed(t.shape), reversed(shape)):
        pads += [0, b - a]
    return F.pad(t, pads)


_POISON = os.environ.get("IRX_WS_POISON", "0") == "1"


class NativeModel:
    """One native model handle (UNet / VAE / CLIP) plus its bound device weight blob."""

    def __init__(self, kind: int, cfg, dtype, device: torch.device | str = "cuda"):
        self.kind = kind
        self.cfg = cfg
        self.dtype = dtype_code(dtype)
        self.device = torch.device(device)
        h = C.c_void_p()
        L.call("irx_model_create", kind, C.byref(model_config(kind, cfg)), self.dtype, C.byref(h))
        self.h = h
        self.blob: Optional[torch.Tensor] = None
        self._ws: Optional[torch.Tensor] = None

    def __del__(self):
        try:
            if getattr(self, "h", None):
                L.call("irx_model_destroy", self.h)
                self.h = None
        except Exception:
            pass

    # ---------------------------------------------------------------- manifest / weights
    def manifest(self) -> List[ParamSpec]:
        n = C.c_int()
        L.call("irx_model_num_params", self.h, C.byref(n))
        out = []
        info = L.ParamInfo()
        for i in range(n.value):
            L.call("irx_model_param_info", self.h, i, C.byref(info))
            out.append(ParamSpec(info.name.decode(), info.layout, info.dtype,
                                 tuple(int(info.shape[k]) for k in range(info.ndim)), int(info.offset),
                                 int(info.bytes), float(info.row_scale), int(info.scale_rows),
                                 (info.aux or b"").decode()))
        return out

    def blob_bytes(self) -> int:
        b = C.c_size_t()
        L.call("irx_model_blob_bytes", self.h, C.byref(b))
        return int(b.value)

    def pack(self, sd: Dict[str, torch.Tensor]) -> torch.Tensor:
        """Host uint8 blob laid out per the native manifest (layout conversion, fusion, padding, cast; the
        LayerNorm fold of IRX_LAYOUT_VEC_LN_U / _LN_V, include/irx.h)."""
        blob = torch.zeros(self.blob_bytes(), dtype=torch.uint8)
        mats: Dict[str, Tuple[ParamSpec, torch.Tensor, torch.Tensor]] = {}   # spec -> (entry, W as packed, cast W')

        def matrix(p: ParamSpec) -> torch.Tensor:      # converted, concatenated, row-scaled (fp32)
            parts = [_convert(sd[n], p.layout) for n in p.name.split("|")]
            t = parts[0] if len(parts) == 1 else torch.cat(parts, dim=0)
            if p.scale_rows:
                t = t.clone()
                t[:p.scale_rows] *= p.row_scale
            return t

        def chain(p: ParamSpec):                       # (A [N][C], B [C][K]) of a MAT_CHAIN / VEC_CHAIN entry
            a, b = p.name.split("|")
            return sd[a].double().reshape(sd[a].shape[0], -1), sd[b].double().reshape(sd[b].shape[0], -1)

        for p in self.manifest():
            if p.layout == L.IRX_LAYOUT_CONV_UP2:        # per-parity 2x2 weights of an upsampler (include/irx.h)
                t = conv_up2(sd[p.name]).float()
            elif p.layout == L.IRX_LAYOUT_MAT_CHAIN:     # [A | A B] (include/irx.h)
                A, Bm = chain(p)
                t = torch.cat([A, A @ Bm], dim=1).float()
            elif p.layout == L.IRX_LAYOUT_VEC_CHAIN:     # a + A b
                A, _ = chain(p)
                an, bn = p.aux.split(";")
                t = (sd[an].double().reshape(-1) + A @ sd[bn].double().reshape(-1)).float()
            elif p.layout == L.IRX_LAYOUT_VEC_LN_U:
                _, _, wq = mats[p.name]
                t = wq.double().sum(dim=1).float()
            elif p.layout == L.IRX_LAYOUT_VEC_LN_V:
                e, w, _ = mats[p.name]
                beta_name, bias_spec = p.aux.split(";")
                t = (w.double() @ sd[beta_name].double().reshape(-1)).float()
                if bias_spec:
                    vl = L.IRX_LAYOUT_VEC_GEGLU64 if e.layout == L.IRX_LAYOUT_MAT_GEGLU64 else L.IRX_LAYOUT_VEC
                    t = t + torch.cat([_convert(sd[n], vl) for n in bias_spec.split("|")])
            else:
                t = matrix(p) if p.layout in (L.IRX_LAYOUT_MAT, L.IRX_LAYOUT_MAT_GEGLU64) else None
                if t is None:
                    parts = [_convert(sd[n], p.layout) for n in p.name.split("|")]
                    t = parts[0] if len(parts) == 1 else torch.cat(parts, dim=0)
                if p.aux:                                  # LayerNorm gamma folded into the columns
                    w = t
                    t = t * sd[p.aux].float().reshape(1, -1)
                    wq = _pad_to(t, p.shape).to(TORCH_DT[p.dtype]).float()[:t.shape[0], :t.shape[1]]
                    mats[p.name] = (p, w, wq)
            t = _pad_to(t, p.shape).to(TORCH_DT[p.dtype]).contiguous()
            if t.numel() * t.element_size() != p.nbytes:
                raise ValueError(f"{p.name}: packed {t.numel() * t.element_size()} bytes, manifest {p.nbytes}")
            blob[p.offset:p.offset + p.nbytes].copy_(t.view(-1).view(torch.uint8))
        return blob

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        self.bind_blob(self.pack(sd).to(self.device))

    def bind_blob(self, dev_blob: torch.Tensor) -> None:
        assert dev_blob.is_cuda and dev_blob.dtype == torch.uint8
        L.call("irx_model_bind", self.h, C.c_void_p(dev_blob.data_ptr()), dev_blob.numel())
        self.blob = dev_blob

    # ---------------------------------------------------------------- workspace
    def workspace(self, nbytes: int) -> torch.Tensor:
        nbytes = max(int(nbytes), 256)
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = None
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        return self._ws

    @staticmethod
    def stream() -> C.c_void_p:
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def _size(self, fn: str, *args) -> int:
        b = C.c_size_t()
        L.call(fn, self.h, *args, C.byref(b))
        return int(b.value)


class UNet(NativeModel):
    def __init__(self, cfg: UNetConfig, dtype, device="cuda"):
        super().__init__(L.IRX_MODEL_UNET, cfg, dtype, device)
        c = C.c_int()
        L.call("irx_unet_input_channels", self.h, C.byref(c))
        self.cin_pad = c.value

    def workspace_bytes(self, batch: int, h: int, w: int) -> int:
        return self._size("irx_unet_workspace_bytes", batch, h, w)

    def prepare_context(self, ctx: torch.Tensor) -> torch.Tensor:
        """Cross-attention K|V of every transformer block for ctx [B, L, 768] (dtype)."""
        B, Lc, _ = ctx.shape
        kv = torch.empty(self._size("irx_unet_context_bytes", B, Lc), dtype=torch.uint8, device=self.device)
        L.call("irx_unet_prepare_context", self.h, self.stream(), C.c_void_p(ctx.data_ptr()), B, Lc,
               C.c_void_p(kv.data_ptr()), None, 0)
        return kv

    def forward(self, x: torch.Tensor, t: torch.Tensor, kv: torch.Tensor, ctx_len: int,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x: [B, h, w, cin_pad] (dtype); t: fp32 [B] on device -> eps fp32 [B, h, w, out_channels]."""
        B, h, w, cp = x.shape
        assert cp == self.cin_pad and x.is_contiguous() and t.dtype == torch.float32 and t.numel() >= B
        if out is None:
            out = torch.empty((B, h, w, self.cfg.out_channels), dtype=torch.float32, device=self.device)
        ws = self.workspace(self.workspace_bytes(B, h, w))
        if _POISON:   # diagnostics (IRX_WS_POISON=1): every workspace byte 0xFF (a NaN in fp16 / bf16 / fp32) first
            ws.fill_(255)
        L.call("irx_unet_forward", self.h, self.stream(), C.c_void_p(x.data_ptr()), B, h, w,
               C.c_void_p(t.data_ptr()), C.c_void_p(kv.data_ptr()), ctx_len, C.c_void_p(out.data_ptr()),
               C.c_void_p(ws.data_ptr()), ws.numel())
        return out


class VAE(NativeModel):
    def __init__(self, cfg: VAEConfig, dtype, device="cuda"):
        super().__init__(L.IRX_MODEL_VAE, cfg, dtype, device)

    def encode(self, img: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """img [B, H, W, 8] (dtype, [-1,1]) -> moments [B, H/8, W/8, 8] (dtype)."""
        B, H, W, c = img.shape
        assert c == 8 and img.is_contiguous()
        if out is None:
            out = torch.empty((B, H // 8, W // 8, 8), dtype=img.dtype, device=self.device)
        ws = self.workspace(self._size("irx_vae_encode_workspace_bytes", B, H, W))
        L.call("irx_vae_encode", self.h, self.stream(), C.c_void_p(img.data_ptr()), B, H, W,
               C.c_void_p(out.data_ptr()), C.c_void_p(ws.data_ptr()), ws.numel())
        return out

    def decode(self, z: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """z [B, h, w, 8] (dtype, latents / scaling_factor) -> image [B, 8h, 8w, 4] (dtype, [-1,1]-ish)."""
        B, h, w, c = z.shape
        assert c == 8 and z.is_contiguous()
        if out is None:
            out = torch.empty((B, h * 8, w * 8, 4), dtype=z.dtype, device=self.device)
        ws = self.workspace(self._size("irx_vae_decode_workspace_bytes", B, h, w))
        L.call("irx_vae_decode", self.h, self.stream(), C.c_void_p(z.data_ptr()), B, h, w,
               C.c_void_p(out.data_ptr()), C.c_void_p(ws.data_ptr()), ws.numel())
        return out


class CLIPText(NativeModel):
    def __init__(self, cfg: CLIPConfig, dtype, device="cuda"):
        super().__init__(L.IRX_MODEL_CLIP, cfg, dtype, device)

    def encode(self, ids: torch.Tensor) -> torch.Tensor:
        """ids int [B, L] -> last_hidden_state [B, L, hidden] (dtype)."""
        ids = ids.to(device=self.device, dtype=torch.int32).contiguous()
        B, Lc = ids.shape
        out = torch.empty((B, Lc, self.cfg.hidden_size), dtype=TORCH_DT[self.dtype], device=self.device)
        ws = self.workspace(self._size("irx_clip_workspace_bytes", B, Lc))
        L.call("irx_clip_encode", self.h, self.stream(), C.c_void_p(ids.data_ptr()), B, Lc,
               C.c_void_p(out.data_ptr()), C.c_void_p(ws.data_ptr()), ws.numel())
        return out
