"""Model / scheduler configuration for the SD-1.5 restoration engine.

The reference never defines these shapes itself: they come from the diffusers
component configs saved next to each task's weights
(`outputs/models/{task}/best/{unet,vae,text_encoder,scheduler}/*.json`, e.g.
`outputs/models/denoising/best/unet/config.json:5-67`,
`outputs/models/denoising/best/vae/config.json:5-37`,
`outputs/models/denoising/best/text_encoder/config.json:10-23`,
`outputs/models/denoising/best/scheduler/scheduler_config.json:2-13`).
The defaults below restate those files; `*.from_dir()` reads the same JSON
layout from a local model directory so a real `best/` directory drives the
engine unchanged.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field, asdict
from pathlib import Path
from typing import List, Optional


@dataclass
class UNetConfig:
    in_channels: int = 4               # 9 for the inpainting UNet (inpainting/best/unet/config.json:37)
    out_channels: int = 4
    block_out_channels: List[int] = field(default_factory=lambda: [320, 640, 1280, 1280])
    layers_per_block: int = 2
    attention_heads: int = 8           # config "attention_head_dim": 8 is the head COUNT in SD-1.5
    cross_attention_dim: int = 768
    norm_num_groups: int = 32
    norm_eps: float = 1e-5
    sample_size: int = 64
    flip_sin_to_cos: bool = True
    freq_shift: int = 0
    # CrossAttnDownBlock2D x3 + DownBlock2D; UpBlock2D + CrossAttnUpBlock2D x3
    down_attn: List[bool] = field(default_factory=lambda: [True, True, True, False])
    up_attn: List[bool] = field(default_factory=lambda: [False, True, True, True])

    @classmethod
    def from_dict(cls, d: dict) -> "UNetConfig":
        c = cls()
        c.in_channels = int(d.get("in_channels", c.in_channels))
        c.out_channels = int(d.get("out_channels", c.out_channels))
        c.block_out_channels = list(d.get("block_out_channels", c.block_out_channels))
        c.layers_per_block = int(d.get("layers_per_block", c.layers_per_block))
        heads = d.get("num_attention_heads") or d.get("attention_head_dim", c.attention_heads)
        if isinstance(heads, (list, tuple)):
            heads = heads[0]
        c.attention_heads = int(heads)
        c.cross_attention_dim = int(d.get("cross_attention_dim", c.cross_attention_dim))
        c.norm_num_groups = int(d.get("norm_num_groups", c.norm_num_groups))
        c.norm_eps = float(d.get("norm_eps", c.norm_eps))
        c.sample_size = int(d.get("sample_size", c.sample_size))
        c.flip_sin_to_cos = bool(d.get("flip_sin_to_cos", c.flip_sin_to_cos))
        c.freq_shift = int(d.get("freq_shift", c.freq_shift))
        if "down_block_types" in d:
            c.down_attn = [t.startswith("CrossAttn") for t in d["down_block_types"]]
        if "up_block_types" in d:
            c.up_attn = [t.startswith("CrossAttn") for t in d["up_block_types"]]
        if d.get("use_linear_projection", False):
            raise ValueError("use_linear_projection=True UNets are not SD-1.5; unsupported")
        return c


@dataclass
class VAEConfig:
    in_channels: int = 3
    out_channels: int = 3
    latent_channels: int = 4
    block_out_channels: List[int] = field(default_factory=lambda: [128, 256, 512, 512])
    layers_per_block: int = 2
    norm_num_groups: int = 32
    norm_eps: float = 1e-6
    scaling_factor: float = 0.18215
    sample_size: int = 512

    @classmethod
    def from_dict(cls, d: dict) -> "VAEConfig":
        c = cls()
        for k in ("in_channels", "out_channels", "latent_channels", "layers_per_block",
                  "norm_num_groups", "sample_size"):
            if k in d:
                setattr(c, k, int(d[k]))
        if "block_out_channels" in d:
            c.block_out_channels = list(d["block_out_channels"])
        if "scaling_factor" in d:
            c.scaling_factor = float(d["scaling_factor"])
        return c


@dataclass
class CLIPConfig:
    vocab_size: int = 49408
    hidden_size: int = 768
    intermediate_size: int = 3072
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    max_position_embeddings: int = 77
    layer_norm_eps: float = 1e-5
    hidden_act: str = "quick_gelu"

    @classmethod
    def from_dict(cls, d: dict) -> "CLIPConfig":
        c = cls()
        for k in ("vocab_size", "hidden_size", "intermediate_size", "num_hidden_layers",
                  "num_attention_heads", "max_position_embeddings"):
            if k in d:
                setattr(c, k, int(d[k]))
        if "layer_norm_eps" in d:
            c.layer_norm_eps = float(d["layer_norm_eps"])
        if "hidden_act" in d:
            c.hidden_act = str(d["hidden_act"])
        if c.hidden_act not in ("quick_gelu", "gelu"):
            raise ValueError(f"unsupported CLIP activation {c.hidden_act}")
        return c


@dataclass
class SchedulerConfig:
    kind: str = "pndm"                 # "pndm" (denoise/sr/colorize) | "ddim" (inpaint)
    num_train_timesteps: int = 1000
    beta_start: float = 0.00085
    beta_end: float = 0.012
    beta_schedule: str = "scaled_linear"
    steps_offset: int = 1
    set_alpha_to_one: bool = False
    skip_prk_steps: bool = True
    timestep_spacing: str = "leading"
    prediction_type: str = "epsilon"

    @classmethod
    def from_dict(cls, d: dict) -> "SchedulerConfig":
        c = cls()
        name = d.get("_class_name", "PNDMScheduler")
        if name == "PNDMScheduler":
            c.kind = "pndm"
        elif name == "DDIMScheduler":
            c.kind = "ddim"
        else:
            raise ValueError(f"unsupported scheduler {name}")
        for k in ("num_train_timesteps", "steps_offset"):
            if k in d:
                setattr(c, k, int(d[k]))
        for k in ("beta_start", "beta_end"):
            if k in d:
                setattr(c, k, float(d[k]))
        for k in ("beta_schedule", "timestep_spacing", "prediction_type"):
            if k in d:
                setattr(c, k, str(d[k]))
        for k in ("set_alpha_to_one", "skip_prk_steps"):
            if k in d:
                setattr(c, k, bool(d[k]))
        if c.beta_schedule != "scaled_linear" or c.timestep_spacing != "leading":
            raise ValueError("only scaled_linear / leading schedules (the saved SD-1.5 configs) are supported")
        if c.prediction_type != "epsilon":
            raise ValueError("only epsilon prediction is supported")
        if c.kind == "pndm" and not c.skip_prk_steps:
            raise ValueError("PNDM with PRK warm-up steps is not used by the reference configs")
        if d.get("thresholding", False) or d.get("clip_sample", False):
            raise ValueError("DDIM thresholding/clip_sample are off in the reference configs")
        return c


@dataclass
class PipelineConfig:
    """Everything one task's `best/` directory describes."""
    unet: UNetConfig
    vae: VAEConfig
    clip: CLIPConfig
    scheduler: SchedulerConfig
    model_dir: Optional[str] = None

    @classmethod
    def default(cls, task: str) -> "PipelineConfig":
        unet = UNetConfig(in_channels=9 if task == "inpaint" else 4)
        sched = SchedulerConfig(kind="ddim" if task == "inpaint" else "pndm")
        return cls(unet=unet, vae=VAEConfig(), clip=CLIPConfig(), scheduler=sched)

    @classmethod
    def from_dir(cls, model_dir: str | Path, task: str) -> "PipelineConfig":
        p = Path(model_dir)
        base = cls.default(task)

        def rd(*parts):
            f = p.joinpath(*parts)
            return json.loads(f.read_text()) if f.exists() else None

        d = rd("unet", "config.json")
        unet = UNetConfig.from_dict(d) if d else base.unet
        d = rd("vae", "config.json")
        vae = VAEConfig.from_dict(d) if d else base.vae
        d = rd("text_encoder", "config.json")
        clip = CLIPConfig.from_dict(d) if d else base.clip
        d = rd("scheduler", "scheduler_config.json")
        sched = SchedulerConfig.from_dict(d) if d else base.scheduler
        return cls(unet=unet, vae=vae, clip=clip, scheduler=sched, model_dir=str(p))

    def to_dict(self) -> dict:
        return {"unet": asdict(self.unet), "vae": asdict(self.vae), "clip": asdict(self.clip),
                "scheduler": asdict(self.scheduler), "model_dir": self.model_dir}
