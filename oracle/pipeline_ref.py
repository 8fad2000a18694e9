"""CPU fp32 restatement of the diffusers pipelines + the reference's task parameters.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* `PNDMRef` / `DDIMRef`             — diffusers PNDMScheduler (skip_prk_steps) / DDIMScheduler (eta 0),
                                       SURVEY.md Appendix A.3-A.5.
* `preprocess` / `postprocess`      — diffusers VaeImageProcessor (lanczos resize to a multiple of 8,
                                       [-1,1] scaling; denormalize/round to uint8), Appendix A.1.
* `img2img_ref`                     — StableDiffusionImg2ImgPipeline.__call__ (Appendix A.1), the call the
                                       reference makes at `src/inference.py:486-495, :566-573, :664-672`.
* `inpaint_ref`                     — StableDiffusionInpaintPipeline.__call__ (Appendix A.2), called at
                                       `src/inference.py:758-767`.
* `TASKS`                           — the per-task constants of `src/inference.py:86-91, :478-495, :549-574,
                                       :653-672, :743-767`.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F
from PIL import Image

from . import sd_ref

# --------------------------------------------------------------------------- schedulers
def alphas_cumprod_ref(beta_start=0.00085, beta_end=0.012, n=1000) -> torch.Tensor:
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, n, dtype=torch.float32) ** 2
    return torch.cumprod(1.0 - betas, dim=0)


class PNDMRef:
    order = 1

    def __init__(self, n_train=1000, steps_offset=1):
        self.n_train = n_train
        self.offset = steps_offset
        self.alphas_cumprod = alphas_cumprod_ref(n=n_train)
        self.final_alpha_cumprod = self.alphas_cumprod[0]

    def set_timesteps(self, n: int):
        self.num_inference_steps = n
        ratio = self.n_train // n
        ts = (np.arange(0, n) * ratio).round() + self.offset
        plms = np.concatenate([ts[:-1], ts[-2:-1], ts[-1:]])[::-1].copy()
        self.timesteps = torch.from_numpy(plms.astype(np.int64))
        self.ets: List[torch.Tensor] = []
        self.counter = 0
        self.cur_sample = None

    def add_noise(self, x0, noise, t):
        a = self.alphas_cumprod[t]
        return (a ** 0.5) * x0 + ((1 - a) ** 0.5) * noise

    def _prev(self, sample, t, prev_t, mo):
        a_t = self.alphas_cumprod[t]
        a_p = self.alphas_cumprod[prev_t] if prev_t >= 0 else self.final_alpha_cumprod
        b_t = 1 - a_t
        b_p = 1 - a_p
        sample_coeff = (a_p / a_t) ** 0.5
        denom = a_t * b_p ** 0.5 + (a_t * b_t * a_p) ** 0.5
        return sample_coeff * sample - (a_p - a_t) * mo / denom

    def step(self, mo, t, sample):
        t = int(t)
        ratio = self.n_train // self.num_inference_steps
        prev_t = t - ratio
        if self.counter != 1:
            self.ets = self.ets[-3:]
            self.ets.append(mo)
        else:
            prev_t = t
            t = t + ratio
        if len(self.ets) == 1 and self.counter == 0:
            self.cur_sample = sample
        elif len(self.ets) == 1 and self.counter == 1:
            mo = (mo + self.ets[-1]) / 2
            sample = self.cur_sample
            self.cur_sample = None
        elif len(self.ets) == 2:
            mo = (3 * self.ets[-1] - self.ets[-2]) / 2
        elif len(self.ets) == 3:
            mo = (23 * self.ets[-1] - 16 * self.ets[-2] + 5 * self.ets[-3]) / 12
        else:
            mo = (1 / 24) * (55 * self.ets[-1] - 59 * self.ets[-2] + 37 * self.ets[-3] - 9 * self.ets[-4])
        out = self._prev(sample, t, prev_t, mo)
        self.counter += 1
        return out


class DDIMRef:
    order = 1

    def __init__(self, n_train=1000, steps_offset=1):
        self.n_train = n_train
        self.offset = steps_offset
        self.alphas_cumprod = alphas_cumprod_ref(n=n_train)
        self.final_alpha_cumprod = self.alphas_cumprod[0]

    def set_timesteps(self, n: int):
        self.num_inference_steps = n
        ratio = self.n_train // n
        ts = (np.arange(0, n) * ratio).round()[::-1].copy().astype(np.int64) + self.offset
        self.timesteps = torch.from_numpy(ts)

    def add_noise(self, x0, noise, t):
        a = self.alphas_cumprod[t]
        return (a ** 0.5) * x0 + ((1 - a) ** 0.5) * noise

    def step(self, mo, t, sample):
        t = int(t)
        prev_t = t - self.n_train // self.num_inference_steps
        a_t = self.alphas_cumprod[t]
        a_p = self.alphas_cumprod[prev_t] if prev_t >= 0 else self.final_alpha_cumprod
        b_t = 1 - a_t
        x0 = (sample - b_t ** 0.5 * mo) / a_t ** 0.5
        direction = (1 - a_p) ** 0.5 * mo
        return a_p ** 0.5 * x0 + direction


def make_scheduler(kind: str):
    return PNDMRef() if kind == "pndm" else DDIMRef()


def get_timesteps(sched, n: int, strength: float):
    init = min(int(n * strength), n)
    t_start = max(n - init, 0)
    return sched.timesteps[t_start * sched.order:], n - t_start


# --------------------------------------------------------------------------- image processing
def preprocess(img: Image.Image, height: Optional[int] = None, width: Optional[int] = None) -> torch.Tensor:
    """VaeImageProcessor.preprocess for one PIL image -> (1, 3, H, W) float32 in [-1, 1]."""
    if height is None or width is None:
        height = img.height - img.height % 8 if height is None else height
        width = img.width - img.width % 8 if width is None else width
    img = img.resize((width, height), resample=Image.LANCZOS)
    a = np.array(img).astype(np.float32) / 255.0
    if a.ndim == 2:
        a = a[..., None]
    t = torch.from_numpy(a).permute(2, 0, 1)[None].contiguous()
    return 2.0 * t - 1.0


def preprocess_mask(mask: Image.Image, height: int, width: int) -> torch.Tensor:
    """mask_processor: L conversion, lanczos resize, /255, binarize at 0.5 -> (1,1,H,W)."""
    m = mask.convert("L").resize((width, height), resample=Image.LANCZOS)
    a = np.array(m).astype(np.float32) / 255.0
    t = torch.from_numpy(a)[None, None].contiguous()
    t[t < 0.5] = 0
    t[t >= 0.5] = 1
    return t


def decoded_to_float(x: torch.Tensor) -> np.ndarray:
    """denormalize + NHWC float (the stage before uint8 rounding)."""
    return (x * 0.5 + 0.5).clamp(0, 1).permute(0, 2, 3, 1).float().numpy()


def postprocess(x: torch.Tensor) -> List[Image.Image]:
    a = decoded_to_float(x)
    a = (a * 255).round().astype("uint8")
    return [Image.fromarray(i) for i in a]


# --------------------------------------------------------------------------- orchestration
@dataclass
class Models:
    unet_w: dict
    unet_cfg: object
    vae_w: dict
    vae_cfg: object
    clip_w: dict
    clip_cfg: object


def encode_prompt(m: Models, ids_pos: torch.Tensor, ids_neg: Optional[torch.Tensor], cfg_on: bool) -> torch.Tensor:
    pos = sd_ref.clip_text_forward(m.clip_w, m.clip_cfg, ids_pos)
    if not cfg_on:
        return pos
    neg = sd_ref.clip_text_forward(m.clip_w, m.clip_cfg, ids_neg)
    return torch.cat([neg, pos])


@dataclass
class RefResult:
    image: Image.Image
    decoded_float: np.ndarray            # (H, W, 3) in [0,1] before uint8 rounding
    latents: torch.Tensor                 # final latents (1,4,h,w)
    timesteps: List[int]


def img2img_ref(m: Models, image: Image.Image, ids_pos, ids_neg, strength: float, steps: int,
                guidance: float, seed: int, sched_kind: str, n_evals: Optional[int] = None) -> RefResult:
    """StableDiffusionImg2ImgPipeline.__call__ with output_type='pil' (batch 1, CPU generator)."""
    if not 0 <= strength <= 1:
        raise ValueError("strength must be in [0, 1]")
    cfg_on = guidance > 1.0
    embeds = encode_prompt(m, ids_pos, ids_neg, cfg_on)
    x = preprocess(image)
    sched = make_scheduler(sched_kind)
    sched.set_timesteps(steps)
    ts, _ = get_timesteps(sched, steps, strength)
    gen = torch.Generator("cpu").manual_seed(seed)
    moments = sd_ref.vae_encode_moments(m.vae_w, m.vae_cfg, x)
    eps1 = torch.randn(moments[:, :4].shape, generator=gen, dtype=torch.float32)
    z = sd_ref.latent_sample(moments, eps1) * m.vae_cfg.scaling_factor
    noise = torch.randn(z.shape, generator=gen, dtype=torch.float32)
    lat = sched.add_noise(z, noise, int(ts[0]))
    done = []
    for i, t in enumerate(ts):
        if n_evals is not None and i >= n_evals:
            break
        inp = torch.cat([lat] * 2) if cfg_on else lat
        eps = sd_ref.unet_forward(m.unet_w, m.unet_cfg, inp, torch.tensor(int(t)), embeds)
        if cfg_on:
            u, c = eps.chunk(2)
            eps = u + guidance * (c - u)
        lat = sched.step(eps, t, lat)
        done.append(int(t))
    dec = sd_ref.vae_decode(m.vae_w, m.vae_cfg, lat / m.vae_cfg.scaling_factor)
    return RefResult(postprocess(dec)[0], decoded_to_float(dec)[0], lat, done)


def inpaint_ref(m: Models, image: Image.Image, mask: Image.Image, ids_pos, ids_neg, strength: float,
                steps: int, guidance: float, seed: int, sched_kind: str = "ddim",
                height: Optional[int] = None, width: Optional[int] = None,
                n_evals: Optional[int] = None) -> RefResult:
    """StableDiffusionInpaintPipeline.__call__ (9-channel UNet), output_type='pil'."""
    height = height or m.unet_cfg.sample_size * 8
    width = width or m.unet_cfg.sample_size * 8
    cfg_on = guidance > 1.0
    embeds = encode_prompt(m, ids_pos, ids_neg, cfg_on)
    sched = make_scheduler(sched_kind)
    sched.set_timesteps(steps)
    ts, n = get_timesteps(sched, steps, strength)
    if n < 1:
        raise ValueError("strength too small: no denoising steps")
    is_strength_max = strength == 1.0
    init = preprocess(image.convert("RGB"), height, width)
    gen = torch.Generator("cpu").manual_seed(seed)
    lat_shape = (1, 4, height // 8, width // 8)
    image_latents = None
    if not is_strength_max:
        mo = sd_ref.vae_encode_moments(m.vae_w, m.vae_cfg, init)
        e = torch.randn(lat_shape, generator=gen, dtype=torch.float32)
        image_latents = sd_ref.latent_sample(mo, e) * m.vae_cfg.scaling_factor
    noise = torch.randn(lat_shape, generator=gen, dtype=torch.float32)
    lat = noise if is_strength_max else sched.add_noise(image_latents, noise, int(ts[0]))
    mask_c = preprocess_mask(mask, height, width)
    masked = init * (mask_c < 0.5)
    mask_l = F.interpolate(mask_c, size=(height // 8, width // 8))
    mo = sd_ref.vae_encode_moments(m.vae_w, m.vae_cfg, masked)
    e = torch.randn(lat_shape, generator=gen, dtype=torch.float32)
    masked_l = sd_ref.latent_sample(mo, e) * m.vae_cfg.scaling_factor
    if cfg_on:
        mask_l = torch.cat([mask_l] * 2)
        masked_l = torch.cat([masked_l] * 2)
    done = []
    for i, t in enumerate(ts):
        if n_evals is not None and i >= n_evals:
            break
        inp = torch.cat([lat] * 2) if cfg_on else lat
        inp = torch.cat([inp, mask_l, masked_l], dim=1)
        eps = sd_ref.unet_forward(m.unet_w, m.unet_cfg, inp, torch.tensor(int(t)), embeds)
        if cfg_on:
            u, c = eps.chunk(2)
            eps = u + guidance * (c - u)
        lat = sched.step(eps, t, lat)
        done.append(int(t))
    dec = sd_ref.vae_decode(m.vae_w, m.vae_cfg, lat / m.vae_cfg.scaling_factor)
    return RefResult(postprocess(dec)[0], decoded_to_float(dec)[0], lat, done)


# --------------------------------------------------------------------------- reference task constants
TASKS = {
    # task: (prompt, strength, steps, guidance)   src/inference.py:86-91, :485-495, :565-573, :663-672, :757-767
    "denoise": ("clean high quality photo, no noise, sharp details", 0.5, 20, 5.0),
    "sr": ("high quality, detailed, sharp", 0.8, 20, 0.0),       # strength = diffusers default 0.8
    "colorize": ("vibrant realistic natural colors, colorful, high quality photo, detailed, full color, "
                 "rich colors", 0.75, 30, 7.5),
    "inpaint": ("high quality detailed photo", 0.6, 30, 5.0),
}


def normalize_mask_ref(mask: Image.Image, size: Tuple[int, int]) -> Image.Image:
    """RestorationPipeline._normalize_mask (src/inference.py:778-803)."""
    if mask.size != size:
        mask = mask.resize(size, Image.LANCZOS)
    a = np.array(mask.convert("L"))
    if np.sum(a > 128) / a.size < 0.1:
        a = 255 - a
        mask = Image.fromarray(a).convert("L")
    return mask
