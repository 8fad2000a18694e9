"""`RestorationPipeline` — drop-in replacement of the reference's `src/inference.py` class, served by the
native MI355X engine (libirx via ctypes) instead of diffusers.

Same surface: `RestorationPipeline(device="auto", config=None, seed=42)`,
`.denoise / .super_resolve / .colorize / .inpaint / .process`, `.load_{denoise,sr,colorize,inpaint}_model`,
attributes `.device .dtype .models .seed .config .prompts`, module-level `TASK_MODEL_DIRS` and `Task`.
Per-task parameters are the reference's (src/inference.py:478-495 denoise: strength 0.5, 20 steps, guidance
5.0; :549-573 sr: area cap 1024^2, diffusers default strength 0.8, 20 steps, guidance 0; :598-672
colorize: grey detection, channel-0 replication, strength 0.75, 30 steps, guidance 7.5; :705-803 inpaint:
mask normalisation / auto-mask, 512x512, strength 0.6, 30 steps, guidance 5.0), and so are the error
semantics: entry points log and fall back to the classical methods (`classical.py`) or return the input
when the diffusion path fails; `process` swallows per-task errors (:885-887).  As in the reference,
`process` passes `prompt=None` for denoise / sr, which the diffusion call rejects, so those two tasks run
their classical fallbacks when reached through `process` (§3.3 of SURVEY.md) — reproduced, not fixed.

Differences that follow from the engine (documented in INTEGRATION.md):
* the diffusion path needs a ROCm GPU; on a CPU-only host the loaders fail and the classical fallbacks
  run (the reference would run diffusers on the CPU).  A missing or unloadable `libirx.so` is never
  hidden: `IrxError` propagates out of every entry point (no silent fallback).
* compute dtype is fp16 on the GPU by default, the reference's own GPU dtype (src/inference.py:57);
  `config["engine"] = {"dtype": "bf16"}` selects the bf16 UNet / CLIP (the VAE stays fp16 unless
  `{"vae_dtype": ...}` says otherwise: the bench configuration) and `{"dtype": "fp32"}` the fp32 engine that
  matches the reference CPU path within 1e-3 per pixel.
* noise is drawn from `torch.Generator("cpu").manual_seed(seed)` — the reference's CPU-path draws.
* weights load from the task's saved `best/` directory (safetensors) or, in pretrained mode
  (`fine_tuned_dir == "nonexistent"`), from a local Hugging Face cache snapshot of `pretrained_id` (no
  network).  `config[task]["weights"] = "random"` selects seeded random weights (benchmarks / tests).
* tasks that resolve to the same weights (denoise / sr / colorize in pretrained mode) share one engine.
"""
from __future__ import annotations

import logging
from pathlib import Path
from typing import Any, Dict, List, Literal, Optional, Sequence

import numpy as np
import torch
from PIL import Image

from . import classical
from . import image_processor as ip
from ._lib import IrxError

logger = logging.getLogger(__name__)

Task = Literal["denoise", "sr", "super_resolution", "colorize", "inpaint"]

TASK_MODEL_DIRS = {
    "denoise": "outputs/models/denoising/best",
    "sr": "outputs/models/super_resolution/best",
    "colorize": "outputs/models/colorization/best",
    "inpaint": "outputs/models/inpainting/best",
}

# (strength, num_inference_steps, guidance_scale) of each reference call site
SD_PARAMS = {
    "denoise": (None, 20, 5.0),      # strength comes from the caller (default 0.5), :486-495
    "sr": (0.8, 20, 0.0),            # diffusers img2img default strength, :566-573
    "colorize": (0.75, 30, 7.5),     # :664-672
    "inpaint": (0.6, 30, 5.0),       # :758-767
}
INPAINT_SIZE = 512                   # unet.sample_size (64) x vae scale factor (8)


class NativeSDModel:
    """What `RestorationPipeline.models[task]` holds when the native engine serves the task (the reference
    stores a diffusers pipeline object there and dispatches on its class, src/inference.py:472)."""

    def __init__(self, engine, kind: str, source: str):
        self.engine = engine          # pipelines.SDEngine
        self.kind = kind              # "img2img" | "inpaint"
        self.source = source          # model directory or "random"

    def __repr__(self):
        return f"NativeSDModel({self.kind}, {self.source})"


def _resolve_pretrained(repo_id: str) -> Path:
    """Local snapshot of a Hugging Face repo (offline: the cache only, never a download)."""
    from huggingface_hub import snapshot_download
    return Path(snapshot_download(repo_id, local_files_only=True))


class RestorationPipeline:
    """Unified restoration pipeline (reference `src/inference.py:48-890`) on the native MI355X engine."""

    def __init__(self, device: str = "auto", config: dict | None = None, seed: int = 42, backend: str | None = None):
        # `backend` is accepted (and ignored) because the reference's own prediction driver passes it
        # (scripts/generate_predictions.py:18), which the reference constructor rejects with a TypeError.
        if backend is not None:
            logger.info(f"backend={backend!r} ignored (per-task backends come from config)")
        if device == "auto":
            self.device = "cuda" if torch.cuda.is_available() else "cpu"
        else:
            self.device = device
        engine_cfg = dict((config or {}).get("engine", {}))
        # fp16 by default: the reference's own GPU dtype (src/inference.py:57), which reproduces the CPU path's
        # PSNR / SSIM at 3 s.f.; a bf16 UNet runs with an fp16 VAE by default (the bf16 VAE is the stage that moves
        # SSIM at the third figure: DESIGN.md §5, profiles/r05_parity_stages.txt)
        self.engine_dtype = engine_cfg.get("dtype", "fp16")
        if self.engine_dtype not in ("bf16", "fp16", "fp32"):
            raise ValueError(f"engine dtype must be 'bf16', 'fp16' or 'fp32', got {self.engine_dtype!r}")
        self.vae_dtype = engine_cfg.get("vae_dtype", "fp16" if self.engine_dtype == "bf16" else self.engine_dtype)
        if self.vae_dtype not in ("bf16", "fp16", "fp32"):
            raise ValueError(f"engine vae_dtype must be 'bf16', 'fp16' or 'fp32', got {self.vae_dtype!r}")
        on_gpu = self.device.startswith("cuda")
        self.dtype = ({"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[self.engine_dtype]
                      if on_gpu else torch.float32)
        self.models: dict[str, object] = {}
        self.seed = seed
        logger.info(f"Using device: {self.device} ({self.dtype}), seed: {seed}")
        default_config = {
            "denoise": {"fine_tuned_dir": TASK_MODEL_DIRS["denoise"],
                        "pretrained_id": "sd-legacy/stable-diffusion-v1-5", "default_backend": "auto"},
            "sr": {"fine_tuned_dir": TASK_MODEL_DIRS["sr"],
                   "pretrained_id": "sd-legacy/stable-diffusion-v1-5", "default_backend": "auto"},
            "colorize": {"fine_tuned_dir": TASK_MODEL_DIRS["colorize"],
                         "pretrained_id": "sd-legacy/stable-diffusion-v1-5"},
            "inpaint": {"fine_tuned_dir": TASK_MODEL_DIRS["inpaint"],
                        "pretrained_id": "runwayml/stable-diffusion-inpainting"},
        }
        self.config = default_config if config is None else {**default_config, **config}
        self.prompts = {
            "denoise": "clean high quality photo, no noise, sharp details",
            "sr": "high quality, detailed, sharp",
            "colorize": "vibrant realistic natural colors, colorful, high quality photo, detailed, full color, "
                        "rich colors",
            "inpaint": "high quality detailed photo",
        }
        self._engines: Dict[tuple, object] = {}

    # ------------------------------------------------------------------------------------ loading
    def _model_source(self, task: str, cfg: dict, train_script: str) -> str:
        """fine-tuned dir if present; pretrained id in pretrained mode; else FileNotFoundError (the
        reference's branch structure, src/inference.py:211-274)."""
        if cfg.get("weights") == "random":
            return "random"
        p = Path(cfg["fine_tuned_dir"])
        if p.exists():
            logger.info("Found fine-tuned model, loading...")
            return str(p)
        if cfg["fine_tuned_dir"] == "nonexistent":
            logger.info("Using pre-trained model from the local Hugging Face cache")
            return str(_resolve_pretrained(cfg["pretrained_id"]))
        raise FileNotFoundError(f"Fine-tuned {task} model not found at {p}. "
                                f"Please train the model first with: python3 scripts/{train_script}")

    def _load_native(self, task: str, source: str) -> NativeSDModel:
        if not self.device.startswith("cuda"):
            raise RuntimeError("the native diffusion engine runs on a ROCm GPU only")
        from .configs import PipelineConfig
        from .pipelines import SDEngine
        kind = "inpaint" if task == "inpaint" else "img2img"
        key = (source, kind, self.engine_dtype, self.vae_dtype)
        if key not in self._engines:
            if source == "random":
                pc = PipelineConfig.default(task)
                eng = SDEngine(pc, self.engine_dtype, self.device, weights="random", weight_seed=0,
                               vae_dtype=self.vae_dtype)
            else:
                pc = PipelineConfig.from_dir(source, task)
                eng = SDEngine(pc, self.engine_dtype, self.device, weights=source, vae_dtype=self.vae_dtype)
            self._engines[key] = eng
            logger.info(f"{task} engine ready ({source}, {self.engine_dtype}, VAE {self.vae_dtype})")
        return NativeSDModel(self._engines[key], kind, source)

    def _try_load(self, task: str, train_script: str) -> NativeSDModel:
        cfg = self.config[task]
        return self._load_native(task, self._model_source(task, cfg, train_script))

    def load_denoise_model(self):
        if "denoise" in self.models:
            return
        backend = self.config["denoise"].get("default_backend", "auto")
        if backend in ("auto", "diffusion"):
            try:
                self.models["denoise"] = self._try_load("denoise", "train_denoising.py")
                return
            except IrxError:
                raise
            except Exception as e:
                if backend == "diffusion":
                    raise RuntimeError(f"Diffusion-based denoising failed: {e}")
                logger.warning(f"Could not load diffusion-based denoising model: {e}")
        if backend in ("auto", "opencv"):
            self.models["denoise"] = None
            logger.info("Denoising model ready (classical fallback)")

    def load_sr_model(self):
        if "sr" in self.models:
            return
        backend = self.config["sr"].get("default_backend", "auto")
        if backend in ("auto", "sd_img2img"):
            try:
                self.models["sr"] = self._try_load("sr", "train_super_resolution.py")
                return
            except IrxError:
                raise
            except Exception as e:
                if backend == "sd_img2img":
                    raise RuntimeError(f"Stable Diffusion Img2Img failed: {e}")
                logger.warning(f"Stable Diffusion Img2Img failed: {e}")
        if backend == "realesrgan":
            raise ImportError("Real-ESRGAN is not available (its weights are a network download)")
        if backend in ("auto", "lanczos", "realesrgan"):
            self.models["sr"] = "lanczos"
            logger.info("Super-resolution model ready (LANCZOS fallback)")

    def load_colorize_model(self):
        if "colorize" in self.models:
            return
        try:
            self.models["colorize"] = self._try_load("colorize", "train_colorization.py")
        except IrxError:
            raise
        except Exception as e:
            logger.warning(f"Could not load Stable Diffusion: {e}")
            self.models["colorize"] = "improved"

    def load_inpaint_model(self):
        if "inpaint" in self.models:
            return
        try:
            self.models["inpaint"] = self._try_load("inpaint", "train_inpainting.py")
        except IrxError:
            raise
        except Exception:
            logger.error("Could not load inpainting model", exc_info=True)
            self.models["inpaint"] = None

    # ------------------------------------------------------------------------------------ engine calls
    def _img2img(self, model: NativeSDModel, images: Sequence[Image.Image], prompt: Optional[str],
                 strength: float, steps: int, guidance: float) -> List[Image.Image]:
        """Same-size RGB PIL images -> restored PIL images (size rounded down to a multiple of 8)."""
        if prompt is None:
            raise ValueError("Provide either `prompt` or `prompt_embeds`.")
        u8 = np.stack([ip.to_uint8(im.convert("RGB")) for im in images])
        if u8.shape[1] < 8 or u8.shape[2] < 8:
            raise ValueError(f"image too small for the VAE: {images[0].size}")
        dev = torch.from_numpy(u8).to(self.device).contiguous()
        res = model.engine.img2img(dev, prompt, strength, steps, guidance, seed=self.seed)
        return [Image.fromarray(a) for a in res.images_u8.cpu().numpy()]

    def _inpaint_native(self, model: NativeSDModel, images: Sequence[Image.Image], masks: Sequence[Image.Image],
                        prompt: str, strength: float, steps: int, guidance: float) -> List[Image.Image]:
        S = INPAINT_SIZE
        u8 = np.stack([ip.to_uint8(im.convert("RGB"), S, S) for im in images])
        m = np.stack([ip.mask_to_binary(mk, S, S) for mk in masks])
        res = model.engine.inpaint(torch.from_numpy(u8).to(self.device).contiguous(),
                                   torch.from_numpy(m).to(self.device).contiguous(), prompt, strength, steps,
                                   guidance, seed=self.seed)
        return [Image.fromarray(a) for a in res.images_u8.cpu().numpy()]

    # ------------------------------------------------------------------------------------ denoise
    def denoise(self, image: Image.Image, strength: float = 0.5, **kwargs) -> Image.Image:
        if "denoise" not in self.models:
            self.load_denoise_model()
        model = self.models.get("denoise")
        if isinstance(model, NativeSDModel):
            return self._denoise_sd(image, model, strength=strength, **kwargs)
        return self._denoise_opencv(image, strength=strength)

    def _denoise_sd(self, image: Image.Image, model, strength: float, **kwargs) -> Image.Image:
        try:
            prompt = kwargs.get("prompt", self.prompts["denoise"])
            _, steps, g = SD_PARAMS["denoise"]
            return self._img2img(model, [image], prompt, strength, steps, g)[0]
        except IrxError:
            raise
        except Exception as e:
            logger.warning(f"Stable Diffusion denoising failed: {e}, using classical fallback")
            return self._denoise_opencv(image, strength=strength)

    def _denoise_opencv(self, image: Image.Image, strength: float) -> Image.Image:
        if self.device.startswith("cuda"):         # NLM + bilateral + median on the GPU; no CPU retry
            from . import nlmeans
            return nlmeans.denoise_opencv(image, strength, device=self.device)
        return classical.denoise_opencv(image, strength)

    # ------------------------------------------------------------------------------------ super-resolution
    def super_resolve(self, image: Image.Image, scale: int = 4, **kwargs) -> Image.Image:
        if "sr" not in self.models:
            self.load_sr_model()
        model = self.models["sr"]
        if isinstance(model, NativeSDModel):
            return self._sr_sd(image, model, scale=scale, **kwargs)
        return self._sr_lanczos(image, scale=scale)

    @staticmethod
    def _cap_area(image: Image.Image) -> Image.Image:
        w, h = image.size
        if w * h > 1024 * 1024:
            new_w, new_h = (1024, int(h * 1024 / w)) if w > h else (int(w * 1024 / h), 1024)
            image = image.resize((new_w, new_h), Image.LANCZOS)
        return image

    def _sr_sd(self, image: Image.Image, model, scale: int, **kwargs) -> Image.Image:
        try:
            image = self._cap_area(image)
            prompt = kwargs.get("prompt", self.prompts["sr"])
            s, steps, g = SD_PARAMS["sr"]
            return self._img2img(model, [image], prompt, s, steps, g)[0]
        except IrxError:
            raise
        except Exception as e:
            logger.warning(f"Stable Diffusion upscaling failed: {e}, falling back to LANCZOS")
            return self._sr_lanczos(image, scale=scale)

    def _sr_lanczos(self, image: Image.Image, scale: int) -> Image.Image:
        return classical.sr_lanczos(image, scale)

    # ------------------------------------------------------------------------------------ colorize
    @staticmethod
    def is_color(image: Image.Image) -> bool:
        """Mean absolute channel difference > 10 -> already colour (src/inference.py:612-630)."""
        a = np.array(image)
        if a.ndim == 3 and a.shape[2] == 3:
            f = a.astype(np.float32)
            d = (np.mean(np.abs(f[..., 0] - f[..., 1])) + np.mean(np.abs(f[..., 1] - f[..., 2]))
                 + np.mean(np.abs(f[..., 0] - f[..., 2]))) / 3.0
            return bool(d > 10.0)
        return False

    @staticmethod
    def gray_to_rgb(image: Image.Image) -> Image.Image:
        """Channel 0 (or the single channel) replicated to RGB (src/inference.py:633-639)."""
        a = np.array(image)
        if a.ndim == 2:
            return Image.fromarray(np.repeat(a[..., None], 3, axis=2))
        if a.ndim == 3 and a.shape[2] == 3:
            return Image.fromarray(np.repeat(a[..., :1], 3, axis=2))
        return image

    def colorize(self, image: Image.Image, **kwargs) -> Image.Image:
        if "colorize" not in self.models:
            self.load_colorize_model()
        model = self.models["colorize"]
        if self.is_color(image):
            logger.info("Image already has color, skipping colorization")
            return image
        image = self.gray_to_rgb(image)
        if isinstance(model, NativeSDModel):
            return self._colorize_sd(image, model, **kwargs)
        return self._colorize_lab(image)

    def _colorize_sd(self, image: Image.Image, model, **kwargs) -> Image.Image:
        try:
            prompt = kwargs.get("prompt") or self.prompts.get("colorize") or \
                "vibrant realistic natural colors, colorful, high quality photo, detailed, full color, rich colors"
            s, steps, g = SD_PARAMS["colorize"]
            return self._img2img(model, [image], prompt, s, steps, g)[0]
        except IrxError:
            raise
        except Exception as e:
            logger.warning(f"Stable Diffusion colorization failed: {e}, using fallback", exc_info=True)
            return self._colorize_lab(image)

    def _colorize_lab(self, image: Image.Image) -> Image.Image:
        try:
            if self.device.startswith("cuda"):     # L + 256-entry colour map on the GPU (same bytes)
                from . import nlmeans
                x = torch.from_numpy(np.array(image.convert("RGB"))).to(self.device)
                return Image.fromarray(nlmeans.colorize_lab(x).cpu().numpy())
            return classical.colorize_lab(image)
        except IrxError:
            raise
        except Exception as e:
            logger.warning(f"LAB colorization failed: {e}, returning grayscale as RGB")
            return image

    # ------------------------------------------------------------------------------------ inpaint
    def inpaint(self, image: Image.Image, mask: Image.Image = None, prompt: str = None, **kwargs) -> Image.Image:
        if "inpaint" not in self.models:
            self.load_inpaint_model()
        model = self.models.get("inpaint")
        if model is None:
            logger.warning("Inpainting model not available, returning original")
            return image
        if prompt is None:
            prompt = kwargs.get("prompt", self.prompts["inpaint"])
        if mask is None:
            mask = self._auto_mask_from_image(image)
            if mask is None:
                return image
        mask = self._normalize_mask(mask, image.size)
        if isinstance(model, NativeSDModel):
            return self._inpaint_sd(image, model, mask, prompt=prompt)
        return image

    def _inpaint_sd(self, image: Image.Image, model, mask: Image.Image, prompt: str) -> Image.Image:
        try:
            s, steps, g = SD_PARAMS["inpaint"]
            return self._inpaint_native(model, [image], [mask], prompt, s, steps, g)[0]
        except IrxError:
            raise
        except Exception:
            logger.error("Error in inpainting", exc_info=True)
            return image

    def _normalize_mask(self, mask: Image.Image, target_size: tuple[int, int]) -> Image.Image:
        return ip.normalize_mask(mask, target_size)

    def _auto_mask_from_image(self, image: Image.Image) -> Image.Image | None:
        if self.device.startswith("cuda"):         # threshold + close + open + count on the GPU
            from . import nlmeans
            x = torch.from_numpy(np.array(image.convert("RGB"))).to(self.device)
            mk, keep = nlmeans.auto_mask(x)
            m = Image.fromarray(mk.cpu().numpy()).convert("L") if keep else None
        else:
            m = classical.auto_mask(image)
        if m is None:
            logger.info("No significant damage detected, skipping inpainting")
        return m

    # ------------------------------------------------------------------------------------ chains
    def process(self, image: Image.Image, tasks: list[Task], **kwargs: Any) -> dict[str, Image.Image]:
        results = {"original": image, "final": image}
        current = image
        for task in tasks:
            try:
                if task == "denoise":
                    current = self.denoise(current, strength=kwargs.get("denoise_strength", 0.5),
                                           prompt=kwargs.get("denoise_prompt", None))
                    results["denoised"] = current
                elif task in ("sr", "super_resolution"):
                    current = self.super_resolve(current, scale=kwargs.get("sr_scale", 4),
                                                 prompt=kwargs.get("sr_prompt", None))
                    results["super_resolved"] = current
                elif task == "colorize":
                    cp = kwargs.get("colorize_prompt")
                    current = self.colorize(current, prompt=cp) if cp else self.colorize(current)
                    results["colorized"] = current
                elif task == "inpaint":
                    current = self.inpaint(current, mask=kwargs.get("mask", None),
                                           prompt=kwargs.get("inpaint_prompt", None))
                    results["inpainted"] = current
            except IrxError:
                raise
            except Exception:
                logger.error(f"Error processing task {task}", exc_info=True)
                continue
        results["final"] = current
        return results

    # ------------------------------------------------------------------------------------ batched API
    def restore_batch(self, task: str, images: Sequence[Image.Image], masks: Optional[Sequence] = None,
                      prompt: Optional[str] = None, strength: Optional[float] = None,
                      max_batch: int = 8) -> List[Image.Image]:
        """Batched form of the single-image entry points (new; the reference loops one image per call).
        Images of equal processed size run as one engine batch of up to `max_batch`; each image gets the
        result the single-image call returns (per-call reseeded noise).  The result does not depend on the
        batch an image shares: every tile / split-K / GroupNorm-chunking decision is made for a canonical
        16-image batch of the per-image shape and GroupNorm partials are per image, so batch 8
        == 3 + 5 bit for bit on every engine (tests/test_batch_invariance_gpu.py).  Falls back to the
        single-image entry point per image (with the caller's prompt) whenever that one would not take the
        diffusion path."""
        task = "sr" if task == "super_resolution" else task
        loader = {"denoise": self.load_denoise_model, "sr": self.load_sr_model,
                  "colorize": self.load_colorize_model, "inpaint": self.load_inpaint_model}[task]
        loader()
        model = self.models.get(task)
        pk = {"prompt": prompt} if prompt else {}
        single = {"denoise": lambda im, mk: self.denoise(im, **({"strength": strength} if strength is not None
                                                                else {}), **pk),
                  "sr": lambda im, mk: self.super_resolve(im, **pk),
                  "colorize": lambda im, mk: self.colorize(im, **pk),
                  "inpaint": lambda im, mk: self.inpaint(im, mask=mk, **pk)}[task]
        masks = list(masks) if masks is not None else [None] * len(images)
        if not isinstance(model, NativeSDModel):
            return [single(im, mk) for im, mk in zip(images, masks)]
        out: List[Optional[Image.Image]] = [None] * len(images)
        groups: Dict[tuple, List[int]] = {}
        prepared = {}
        for i, (im, mk) in enumerate(zip(images, masks)):
            if task == "colorize":
                if self.is_color(im):
                    out[i] = im
                    continue
                im = self.gray_to_rgb(im)
            if task == "sr":
                im = self._cap_area(im)
            if task == "inpaint":
                if mk is None:
                    out[i] = single(im, mk)
                    continue
                mk = self._normalize_mask(mk, im.size)
            prepared[i] = (im, mk)
            groups.setdefault(ip.target_size(im) if task != "inpaint" else (INPAINT_SIZE,) * 2, []).append(i)
        s_default, steps, g = SD_PARAMS[task]
        s = strength if strength is not None else (0.5 if task == "denoise" else s_default)
        p = prompt or self.prompts[task]
        for _, idx in groups.items():
            for k in range(0, len(idx), max_batch):
                chunk = idx[k:k + max_batch]
                ims = [prepared[i][0] for i in chunk]
                try:
                    if task == "inpaint":
                        res = self._inpaint_native(model, ims, [prepared[i][1] for i in chunk], p, s, steps, g)
                    else:
                        res = self._img2img(model, ims, p, s, steps, g)
                except IrxError:
                    raise
                except Exception as e:     # as the single-image entry points: log, then their fallbacks
                    logger.warning(f"batched {task} failed ({e}); running the single-image entry point per image")
                    res = [single(images[i], masks[i]) for i in chunk]
                for i, r in zip(chunk, res):
                    out[i] = r
        return out  # type: ignore[return-value]
