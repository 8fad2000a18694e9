"""Batched SD-1.5 img2img / inpaint orchestration over the native engine.

Restates the control flow of diffusers 0.35.2 `StableDiffusionImg2ImgPipeline.__call__` and
`StableDiffusionInpaintPipeline.__call__` — the calls the reference
makes at `src/inference.py:486-495, :566-573, :664-672, :758-767` — for a batch of images that
share a prompt.  Everything between the uint8 input pixels and the uint8 output pixels runs on the
GPU through libirx: pixel normalisation, VAE encode, posterior sampling + add_noise, CLIP text
encoding, the denoising loop (UNet + fused CFG/scheduler/pack step kernel), VAE decode and the
uint8 post-processing.  The host only resizes with PIL, draws the seeded noise (CPU
`torch.Generator`, exactly like the reference on a CPU device) and plans scheduler coefficients.

Every image gets the noise of a fresh `Generator.manual_seed(seed)`, because the reference
reseeds per call (`src/inference.py:482-483, :562-563, :660-661, :754-755`) and calls the
pipeline once per image.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib as L
from . import image_processor as ip
from . import weights as W
from .configs import PipelineConfig
from .engine import CLIPText, UNet, VAE, TORCH_DT, dtype_code
from .schedulers import make_planner, StepPlan
from .tokenizer import PromptTokenizer


@dataclass
class BatchResult:
    images_u8: torch.Tensor                 # [B, H, W, 3] uint8 (device)
    decoded01: Optional[torch.Tensor]       # [B, H, W, 3] fp32 in [0, 1] before rounding (device) or None
    latents: torch.Tensor                   # [B, h, w, 4] fp32 final latents (device)
    timesteps: List[int]


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def draw_noise(seed: int, h: int, w: int, n: int) -> List[torch.Tensor]:
    """The reference's RNG draws for one image: n x randn(1, 4, h, w) from Generator('cpu').manual_seed(seed),
    returned as NHWC [h, w, 4] fp32 (CPU)."""
    g = torch.Generator("cpu").manual_seed(seed)
    out = []
    for _ in range(n):
        e = torch.randn((1, 4, h, w), generator=g, dtype=torch.float32)
        out.append(e[0].permute(1, 2, 0).contiguous())
    return out


class SDEngine:
    """The three native models of one task directory + the batched denoising loop."""

    def __init__(self, cfg: PipelineConfig, dtype="bf16", device="cuda", weights="random", weight_seed: int = 0,
                 state_dicts: Optional[Dict[str, Dict[str, torch.Tensor]]] = None, vae_dtype=None, clip_dtype=None):
        """`dtype` is the UNet's compute type (and the default of the other two models); `vae_dtype` /
        `clip_dtype` override it per model (e.g. a bf16 UNet with an fp16 VAE)."""
        self.cfg = cfg
        self.dt = dtype_code(dtype)
        self.tdt = TORCH_DT[self.dt]
        self.vdt = dtype_code(vae_dtype) if vae_dtype is not None else self.dt     # VAE + its pixel / latent I/O
        self.vtdt = TORCH_DT[self.vdt]
        self.cdt = dtype_code(clip_dtype) if clip_dtype is not None else self.dt
        self.device = torch.device(device)
        self.unet = UNet(cfg.unet, self.dt, self.device)
        self.vae = VAE(cfg.vae, self.vdt, self.device)
        self.clip = CLIPText(cfg.clip, self.cdt, self.device)
        if state_dicts is None:
            state_dicts = self._load_weights(weights, weight_seed)
        if state_dicts is not None:
            self.unet.load_state_dict(state_dicts["unet"])
            self.vae.load_state_dict(state_dicts["vae"])
            self.clip.load_state_dict(state_dicts["clip"])
        tok_dir = Path(cfg.model_dir) / "tokenizer" if cfg.model_dir else None
        self.tokenizer = PromptTokenizer(tok_dir)
        self._ctx_cache: Dict[tuple, torch.Tensor] = {}
        # HIP-graph replay of repeated denoising loops (IRX_GRAPHS=0 disables)
        self.use_graphs = os.environ.get("IRX_GRAPHS", "1") != "0" and self.device.type == "cuda"
        self._graphs: Dict[tuple, dict] = {}
        self._graph_stream = torch.cuda.Stream(self.device) if self.use_graphs else None

    def __del__(self):
        for g in getattr(self, "_graphs", {}).values():
            try:
                L.load().irx_graph_destroy(g["exec"])
            except Exception:
                pass

    # ------------------------------------------------------------------ weights
    def _load_weights(self, weights, seed):
        if weights == "none":
            return None          # caller binds blobs itself (e.g. after an RCCL broadcast)
        if weights == "random":
            return {k: W.random_state_dict(k, getattr(self.cfg, k), seed) for k in ("unet", "vae", "clip")}
        root = Path(weights if weights != "dir" else self.cfg.model_dir)
        sds = {"unet": W.load_component_dir(root / "unet"), "vae": W.load_component_dir(root / "vae"),
               "clip": W.load_component_dir(root / "text_encoder")}
        for k in sds:
            W.check_state_dict(k, getattr(self.cfg, k), sds[k])
        return sds

    def models(self):
        return {"unet": self.unet, "vae": self.vae, "clip": self.clip}

    # ------------------------------------------------------------------ text
    def text_embeddings(self, prompt: str, cfg_on: bool, negative: str = "") -> torch.Tensor:
        """encode_prompt: [neg, pos] (CFG) or [pos] -> [n, 77, 768] (dtype, device)."""
        key = (prompt, negative, cfg_on)
        if key not in self._ctx_cache:
            ids = [self.tokenizer(negative), self.tokenizer(prompt)] if cfg_on else [self.tokenizer(prompt)]
            ids = torch.from_numpy(np.stack(ids))
            emb = self.clip.encode(ids)
            self._ctx_cache[key] = emb if emb.dtype == self.tdt else emb.to(self.tdt)
        return self._ctx_cache[key]

    def context_kv(self, emb: torch.Tensor, batch: int) -> torch.Tensor:
        """UNet batch rows are [uncond x B, cond x B] (CFG) -> per-row cross-attention K|V."""
        ctx = emb.repeat_interleave(batch, dim=0).contiguous()
        return self.unet.prepare_context(ctx)

    # ------------------------------------------------------------------ building blocks
    def to_tensor(self, u8: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, H, W_, _ = u8.shape
        out = torch.empty((B, H, W_, 8), dtype=self.vtdt, device=self.device)
        L.call("irx_image_to_tensor", _stream(), self.vdt, _p(u8), _p(mask), B, H, W_, 8, _p(out))
        return out

    def sample_latents(self, moments: torch.Tensor, eps: torch.Tensor, noise: Optional[torch.Tensor],
                       a: float = 1.0, b: float = 0.0) -> torch.Tensor:
        B, h, w, _ = moments.shape
        out = torch.empty((B, h, w, 4), dtype=torch.float32, device=self.device)
        L.call("irx_latent_sample", _stream(), self.vdt, _p(moments), B, h, w, _p(eps), _p(noise), 1,
               float(self.cfg.vae.scaling_factor), float(a), float(b), _p(out))
        return out

    def decode(self, lat: torch.Tensor, want_float: bool) -> tuple:
        B, h, w, _ = lat.shape
        z = torch.empty((B, h, w, 8), dtype=self.vtdt, device=self.device)
        L.call("irx_latents_to_vae", _stream(), self.vdt, _p(lat), B, h, w, float(self.cfg.vae.scaling_factor), _p(z))
        img = self.vae.decode(z)
        H, W_ = h * 8, w * 8
        u8 = torch.empty((B, H, W_, 3), dtype=torch.uint8, device=self.device)
        f01 = torch.empty((B, H, W_, 3), dtype=torch.float32, device=self.device) if want_float else None
        L.call("irx_tensor_to_image", _stream(), self.vdt, _p(img), B, H, W_, 4, _p(u8), _p(f01))
        return u8, f01

    def _loop_buffers(self, lat: torch.Tensor, plans: List[StepPlan], cfg_on: bool) -> dict:
        B, h, w, _ = lat.shape
        UB = 2 * B if cfg_on else B
        n_slots = max([(-1 if p.store_slot is None else p.store_slot) for p in plans] + [-1]) + 1
        return {
            "x_in": torch.empty((UB, h, w, self.unet.cin_pad), dtype=self.tdt, device=self.device),
            "eps": torch.empty((UB, h, w, 4), dtype=torch.float32, device=self.device),
            "slots": [torch.empty_like(lat) for _ in range(n_slots)],
            "cur": torch.empty_like(lat) if any(p.save_cur for p in plans) else None,
            "t_all": torch.tensor([[float(p.t)] * UB for p in plans], dtype=torch.float32).to(self.device),
        }

    def denoise_loop(self, lat: torch.Tensor, kv: torch.Tensor, plans: List[StepPlan], guidance: float,
                     cfg_on: bool, mask_l: Optional[torch.Tensor] = None,
                     masked_l: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The denoising loop.  With `use_graphs`, the first call of a loop (shapes, plans, guidance) runs eagerly
        on the engine's stream and then records the same loop as one HIP graph (irx_graph_*) into persistent
        buffers — host-only work that overlaps the eager kernels still queued on the GPU; every later call
        replays it: ~600 launches per UNet eval issued by one hipGraphLaunch."""
        if not self.use_graphs or not lat.is_cuda:
            return self._loop_body(lat, kv, plans, guidance, cfg_on, mask_l, masked_l,
                                   self._loop_buffers(lat, plans, cfg_on))
        # the graph bakes in the UNet weight-blob pointer: the bound blob is part of the key (and each entry holds a
        # reference to it, so a rebind can neither replay stale weights nor let the old blob be freed under it)
        key = (self.unet.blob.data_ptr(), tuple(lat.shape), tuple(kv.shape), bool(cfg_on), float(guidance),
               mask_l is not None,
               tuple((p.t, p.mode, tuple(p.c), tuple(p.hw), p.e_div, p.e_mul, p.store_slot, tuple(p.hist),
                      p.x_from_cur, p.save_cur) for p in plans))
        cs = torch.cuda.current_stream(self.device)
        gs = self._graph_stream
        gs.wait_stream(cs)
        with torch.cuda.stream(gs):
            g = self._graphs.get(key)
            if g is None:
                # first sight: eager on the graph stream (sizes the workspaces, creates its split-K tickets), then
                # record the graph for the next call while those kernels run
                out = self._loop_body(lat, kv, plans, guidance, cfg_on, mask_l, masked_l,
                                      self._loop_buffers(lat, plans, cfg_on))
                self._capture(key, lat, kv, plans, guidance, cfg_on, mask_l, masked_l)
            else:
                g["lat"].copy_(lat)
                g["kv"].copy_(kv)
                if mask_l is not None:
                    g["mask"].copy_(mask_l)
                    g["masked"].copy_(masked_l)
                L.call("irx_graph_launch", g["exec"], _stream())
                out = g["lat"].clone()
        cs.wait_stream(gs)
        return out

    def _capture(self, key, lat, kv, plans, guidance, cfg_on, mask_l, masked_l) -> dict:
        g = {"lat": torch.empty_like(lat), "kv": torch.empty_like(kv),
             "mask": torch.empty_like(mask_l) if mask_l is not None else None,
             "masked": torch.empty_like(masked_l) if masked_l is not None else None,
             "bufs": self._loop_buffers(lat, plans, cfg_on)}
        h = C.c_void_p()
        L.call("irx_graph_begin", _stream())
        try:
            self._loop_body(g["lat"], g["kv"], plans, guidance, cfg_on, g["mask"], g["masked"], g["bufs"])
        except BaseException:
            L.load().irx_graph_end(_stream(), C.byref(h))   # leave capture mode, drop the partial graph
            if h.value:
                L.call("irx_graph_destroy", h)
            raise
        L.call("irx_graph_end", _stream(), C.byref(h))
        g["exec"] = h
        g["ws"] = self.unet._ws          # the workspace the graph's launches point into stays alive with it
        g["blob"] = self.unet.blob       # ... and so do the weights they read
        while len(self._graphs) >= 4:                         # a few loop shapes per engine
            old = self._graphs.pop(next(iter(self._graphs)))
            # a replay of the evicted exec may still be queued on this stream: drain it before destroying
            torch.cuda.current_stream(self.device).synchronize()
            L.call("irx_graph_destroy", old["exec"])
        self._graphs[key] = g
        return g

    def _loop_body(self, lat, kv, plans, guidance, cfg_on, mask_l, masked_l, bufs) -> torch.Tensor:
        B, h, w, _ = lat.shape
        UB = 2 * B if cfg_on else B
        inpaint = int(mask_l is not None)
        cp = self.unet.cin_pad
        x_in, eps, slots, cur, t_all = bufs["x_in"], bufs["eps"], bufs["slots"], bufs["cur"], bufs["t_all"]
        L.call("irx_pack_unet_input", _stream(), self.dt, _p(lat), B, h, w, int(cfg_on), cp, inpaint, _p(mask_l),
               _p(masked_l), _p(x_in))
        for i, p in enumerate(plans):
            self.unet.forward(x_in, t_all[i], kv, 77, out=eps)
            sp = L.StepParams()
            sp.dtype, sp.batch, sp.h, sp.w = self.dt, B, h, w
            sp.eps, sp.cfg, sp.guidance = eps.data_ptr(), int(cfg_on), float(guidance)
            sp.hist_store = slots[p.store_slot].data_ptr() if p.store_slot is not None else None
            for k in range(4):
                sp.hist[k] = slots[p.hist[k]].data_ptr() if p.hist[k] is not None else None
            for k in range(5):
                sp.hw[k] = float(p.hw[k])
            sp.e_div, sp.e_mul = float(p.e_div), float(p.e_mul)
            sp.mode = p.mode
            sp.c0, sp.c1, sp.c2, sp.c3 = (float(v) for v in p.c)
            sp.x_src = (cur if p.x_from_cur else lat).data_ptr()
            sp.cur_store = cur.data_ptr() if p.save_cur else None
            sp.x_out = lat.data_ptr()
            last = i + 1 == len(plans)
            sp.unet_in = None if last else x_in.data_ptr()
            sp.cin_pad, sp.inpaint = cp, inpaint
            sp.mask, sp.masked = (mask_l.data_ptr() if inpaint else None), (masked_l.data_ptr() if inpaint else None)
            L.call("irx_sched_step", _stream(), C.byref(sp))
        return lat

    # ------------------------------------------------------------------ pipelines
    def img2img(self, u8: torch.Tensor, prompt: str, strength: float, steps: int, guidance: float, seed: int = 42,
                want_float: bool = False, n_evals: Optional[int] = None,
                noise: Optional[Sequence[torch.Tensor]] = None) -> BatchResult:
        """u8: device uint8 [B, H, W, 3], H and W multiples of 8 (already preprocessed)."""
        if not 0 <= strength <= 1:
            raise ValueError(f"The value of strength should in [0.0, 1.0] but is {strength}")
        if prompt is None:
            raise ValueError("Provide either `prompt` or `prompt_embeds`.")
        B, H, W_, _ = u8.shape
        h, w = H // 8, W_ // 8
        cfg_on = guidance > 1.0
        planner = make_planner(self.cfg.scheduler)
        planner.set_timesteps(steps)
        ts, _ = planner.get_timesteps(steps, strength)
        if len(ts) == 0:
            raise ValueError("strength too small: no denoising steps")
        plans = planner.plan(ts)
        if n_evals is not None:
            plans = plans[:n_evals]
        emb = self.text_embeddings(prompt, cfg_on)
        kv = self.context_kv(emb, B)
        if noise is None:
            noise = draw_noise(seed, h, w, 2)
        eps1, nz = (x.to(self.device) for x in noise[:2])
        img = self.to_tensor(u8)
        mom = self.vae.encode(img)
        a, b = planner.add_noise_coeffs(int(ts[0]))
        lat = self.sample_latents(mom, eps1, nz, a, b)
        lat = self.denoise_loop(lat, kv, plans, guidance, cfg_on)
        u8o, f01 = self.decode(lat, want_float)
        return BatchResult(u8o, f01, lat, [p.t for p in plans])

    def inpaint(self, u8: torch.Tensor, mask01: torch.Tensor, prompt: str, strength: float, steps: int,
                guidance: float, seed: int = 42, want_float: bool = False,
                n_evals: Optional[int] = None) -> BatchResult:
        """u8: device uint8 [B, H, W, 3] at the processor size; mask01: fp32 [B, H, W] of {0,1} (1 = inpaint)."""
        B, H, W_, _ = u8.shape
        h, w = H // 8, W_ // 8
        cfg_on = guidance > 1.0
        planner = make_planner(self.cfg.scheduler)
        planner.set_timesteps(steps)
        ts, n = planner.get_timesteps(steps, strength)
        if n < 1:
            raise ValueError("strength too small: no denoising steps")
        plans = planner.plan(ts)
        if n_evals is not None:
            plans = plans[:n_evals]
        emb = self.text_embeddings(prompt, cfg_on)
        kv = self.context_kv(emb, B)
        is_max = strength == 1.0
        draws = draw_noise(seed, h, w, 2 if is_max else 3)
        draws = [d.to(self.device) for d in draws]
        img = self.to_tensor(u8)
        if is_max:
            nz, e3 = draws
            # latents = noise * init_noise_sigma (1.0): a z-free sample (moments unused -> pass zeros)
            lat = nz.unsqueeze(0).expand(B, h, w, 4).contiguous()
        else:
            e1, nz, e3 = draws
            mom = self.vae.encode(img)
            a, b = planner.add_noise_coeffs(int(ts[0]))
            lat = self.sample_latents(mom, e1, nz, a, b)
        masked_img = self.to_tensor(u8, mask01.contiguous())
        mom2 = self.vae.encode(masked_img)
        masked_l = self.sample_latents(mom2, e3, None)
        mask_l = torch.from_numpy(ip.nearest_downsample(mask01.cpu().numpy(), h, w)).to(self.device).contiguous()
        lat = self.denoise_loop(lat, kv, plans, guidance, cfg_on, mask_l, masked_l)
        u8o, f01 = self.decode(lat, want_float)
        return BatchResult(u8o, f01, lat, [p.t for p in plans])
