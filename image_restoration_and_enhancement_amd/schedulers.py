"""Host-side scheduler state machines; the arithmetic runs in the fused `irx_sched_step` kernel.

Restates diffusers 0.35.2 `PNDMScheduler` (skip_prk_steps, leading spacing, steps_offset 1 — the
saved config `outputs/models/denoising/best/scheduler/scheduler_config.json:2-13`) and
`DDIMScheduler` (eta 0 — `outputs/models/inpainting/best/scheduler/scheduler_config.json:2-18`),
SURVEY.md Appendix A.3-A.5.  Per step the host decides *which* history entries and scalar
coefficients apply (all scalar math in float32 exactly as diffusers computes it with 0-d torch
tensors); the device kernel combines CFG, the PLMS multistep sum and the update in one pass.
The PNDM img2img quirk (the duplicated step is sliced away but the counter==1 branch still
fires on the 2nd executed step) is reproduced, not fixed.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np
import torch

from .configs import SchedulerConfig


def alphas_cumprod(cfg: SchedulerConfig) -> torch.Tensor:
    betas = torch.linspace(cfg.beta_start ** 0.5, cfg.beta_end ** 0.5, cfg.num_train_timesteps,
                           dtype=torch.float32) ** 2
    return torch.cumprod(1.0 - betas, dim=0)


def _f(x) -> float:
    return float(x.item() if isinstance(x, torch.Tensor) else x)


@dataclass
class StepPlan:
    """Everything the fused step kernel needs for one denoising step."""
    t: int                         # the UNet timestep of this step
    mode: int                      # 0 PNDM, 1 DDIM
    c: Tuple[float, float, float, float]
    hw: Tuple[float, ...] = (1.0, 0.0, 0.0, 0.0, 0.0)
    hist: Tuple[Optional[int], ...] = (None, None, None, None)   # history slot per hw[1..4]
    e_div: float = 1.0
    e_mul: float = 1.0
    store_slot: Optional[int] = None   # slot the CFG-combined eps is stored into
    x_from_cur: bool = False           # PNDM counter==1: update applies to the saved cur_sample
    save_cur: bool = False             # PNDM counter==0: save the sample as cur_sample


class _Base:
    order = 1

    def __init__(self, cfg: SchedulerConfig):
        self.cfg = cfg
        self.alphas_cumprod = alphas_cumprod(cfg)
        self.final_alpha_cumprod = torch.tensor(1.0) if cfg.set_alpha_to_one else self.alphas_cumprod[0]
        self.timesteps = np.zeros(0, dtype=np.int64)
        self.num_inference_steps = 0

    def add_noise_coeffs(self, t: int) -> Tuple[float, float]:
        a = self.alphas_cumprod[int(t)]
        return _f(a ** 0.5), _f((1 - a) ** 0.5)

    def get_timesteps(self, n: int, strength: float) -> Tuple[np.ndarray, int]:
        """StableDiffusion{Img2Img,Inpaint}Pipeline.get_timesteps."""
        init = min(int(n * strength), n)
        t_start = max(n - init, 0)
        return self.timesteps[t_start * self.order:], n - t_start

    def _alpha(self, t: int):
        return self.alphas_cumprod[t] if t >= 0 else self.final_alpha_cumprod


class PNDMPlanner(_Base):
    N_SLOTS = 5

    def set_timesteps(self, n: int) -> None:
        self.num_inference_steps = n
        ratio = self.cfg.num_train_timesteps // n
        ts = (np.arange(0, n) * ratio).round() + self.cfg.steps_offset
        plms = np.concatenate([ts[:-1], ts[-2:-1], ts[-1:]])[::-1].copy()
        self.timesteps = plms.astype(np.int64)

    def plan(self, ts: np.ndarray) -> List[StepPlan]:
        ratio = self.cfg.num_train_timesteps // self.num_inference_steps
        ets: List[int] = []          # slot ids, oldest first
        counter = 0
        plans = []
        for t0 in ts:
            t = int(t0)
            prev_t = t - ratio
            store = None
            if counter != 1:
                ets = ets[-3:]
                store = next(s for s in range(self.N_SLOTS) if s not in ets)
                ets = ets + [store]
            else:
                prev_t = t
                t = t + ratio
            p = StepPlan(t=int(t0), mode=0, c=(0, 0, 0, 0), store_slot=store)
            n = len(ets)
            if n == 1 and counter == 0:
                p.save_cur = True
            elif n == 1 and counter == 1:
                p.hw, p.hist, p.e_div, p.x_from_cur = (1.0, 1.0, 0, 0, 0), (ets[-1], None, None, None), 2.0, True
            elif n == 2:
                p.hw, p.hist, p.e_div = (3.0, -1.0, 0, 0, 0), (ets[-2], None, None, None), 2.0
            elif n == 3:
                p.hw, p.hist, p.e_div = (23.0, -16.0, 5.0, 0, 0), (ets[-2], ets[-3], None, None), 12.0
            else:
                p.hw, p.hist = (55.0, -59.0, 37.0, -9.0, 0), (ets[-2], ets[-3], ets[-4], None)
                p.e_mul = float(np.float32(1 / 24))
            a_t, a_p = self._alpha(t), self._alpha(prev_t)
            b_t, b_p = 1 - a_t, 1 - a_p
            sc = (a_p / a_t) ** 0.5
            denom = a_t * b_p ** 0.5 + (a_t * b_t * a_p) ** 0.5
            p.c = (_f(sc), _f(a_p - a_t), _f(denom), 0.0)
            plans.append(p)
            counter += 1
        return plans


class DDIMPlanner(_Base):
    N_SLOTS = 0

    def set_timesteps(self, n: int) -> None:
        self.num_inference_steps = n
        ratio = self.cfg.num_train_timesteps // n
        ts = (np.arange(0, n) * ratio).round()[::-1].copy().astype(np.int64)
        self.timesteps = ts + self.cfg.steps_offset

    def plan(self, ts: np.ndarray) -> List[StepPlan]:
        ratio = self.cfg.num_train_timesteps // self.num_inference_steps
        plans = []
        for t0 in ts:
            t = int(t0)
            a_t, a_p = self._alpha(t), self._alpha(t - ratio)
            b_t = 1 - a_t
            std = torch.tensor(0.0)                        # eta = 0
            plans.append(StepPlan(t=t, mode=1, c=(_f(b_t ** 0.5), _f(a_t ** 0.5), _f(a_p ** 0.5),
                                                  _f((1 - a_p - std ** 2) ** 0.5))))
        return plans


def make_planner(cfg: SchedulerConfig):
    return PNDMPlanner(cfg) if cfg.kind == "pndm" else DDIMPlanner(cfg)
