"""Diffusion schedulers as per-step coefficient tables for one fused device kernel (K11).

Every scheduler used here (DDIM η=0, PNDM/PLMS with ``skip_prk_steps`` — SD-1.5's default —
and Euler-discrete — SDXL's default) is, per step, *linear* in the latent x, a saved latent
XS, the current CFG-combined noise estimate e and up to three earlier e's.  So each scheduler
is compiled on the host into a ``[steps, 16]`` fp32 table and the device runs ONE elementwise
kernel per step (``ops.latent_step``) that

    e_cur = eps_u + g (eps_c - eps_u)                          (classifier-free guidance)
    e'    = w_cur e_cur + w1 H[s1] + w2 H[s2] + w3 H[s3]        (multistep history)
    x     = ax x + axs XS + b e'
    H[save] = e_cur;  XS = x_old (if save_x);  unet_in = c_in_next * x  (bf16, duplicated ×2 for CFG)

reading its row through a device step counter, so a whole denoise step (UNet + this kernel +
counter bump) is captured once as a hipGraph and replayed per step with no host sync.

Row layout (floats): 0 w_cur, 1 w1, 2 w2, 3 w3, 4 ax, 5 axs, 6 b, 7 c_in_next, 8 s1, 9 s2,
10 s3, 11 save_slot(-1 none), 12 save_x, 13 guidance, 14 t_model (UNet timestep), 15 unused.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Tuple

import numpy as np
import torch

ROW = 16


def scaled_linear_alphas_cumprod(beta_start=0.00085, beta_end=0.012, n=1000) -> np.ndarray:
    betas = np.linspace(beta_start ** 0.5, beta_end ** 0.5, n, dtype=np.float64) ** 2
    return np.cumprod(1.0 - betas)


@dataclass
class SchedulePlan:
    table: np.ndarray          # [evals, 16]
    init_sigma: float          # initial latent scale (noise * init_sigma)
    c_in0: float               # model-input scale for the first evaluation
    name: str

    @property
    def evals(self) -> int:
        return self.table.shape[0]

    def timesteps(self) -> np.ndarray:
        return self.table[:, 14].copy()


def _row(**kw) -> np.ndarray:
    r = np.zeros(ROW, dtype=np.float64)
    r[8:12] = -1
    names = dict(w_cur=0, w1=1, w2=2, w3=3, ax=4, axs=5, b=6, c_in_next=7, s1=8, s2=9, s3=10,
                 save=11, save_x=12, guidance=13, t=14)
    for k, v in kw.items():
        r[names[k]] = v
    return r


def ddim_plan(steps: int, guidance: float, offset: int = 1) -> SchedulePlan:
    acp = scaled_linear_alphas_cumprod()
    ratio = 1000 // steps
    ts = (np.arange(0, steps) * ratio)[::-1] + offset
    final = acp[0]                                  # set_alpha_to_one=False
    rows = []
    for i, t in enumerate(ts):
        a_t = acp[t]
        a_p = acp[ts[i + 1]] if i + 1 < len(ts) else final
        ax = math.sqrt(a_p / a_t)
        b = math.sqrt(1 - a_p) - math.sqrt(a_p) * math.sqrt(1 - a_t) / math.sqrt(a_t)
        rows.append(_row(w_cur=1, ax=ax, b=b, c_in_next=1.0, guidance=guidance, t=t))
    return SchedulePlan(np.stack(rows).astype(np.float32), 1.0, 1.0, "ddim")


def pndm_plan(steps: int, guidance: float, offset: int = 1) -> SchedulePlan:
    """PLMS with skip_prk_steps (diffusers PNDMScheduler semantics) → steps+1 evaluations."""
    acp = scaled_linear_alphas_cumprod()
    final = acp[0]
    ratio = 1000 // steps
    _ts = np.arange(0, steps) * ratio + offset
    plms = np.concatenate([_ts[:-1], _ts[-2:-1], _ts[-1:]])[::-1]
    rows = []
    ets: List[int] = []      # ring slots of history, oldest first
    n_app = 0
    for counter, t in enumerate(plms):
        t = int(t)
        prev_t = t - ratio
        save = -1
        if counter != 1:
            slot = n_app % 4
            n_app += 1
            ets = ets[-3:] + [slot]
            save = slot
        else:
            prev_t = t
            t = t + ratio
        w = dict(w_cur=0.0, w1=0.0, w2=0.0, w3=0.0, s1=-1, s2=-1, s3=-1)
        ax, axs, save_x = 1.0, 0.0, 0
        if len(ets) == 1 and counter == 0:
            w["w_cur"] = 1.0
            save_x = 1
        elif len(ets) == 1 and counter == 1:
            w.update(w_cur=0.5, w1=0.5, s1=ets[-1])
            ax, axs = 0.0, 1.0                       # sample = cur_sample
        elif len(ets) == 2:
            w.update(w_cur=1.5, w1=-0.5, s1=ets[-2])
        elif len(ets) == 3:
            w.update(w_cur=23 / 12, w1=-16 / 12, s1=ets[-2], w2=5 / 12, s2=ets[-3])
        else:
            w.update(w_cur=55 / 24, w1=-59 / 24, s1=ets[-2], w2=37 / 24, s2=ets[-3], w3=-9 / 24, s3=ets[-4])
        a_t = acp[t]
        a_p = acp[prev_t] if prev_t >= 0 else final
        beta_t, beta_p = 1 - a_t, 1 - a_p
        sc = (a_p / a_t) ** 0.5
        denom = a_t * beta_p ** 0.5 + (a_t * beta_t * a_p) ** 0.5
        b = -(a_p - a_t) / denom
        rows.append(_row(ax=ax * sc, axs=axs * sc, b=b, c_in_next=1.0, save=save, save_x=save_x,
                         guidance=guidance, t=int(plms[counter]), **w))
    return SchedulePlan(np.stack(rows).astype(np.float32), 1.0, 1.0, "pndm")


def euler_plan(steps: int, guidance: float, offset: int = 1) -> SchedulePlan:
    """EulerDiscrete, epsilon prediction, 'leading' spacing (SDXL defaults)."""
    acp = scaled_linear_alphas_cumprod()
    all_sig = np.sqrt((1 - acp) / acp)
    ratio = 1000 // steps
    ts = (np.arange(0, steps) * ratio).round()[::-1].astype(np.float64) + offset
    sig = np.interp(ts, np.arange(1000), all_sig)
    sig = np.concatenate([sig, [0.0]])
    init_sigma = math.sqrt(sig.max() ** 2 + 1)
    rows = []
    for i, t in enumerate(ts):
        dt = sig[i + 1] - sig[i]
        c_next = 1.0 / math.sqrt(sig[i + 1] ** 2 + 1) if i + 1 < len(ts) else 1.0
        rows.append(_row(w_cur=1, ax=1.0, b=dt, c_in_next=c_next, guidance=guidance, t=t))
    return SchedulePlan(np.stack(rows).astype(np.float32), init_sigma, 1.0 / math.sqrt(sig[0] ** 2 + 1), "euler")


def make_plan(name: str, steps: int, guidance: float) -> SchedulePlan:
    return {"ddim": ddim_plan, "pndm": pndm_plan, "euler": euler_plan}[name](steps, guidance)


def latent_step_reference(eps, x, hist, xs, coef, step, unet_in, cfg: bool) -> None:
    """PyTorch semantics of the fused latent-step kernel (in place)."""
    i = int(step.item())
    r = coef[i].double().tolist()
    if cfg:
        u, c = eps.float().chunk(2)
        e = u + r[13] * (c - u)
    else:
        e = eps.float()
    ep = r[0] * e
    for wi, si in ((1, 8), (2, 9), (3, 10)):
        if r[si] >= 0 and r[wi] != 0:
            ep = ep + r[wi] * hist[int(r[si])]
    x_old = x.clone()
    x.copy_(r[4] * x_old + r[5] * xs + r[6] * ep)
    if r[11] >= 0:
        hist[int(r[11])].copy_(e)
    if r[12] > 0:
        xs.copy_(x_old)
    nxt = (r[7] * x).to(unet_in.dtype)
    C = x.shape[-1]                  # unet_in may carry zero padding channels beyond C
    if cfg:
        B = x.shape[0]
        unet_in[:B, ..., :C].copy_(nxt)
        unet_in[B:, ..., :C].copy_(nxt)
    else:
        unet_in[..., :C].copy_(nxt)
