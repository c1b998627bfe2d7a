"""Plain-PyTorch reference implementations of every fused op.

These define the semantics the HIP kernels in ``ops/csrc`` must match (numerics tests compare
the kernels against these, computed in fp32) and are the CPU execution path (tests, the
no-GPU front-end).  On a GPU the HIP path is mandatory unless the caller explicitly opts into
``CASSMANTLE_OPS=torch`` (used only to measure the stock-PyTorch baseline).

Layout conventions (MI355X-first, see ``ops/__init__``):
* image activations are NHWC ``[B, H, W, C]`` contiguous (GEMM-friendly for implicit-GEMM
  conv; transformer tokens ``[B, H*W, C]`` are then a free view);
* conv weights are ``[Cout, kh, kw, Cin]`` (K-contiguous GEMM "B^T" operand);
* linear weights are ``[N, K]``.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F


def _act(y: torch.Tensor, act: Optional[str]) -> torch.Tensor:
    if act is None or act == "none":
        return y
    if act == "gelu":
        return F.gelu(y)
    if act == "gelu_tanh":
        return F.gelu(y, approximate="tanh")
    if act == "silu":
        return F.silu(y)
    if act == "quick_gelu":
        return y * torch.sigmoid(1.702 * y)
    raise ValueError(act)


def linear(x, w, bias=None, residual=None, act=None, out_dtype=None):
    """y = act(x @ w^T + bias) + residual;  act='geglu': w is [2N, K] ->
    y = (x@w[:N]^T + b[:N]) * gelu(x@w[N:]^T + b[N:])."""
    od = out_dtype or x.dtype
    y = torch.matmul(x.float(), w.float().t())
    if bias is not None:
        y = y + bias.float()
    if act == "geglu":
        h, g = y.chunk(2, dim=-1)
        y = h * F.gelu(g)
    elif act == "swiglu":
        h, g = y.chunk(2, dim=-1)
        y = h * F.silu(g)
    else:
        y = _act(y, act)
    if residual is not None:
        y = y + residual.float()
    return y.to(od)


def conv2d(x, w, bias=None, stride=1, padding=1, residual=None, upsample=False, chan_bias=None):
    """NHWC conv.  x [B,H,W,Cin], w [Cout,kh,kw,Cin].  ``upsample`` = nearest 2x on the input
    first (fused in the HIP kernel's address generation).  ``chan_bias`` [B, Cout] is a
    per-sample bias (ResNet time-embedding add fused into the epilogue)."""
    xi = x.float().permute(0, 3, 1, 2)
    if upsample:
        xi = F.interpolate(xi, scale_factor=2.0, mode="nearest")
    wi = w.float().permute(0, 3, 1, 2)
    y = F.conv2d(xi, wi, None if bias is None else bias.float(), stride=stride, padding=padding)
    y = y.permute(0, 2, 3, 1)
    if chan_bias is not None:
        y = y + chan_bias.float()[:, None, None, :]
    if residual is not None:
        y = y + residual.float()
    return y.to(x.dtype).contiguous()


def group_norm(x, num_groups, weight, bias, eps, silu=False):
    """NHWC GroupNorm (+ fused SiLU).  x [B, ..., C] (any spatial rank, channels last)."""
    B, C = x.shape[0], x.shape[-1]
    xf = x.float().reshape(B, -1, num_groups, C // num_groups)
    mean = xf.mean(dim=(1, 3), keepdim=True)
    var = xf.var(dim=(1, 3), keepdim=True, unbiased=False)
    y = (xf - mean) * torch.rsqrt(var + eps)
    y = y.reshape(B, -1, C) * weight.float() + bias.float()
    if silu:
        y = F.silu(y)
    return y.reshape(x.shape).to(x.dtype)


def layer_norm(x, weight, bias, eps):
    return F.layer_norm(x.float(), (x.shape[-1],), weight.float(), None if bias is None else bias.float(), eps).to(x.dtype)


def rms_norm(x, weight, eps):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * weight.float()).to(x.dtype)


def rope(x, pos, theta):
    """Rotate-half rotary embedding.  x [B, T, h, d]; pos [B, T] int positions."""
    d = x.shape[-1]
    inv = theta ** (-torch.arange(0, d // 2, device=x.device, dtype=torch.float32) * 2.0 / d)
    ang = pos.float()[..., None] * inv                       # [B, T, d/2]
    cos, sin = ang.cos()[:, :, None, :], ang.sin()[:, :, None, :]
    xf = x.float()
    x0, x1 = xf[..., : d // 2], xf[..., d // 2:]
    return torch.cat([x0 * cos - x1 * sin, x1 * cos + x0 * sin], dim=-1).to(x.dtype)


def rope_kv(qkv, pos0, q_out, k_cache, v_cache, H, Hk, theta):
    """Reference of the fused RoPE + KV-cache append (in place on q_out / caches)."""
    B, T, _ = qkv.shape
    d = q_out.shape[-1]
    x = qkv.view(B, T, H + 2 * Hk, d)
    pos = pos0.long()[:, None] + torch.arange(T, device=qkv.device)[None, :]
    q_out.copy_(rope(x[:, :, :H], pos, theta))
    kr = rope(x[:, :, H:H + Hk], pos, theta)
    for b in range(B):
        p0 = int(pos0[b])
        n = max(0, min(T, k_cache.shape[1] - p0))
        k_cache[b, p0:p0 + n] = kr[b, :n]
        v_cache[b, p0:p0 + n] = x[b, :n, H + Hk:]


def decode_attention(q, k_cache, v_cache, lens, scale):
    """q [B, H, d] one token vs cache [B, L, Hk, d] with lens[b] valid keys -> [B, H, d]."""
    B, H, d = q.shape
    out = torch.empty_like(q)
    for b in range(B):
        n = int(lens[b])
        o = attention(q[b:b + 1, None], k_cache[b:b + 1, :n], v_cache[b:b + 1, :n], scale)
        out[b] = o[0, 0]
    return out


def attention(q, k, v, scale=None, causal=False, kv_lens=None):
    """q [B,Nq,H,d], k/v [B,Nk,H,d] (any strides, last dim contiguous) -> o [B,Nq,H,d].
    ``kv_lens`` [B] int: keys >= len are masked (padding mask)."""
    d = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(d)
    if k.shape[2] != q.shape[2]:   # grouped-query attention: expand the kv heads
        g = q.shape[2] // k.shape[2]
        k, v = k.repeat_interleave(g, dim=2), v.repeat_interleave(g, dim=2)
    qf = q.float().permute(0, 2, 1, 3)
    kf = k.float().permute(0, 2, 1, 3)
    vf = v.float().permute(0, 2, 1, 3)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    Nq, Nk = s.shape[-2], s.shape[-1]
    if causal:
        m = torch.ones(Nq, Nk, dtype=torch.bool, device=s.device).triu(1)
        s = s.masked_fill(m, float("-inf"))
    if kv_lens is not None:
        ar = torch.arange(Nk, device=s.device)
        m = ar[None, :] >= kv_lens.to(s.device)[:, None]
        s = s.masked_fill(m[:, None, None, :], float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, vf).permute(0, 2, 1, 3)
    return o.to(q.dtype).contiguous()


def gather_cosine(table, ia, ib):
    """cos(table[ia[i]], table[ib[i]]); NaN where either index < 0."""
    ia = ia.long()
    ib = ib.long()
    valid = (ia >= 0) & (ib >= 0)
    a = table[ia.clamp(min=0)].float()
    b = table[ib.clamp(min=0)].float()
    s = (a * b).sum(-1) / (a.norm(dim=-1) * b.norm(dim=-1)).clamp_min(1e-12)
    return torch.where(valid, s, torch.full_like(s, float("nan")))


def pair_cosine(a, b):
    """Row-wise cosine of two [N, D] matrices -> [N] fp32."""
    a = a.float()
    b = b.float()
    return (a * b).sum(-1) / (a.norm(dim=-1) * b.norm(dim=-1)).clamp_min(1e-12)


def cosine_topk(table, vec, k):
    t = table.float()
    v = vec.float()
    s = (t @ v) / (t.norm(dim=-1) * v.norm()).clamp_min(1e-12)
    # deterministic ties (the HIP kernel's contract): equal scores rank the lower row first
    vals, idx = torch.sort(s, descending=True, stable=True)
    return torch.return_types.topk((vals[:k], idx[:k]))


def gaussian_kernel1d(sigma: float, device=None):
    r = max(1, int(math.ceil(3.0 * sigma)))
    xs = torch.arange(-r, r + 1, dtype=torch.float32, device=device)
    w = torch.exp(-0.5 * (xs / sigma) ** 2)
    return w / w.sum()


def gaussian_blur(img, sigma: float):
    """Separable Gaussian blur with edge clamping.  img uint8/float [H, W, C]."""
    if sigma <= 0:
        return img
    dt = img.dtype
    x = img.float().permute(2, 0, 1)[None]
    w = gaussian_kernel1d(sigma, x.device)
    r = (w.numel() - 1) // 2
    C = x.shape[1]
    x = F.pad(x, (r, r, 0, 0), mode="replicate")
    x = F.conv2d(x, w.view(1, 1, 1, -1).expand(C, 1, 1, -1), groups=C)
    x = F.pad(x, (0, 0, r, r), mode="replicate")
    x = F.conv2d(x, w.view(1, 1, -1, 1).expand(C, 1, -1, 1), groups=C)
    y = x[0].permute(1, 2, 0)
    if dt == torch.uint8:
        y = y.round().clamp(0, 255)
    return y.to(dt)


def timestep_embedding(t, dim, flip_sin_to_cos=True, shift=0.0, max_period=10000.0):
    """Sinusoidal timestep features (SD convention: [cos, sin] with flip, shift 0)."""
    half = dim // 2
    ex = -math.log(max_period) * torch.arange(half, dtype=torch.float32, device=t.device) / (half - shift)
    arg = t.float()[:, None] * torch.exp(ex)[None, :]
    e = torch.cat([torch.sin(arg), torch.cos(arg)], dim=-1)
    if flip_sin_to_cos:
        e = torch.cat([e[:, half:], e[:, :half]], dim=-1)
    return e


def cfg_combine(eps, guidance):
    """eps [2B, ...] = [uncond; cond] -> eps_u + g (eps_c - eps_u)  (fp32 result)."""
    u, c = eps.float().chunk(2)
    return u + guidance * (c - u)


def latent_step(sample, eps, coef, guidance, cfg=True):
    """Fused CFG + linear scheduler update used by every scheduler here:
        e    = cfg(eps)                                   (if cfg)
        x'   = a * x + b * e + c * h1 + d * h2 + f * h3   (h* = scheduler history of e)
    ``coef`` is a float tensor [8]: (a, b, c, d, f, save_slot, _, _) – see schedulers.py.
    Returns (x', e)."""
    e = cfg_combine(eps, guidance) if cfg else eps.float()
    return (coef[0] * sample.float() + coef[1] * e), e


def silu(x):
    return F.silu(x.float()).to(x.dtype)


def mean_pool_l2(hidden, lens):
    """Masked mean over tokens then L2-normalise: hidden [B, T, D], lens [B] -> [B, D] fp32."""
    T = hidden.shape[1]
    m = (torch.arange(T, device=hidden.device)[None, :] < lens.to(hidden.device)[:, None]).float()
    s = (hidden.float() * m[..., None]).sum(1) / m.sum(1, keepdim=True).clamp_min(1.0)
    return s / s.norm(dim=-1, keepdim=True).clamp_min(1e-12)


def lm_sample(logits, noise, eos_bias, eos: int, temperature: float, k: int, step, out, tok, pos, lens) -> None:
    """Decode-step sampler (the contract of lm.hip's lm_sample_kernel), graph-capturable: v =
    logits / T with the step's EOS bias added at ``eos``; the k largest v (stable: ties keep the
    LOWER id); the id maximising v + noise[step] among them (first in that order on ties); then
    out[step] = tok = id and pos, lens, step advance by one."""
    lg = logits.float().reshape(1, -1) / temperature
    V = lg.shape[-1]
    if 0 <= eos < V:
        lg[:, eos] += eos_bias.index_select(0, step)
    srt = torch.sort(lg, dim=-1, descending=True, stable=True)
    vals, ids = srt.values[:, :k], srt.indices[:, :k]
    g = noise.index_select(0, step)[0].gather(1, ids)
    choice = (vals + g).argmax(dim=-1, keepdim=True)
    nxt = ids.gather(1, choice)[:, 0]
    out.index_copy_(0, step, nxt[None])
    tok.copy_(nxt)
    pos.add_(1)
    lens.add_(1)
    step.add_(1)
