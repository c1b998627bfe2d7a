"""AutoencoderKL decoder (SD VAE), NHWC, on ``cassmantle_amd.ops``.

Implied by the reference's remote txt2img: latent/scaling →
post_quant_conv → conv_in(4→512) → mid [ResNet, single-head attention (d=512), ResNet] →
4 up levels × 3 ResNets (512, 512, 256, 128) with nearest-2× upsample fused into the next
conv → GroupNorm+SiLU → conv_out(→3) → clamp → uint8.  The 512² levels are the largest
activations of the whole pipeline (memory-bound convs), NHWC keeps them GEMM-shaped.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn as nn

from .. import ops
from .layers import Conv2d, GroupNorm, Linear, StatsArena


@dataclass
class VAEConfig:
    latent_channels: int = 4
    out_channels: int = 3
    block_out_channels: Tuple[int, ...] = (128, 256, 512, 512)
    layers_per_block: int = 2
    norm_groups: int = 32
    eps: float = 1e-6
    scaling_factor: float = 0.18215


SD_VAE = VAEConfig()
SDXL_VAE = VAEConfig(scaling_factor=0.13025)
TINY_VAE = VAEConfig(block_out_channels=(16, 32), layers_per_block=1, norm_groups=8)


class VAEResnet(nn.Module):
    def __init__(self, cin, cout, groups, eps, gen, dtype):
        super().__init__()
        self.norm1 = GroupNorm(groups, cin, eps, dtype)
        self.conv1 = Conv2d(cin, cout, 3, gen=gen, dtype=dtype)
        self.norm2 = GroupNorm(groups, cout, eps, dtype)
        self.conv2 = Conv2d(cout, cout, 3, gen=gen, dtype=dtype)
        self.conv_shortcut = Conv2d(cin, cout, 1, padding=0, gen=gen, dtype=dtype) if cin != cout else None

    def forward(self, x, arena: Optional[StatsArena] = None, xs=None):
        """-> (out, epilogue statistics of out or None); see :class:`StatsArena`."""
        B = x.shape[0]
        s1 = arena.take(B, self.conv1.cout) if arena is not None else None
        h = self.conv1(self.norm1(x, silu=True, stats=xs), stats=s1)
        h = self.norm2(h, silu=True, stats=s1)
        sc = self.conv_shortcut(x) if self.conv_shortcut is not None else x
        s2 = arena.take(B, self.conv2.cout) if arena is not None else None
        return self.conv2(h, residual=sc, stats=s2), s2


class VAEAttention(nn.Module):
    """Single-head spatial self-attention (head dim = C = 512)."""

    def __init__(self, c, groups, eps, gen, dtype):
        super().__init__()
        self.group_norm = GroupNorm(groups, c, eps, dtype)
        self.to_qkv = Linear(c, 3 * c, gen=gen, dtype=dtype)
        self.to_out = Linear(c, c, gen=gen, dtype=dtype)

    def forward(self, x, arena: Optional[StatsArena] = None, xs=None):
        B, H, W, C = x.shape
        h = self.group_norm(x, stats=xs).view(B, H * W, C)
        qkv = self.to_qkv(h).view(B, H * W, 3, 1, C)
        o = ops.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2])
        so = arena.take(B, C) if arena is not None else None
        out = self.to_out(o.reshape(B, H * W, C), residual=x.view(B, H * W, C), stats=so)
        return out.view(B, H, W, C), so


class VAEDecoder(nn.Module):
    def __init__(self, cfg: VAEConfig = SD_VAE, seed: int = 0, dtype=torch.bfloat16):
        super().__init__()
        self.cfg = cfg
        gen = torch.Generator().manual_seed(seed + 7)
        ch = list(reversed(cfg.block_out_channels))
        g, eps = cfg.norm_groups, cfg.eps
        self.post_quant_conv = Conv2d(cfg.latent_channels, cfg.latent_channels, 1, padding=0, gen=gen, dtype=dtype)
        self.conv_in = Conv2d(cfg.latent_channels, ch[0], 3, gen=gen, dtype=dtype)
        self.conv_in.pad_in = 8 if cfg.latent_channels % 8 else 0   # fed by the 8-channel post-quant GEMM
        self.mid_res1 = VAEResnet(ch[0], ch[0], g, eps, gen, dtype)
        self.mid_attn = VAEAttention(ch[0], g, eps, gen, dtype)
        self.mid_res2 = VAEResnet(ch[0], ch[0], g, eps, gen, dtype)
        self.up = nn.ModuleList()
        cur = ch[0]
        for i, c in enumerate(ch):
            blk = nn.Module()
            blk.resnets = nn.ModuleList()
            for _ in range(cfg.layers_per_block + 1):
                blk.resnets.append(VAEResnet(cur, c, g, eps, gen, dtype))
                cur = c
            blk.upsample_conv = Conv2d(cur, cur, 3, gen=gen, dtype=dtype) if i < len(ch) - 1 else None
            if blk.upsample_conv is not None:
                blk.upsample_conv.upsampling = True
            self.up.append(blk)
        self.conv_norm_out = GroupNorm(g, cur, eps, dtype)
        self.conv_out = Conv2d(cur, cfg.out_channels, 3, gen=gen, dtype=dtype)
        self._arena = StatsArena()

    def prepare(self) -> "VAEDecoder":
        """Derived weights now (on the CPU before the move to the GPU, like UNet.prepare): the
        upsampling convs' parity weights and the 1/scaling_factor folded into post_quant_conv."""
        for m in self.modules():
            if isinstance(m, Conv2d):
                m.prepare()
        self.pq_scaled()
        return self

    def pq_scaled(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """post_quant_conv as a GEMM with 1/scaling_factor folded in and its output padded to 8
        channels (zero rows): conv_in then reads whole 16-byte k-chunks with its padded weight
        instead of padding its input and weight on every call."""
        pq = self.post_quant_conv
        cp = 8 if pq.cout % 8 else pq.cout

        def wfn():
            w = torch.zeros((cp, pq.cin), dtype=torch.float32, device=pq.weight.device)
            w[:pq.cout] = pq.weight.float().view(pq.cout, pq.cin) / self.cfg.scaling_factor
            return w.to(pq.weight.dtype).contiguous()

        def bfn():
            b = torch.zeros((cp,), dtype=pq.weight.dtype, device=pq.weight.device)
            if pq.bias is not None:
                b[:pq.cout] = pq.bias
            return b
        key = (pq.weight._version, None if pq.bias is None else pq.bias._version)
        return pq._derived("wscaled", key, wfn), pq._derived("bpadded", key, bfn)

    def forward(self, z: torch.Tensor) -> torch.Tensor:
        """z: scaled latents [B, h, w, 4] NHWC -> image [B, 8h, 8w, 3] in [-1, 1] (model dtype)."""
        if z.device.type == "cuda" and ops.get_mode() == "hip" and z.dtype == self.conv_in.weight.dtype:
            # 1/scaling_factor lives in the post_quant_conv weight: no scale / cast launches;
            # its 8-channel output feeds conv_in's padded weight (no per-call pad copies)
            w, b = self.pq_scaled()
            h = ops.linear(z, w, b)
        else:
            z = (z.float() / self.cfg.scaling_factor).to(self.conv_in.weight.dtype)
            h = self.post_quant_conv(z)
        ar = self._arena.begin(tuple(z.shape), z)
        B = z.shape[0]
        hs = ar.take(B, self.conv_in.cout)
        h = self.conv_in(h, stats=hs)
        h, hs = self.mid_res1(h, ar, hs)
        h, hs = self.mid_attn(h, ar, hs)
        h, hs = self.mid_res2(h, ar, hs)
        for blk in self.up:
            for r in blk.resnets:
                h, hs = r(h, ar, hs)
            if blk.upsample_conv is not None:
                hs = ar.take(B, blk.upsample_conv.cout)
                h = blk.upsample_conv(h, upsample=True, stats=hs)
        h = self.conv_norm_out(h, silu=True, stats=hs)
        return self.conv_out(h)

    def decode_uint8(self, z: torch.Tensor) -> torch.Tensor:
        return ops.vae_postprocess(self.forward(z))
