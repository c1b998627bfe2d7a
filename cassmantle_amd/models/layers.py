"""NHWC building blocks for the diffusion / text models, routed through ``cassmantle_amd.ops``.

Design (MI355X-first):
* activations NHWC bf16, so every conv is an implicit GEMM with K-contiguous operands and a
  transformer's ``[B, H*W, C]`` token view is free (no permutes around attention blocks);
* Q/K/V projections are one fused ``[3C, C]`` GEMM; the attention kernel reads Q/K/V as
  strided views of its output (no split/transposes);
* bias, residual adds, GEGLU, SiLU/GELU and the ResNet time-embedding add are GEMM/conv
  epilogues; GroupNorm+SiLU is one kernel.

Module names follow the diffusers/transformers parameter naming so a real checkpoint can be
mapped in (``models/weights.py``); weights are random-init by default (BASELINE.json).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.nn as nn

from .. import ops


def _param(shape, std, gen: Optional[torch.Generator], dtype) -> nn.Parameter:
    t = torch.randn(*shape, generator=gen, dtype=torch.float32) * std
    return nn.Parameter(t.to(dtype), requires_grad=False)


def _zeros(shape, dtype) -> nn.Parameter:
    return nn.Parameter(torch.zeros(*shape, dtype=dtype), requires_grad=False)


def _ones(shape, dtype) -> nn.Parameter:
    return nn.Parameter(torch.ones(*shape, dtype=dtype), requires_grad=False)


_GN_FUSE = os.environ.get("CASSMANTLE_GN_FUSE", "1") != "0"   # A/B knob (0: two-pass GroupNorm)
_UP2 = os.environ.get("CASSMANTLE_UP2", "1") != "0"           # A/B knob (0: upsampled 3x3 conv)


class StatsArena:
    """GroupNorm statistics produced by GEMM/conv epilogues: one zeroed slab per forward (int64
    fixed point, see ``ops.new_stats``).

    A producer (conv / linear called with ``stats=arena.take(...)``) accumulates the
    per-(image, channel) sum and sum-of-squares of its output in its epilogue; the GroupNorm
    that consumes the tensor then runs only its apply pass (no statistics read of the
    activation).  All slices of one forward come from ONE buffer cleared by ONE memset in
    :meth:`begin`.  Buffers are kept per activation shape and never reallocated once sized, so
    a captured denoise graph keeps valid addresses: the first forward of a shape only measures
    the slab (its slices are plain ``torch.zeros``); later forwards — including the
    graph-capture warmups — slice the slab.  Disabled (``take`` returns None) off the HIP path,
    where GroupNorm computes its own statistics."""

    def __init__(self) -> None:
        self._bufs: dict = {}
        self._need: dict = {}
        self.key = None
        self.buf: Optional[torch.Tensor] = None
        self.off = 0
        self.on = False

    def begin(self, key, x: torch.Tensor) -> "StatsArena":
        self.on = x.device.type == "cuda" and ops.get_mode() == "hip" and _GN_FUSE
        self.key, self.off = key, 0
        if not self.on:
            return self
        self.buf = self._bufs.get(key)
        need = self._need.get(key, 0)
        if need and self.buf is None:
            self.buf = self._bufs[key] = torch.empty(need, device=x.device, dtype=torch.int64)
        if self.buf is not None:
            ops.zero_(self.buf)
        self.device = x.device
        return self

    def take_rows(self, rows: int) -> Optional[torch.Tensor]:
        """A zeroed int64 [rows, 2] slice for LayerNorm row statistics (ops.linear row_stats)."""
        s = self.take(1, rows)
        return None if s is None else s.view(rows, 2)

    def take(self, B: int, C: int) -> Optional[torch.Tensor]:
        if not self.on:
            return None
        n = B * C * 2
        end = self.off + n
        if self.buf is not None and end <= self.buf.numel():
            s = self.buf[self.off:end].view(B, C, 2)
        else:
            self._need[self.key] = max(self._need.get(self.key, 0), end)
            s = ops.new_stats(B, C, self.device)
        self.off = end
        return s


class Linear(nn.Module):
    def __init__(self, fin: int, fout: int, bias: bool = True, gen=None, dtype=torch.bfloat16,
                 std: Optional[float] = None):
        super().__init__()
        self.fin, self.fout = fin, fout
        self.weight = _param((fout, fin), std if std is not None else 1.0 / math.sqrt(fin), gen, dtype)
        self.bias = _param((fout,), 0.02, gen, dtype) if bias else None

    def forward(self, x, residual=None, act=None, stats=None, row_stats=None):
        return ops.linear(x, self.weight, self.bias, residual=residual, act=act, stats=stats, row_stats=row_stats)


class Conv2d(nn.Module):
    """NHWC conv; weight [Cout, kh, kw, Cin]."""

    def __init__(self, cin: int, cout: int, k: int = 3, stride: int = 1, padding: Optional[int] = None,
                 bias: bool = True, gen=None, dtype=torch.bfloat16):
        super().__init__()
        self.cin, self.cout, self.k, self.stride = cin, cout, k, stride
        self.padding = (k // 2) if padding is None else padding
        self.weight = _param((cout, k, k, cin), 1.0 / math.sqrt(cin * k * k), gen, dtype)
        self.bias = _param((cout,), 0.02, gen, dtype) if bias else None

    # Derived weights are non-persistent BUFFERS keyed by the source weight's version counter:
    # computed once (StableDiffusion prepares them on the CPU before moving the model, so no
    # ATen kernel runs on the GPU for them), they follow .to(device), and an in-place weight
    # load (version bump) recomputes them.
    upsampling = False   # set by the Upsample blocks: prepare() folds the parity weights
    pad_in = 0           # channel-padded input width prepare() builds padded weights for

    def _derived(self, name: str, key, fn):
        buf = self._buffers.get(name)
        if buf is None or getattr(self, "_key_" + name, None) != key or buf.device != self.weight.device:
            self.register_buffer(name, fn(), persistent=False)
            setattr(self, "_key_" + name, key)
        return self._buffers[name]

    def up2_weights(self):
        """Folded per-parity weights of an upsampling 3x3 conv (ops.fold_upsample_weights)."""
        return self._derived("w4", self.weight._version, lambda: ops.fold_upsample_weights(self.weight))

    def padded_weight(self, cin: int):
        """Weight zero-padded to a channel-padded input (UNet conv_in: 4 -> 8 channels)."""
        return self._derived("wpad", (self.weight._version, cin),
                             lambda: torch.nn.functional.pad(self.weight, (0, cin - self.cin)).contiguous())

    def prepare(self) -> None:
        if self.upsampling and self.k == 3 and self.cin % 64 == 0:
            self.up2_weights()
        if self.pad_in > self.cin:
            self.padded_weight(self.pad_in)

    def forward(self, x, residual=None, upsample=False, chan_bias=None, stats=None, out=None):
        if out is not None:         # (a caller-provided output buffer)
            w = self.padded_weight(x.shape[-1]) if x.shape[-1] > self.cin else self.weight
            return ops.conv2d(x, w, self.bias, self.stride, self.padding, residual=residual,
                              upsample=upsample, chan_bias=chan_bias, stats=stats, out=out)
        if x.shape[-1] > self.cin:
            # input carries zero padding channels (graph-static UNet input): padded weights,
            # cached, instead of a pad copy of input and weight on every call
            return ops.conv2d(x, self.padded_weight(x.shape[-1]), self.bias, self.stride, self.padding,
                              residual=residual, upsample=upsample, chan_bias=chan_bias, stats=stats)
        if upsample and self.k == 3 and self.stride == 1 and _UP2 and x.device.type == "cuda" \
                and ops.get_mode() == "hip" and self.cin % 64 == 0:
            # nearest-2x upsample + 3x3 conv as four parity-class 2x2 convs (4/9 of the MACs)
            return ops.conv2d_up2(x, self.weight, self.up2_weights(), self.bias, residual=residual,
                                  chan_bias=chan_bias, stats=stats)
        if self.k == 1 and self.stride == 1 and not upsample and chan_bias is None:
            return ops.linear(x, self.weight.view(self.cout, self.cin), self.bias, residual=residual, stats=stats)
        return ops.conv2d(x, self.weight, self.bias, self.stride, self.padding, residual=residual,
                          upsample=upsample, chan_bias=chan_bias, stats=stats)


class GroupNorm(nn.Module):
    def __init__(self, groups: int, channels: int, eps: float = 1e-5, dtype=torch.bfloat16):
        super().__init__()
        self.groups, self.eps = groups, eps
        self.weight = _ones((channels,), dtype)
        self.bias = _zeros((channels,), dtype)

    def forward(self, x, silu=False, stats=None, stats2=None):
        """``stats`` / ``stats2``: producer statistics (see :class:`StatsArena`); ``stats2``
        covers the trailing channels of a channel concatenation."""
        return ops.group_norm(x, self.groups, self.weight, self.bias, self.eps, silu, stats=stats, stats2=stats2)


class LayerNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-5, dtype=torch.bfloat16):
        super().__init__()
        self.eps = eps
        self.weight = _ones((dim,), dtype)
        self.bias = _zeros((dim,), dtype)

    def forward(self, x):
        return ops.layer_norm(x, self.weight, self.bias, self.eps)


class SelfAttention(nn.Module):
    """Multi-head self attention with fused QKV projection; output projection fuses the
    residual add."""

    def __init__(self, dim: int, heads: int, gen=None, dtype=torch.bfloat16, qkv_bias=False,
                 out_bias=True):
        super().__init__()
        self.dim, self.heads = dim, heads
        self.head_dim = dim // heads
        self.to_qkv = Linear(dim, 3 * dim, bias=qkv_bias, gen=gen, dtype=dtype)
        self.to_out = Linear(dim, dim, bias=out_bias, gen=gen, dtype=dtype)

    def forward(self, x, residual=None, causal=False, kv_lens=None, fp8=False, qkv=None, kv8=None,
                row_stats=None):
        """``qkv``: the fused projection already computed (e.g. with a folded LayerNorm);
        ``kv8``: its K/V as the fp8 attention image (ops.ln_linear(kv8=...)), fp8 only;
        ``row_stats``: LayerNorm row statistics of the output for the next folded projection."""
        if qkv is None:
            qkv = self.to_qkv(x)
        B, N = qkv.shape[0], qkv.shape[1]
        C = self.dim
        qkv = qkv.view(B, N, 3, self.heads, self.head_dim)
        if kv8 is not None:
            assert fp8 and kv_lens is None, "kv8: fp8 self-attention without key lengths"
            o = ops.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], causal=causal, fp8=True, kv8=kv8)
        else:
            o = ops.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], causal=causal, kv_lens=kv_lens, fp8=fp8)
        return self.to_out(o.reshape(B, N, C), residual=residual, row_stats=row_stats)


class CrossAttention(nn.Module):
    def __init__(self, dim: int, ctx_dim: int, heads: int, gen=None, dtype=torch.bfloat16):
        super().__init__()
        self.dim, self.heads = dim, heads
        self.head_dim = dim // heads
        self.to_q = Linear(dim, dim, bias=False, gen=gen, dtype=dtype)
        self.to_kv = Linear(ctx_dim, 2 * dim, bias=False, gen=gen, dtype=dtype)
        self.to_out = Linear(dim, dim, bias=True, gen=gen, dtype=dtype)

    _kv = None   # view into the UNet's batched context-K/V buffer (set by UNet.set_context)
    _kv8 = None  # its OCP-e4m3 image for the fp8 kernel (set by UNet.set_context(fp8=True))

    def forward(self, x, ctx, residual=None, fp8=False, q=None, row_stats=None):
        """``q``: the query projection already computed (e.g. with a folded LayerNorm);
        ``row_stats``: LayerNorm row statistics of the output for the next folded projection."""
        if q is None:
            q = self.to_q(x)
        B, N = q.shape[0], q.shape[1]
        C = self.dim
        q = q.view(B, N, self.heads, self.head_dim)
        kv8 = None
        if self._kv is not None and self._kv.shape[0] == B:
            # the text context is constant over the denoise loop: K/V of every cross-attention
            # layer come from ONE GEMM per generation (strided views, no copies), and with fp8
            # their e4m3 image is packed once per generation too
            kv = self._kv.view(B, self._kv.shape[1], 2, self.heads, self.head_dim)
            kv8 = self._kv8 if fp8 else None
        else:
            kv = self.to_kv(ctx).view(B, ctx.shape[1], 2, self.heads, self.head_dim)
        o = ops.attention(q, kv[:, :, 0], kv[:, :, 1], fp8=fp8, kv8=kv8)
        return self.to_out(o.reshape(B, N, C), residual=residual, row_stats=row_stats)


class GEGLUFeedForward(nn.Module):
    def __init__(self, dim: int, mult: int = 4, gen=None, dtype=torch.bfloat16):
        super().__init__()
        inner = dim * mult
        self.proj_in = Linear(dim, 2 * inner, gen=gen, dtype=dtype)  # [value; gate] rows
        self.proj_out = Linear(inner, dim, gen=gen, dtype=dtype)

    def forward(self, x, residual=None):
        return self.proj_out(self.proj_in(x, act="geglu"), residual=residual)
