"""Local causal language model for round prompts (optional generator, SURVEY §2.3 'Prompt LLM').

The reference calls a remote Mistral-7B-Instruct endpoint (``src/backend.py:240-268``:
``{"inputs": seed, "parameters": {"min_new_tokens": 32, "max_new_tokens": 96}}``) and keeps the
first two sentences of the continuation.  Here the same model family runs on the GPU that
already hosts the diffusion pipeline (7B bf16 = 14.5 GB of the 288 GB HBM):

* Mistral/Llama architecture: RMSNorm (HIP), fused QKV projection, rotate-half RoPE fused with
  the KV-cache append (HIP ``rope_kv``), grouped-query attention (prefill: the flash kernel with a
  head group; decode: the split-KV ``decode_attention`` kernel), SwiGLU MLP as one gated GEMM
  epilogue (``act="swiglu"``), residual adds fused into the output projections.
* Decode is weight-streaming (M = batch rows): every projection goes through the skinny-M GEMV
  path of the GEMM dispatcher.
* The whole per-token step (embedding gather → 32 layers → logits → temperature/top-k Gumbel
  sampling → position bump) reads and writes only device buffers, so it is captured ONCE as a
  hipGraph and replayed ``max_new_tokens`` times with a single host sync at the end
  (min-new-tokens is an on-device EOS bias table, sampling noise a pre-drawn table).

Weights are random-init by default (no checkpoints on the box); ``models/weights.py``
``load_causal_lm`` maps a HF-layout safetensors checkpoint in.  Without a real tokenizer a
byte-level tokenizer is used, so random weights emit unusable text and
``game.prompts.LMPromptGenerator`` falls back to the template generator (2-sentence contract).
"""
from __future__ import annotations

import math
import threading
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.nn as nn

from .. import ops
from ..utils.tracing import TRACER


@dataclass(frozen=True)
class CausalLMConfig:
    name: str
    vocab: int
    dim: int
    layers: int
    heads: int
    kv_heads: int
    ffn: int
    rope_theta: float = 10000.0
    eps: float = 1e-5
    max_ctx: int = 512            # KV-cache capacity used for prompt generation

    @property
    def head_dim(self) -> int:
        return self.dim // self.heads


# mistralai/Mistral-7B-v0.1 shapes (public config) — the reference's remote model family
MISTRAL_7B = CausalLMConfig("mistral-7b", 32000, 4096, 32, 32, 8, 14336, 10000.0, 1e-5, 512)
TINY_LM = CausalLMConfig("tiny-lm", 320, 256, 2, 4, 2, 512, 10000.0, 1e-5, 256)
LM_CONFIGS = {"mistral-7b": MISTRAL_7B, "tiny-lm": TINY_LM}


class ByteTokenizer:
    """UTF-8 bytes + BOS/EOS.  Used when no sentencepiece model is available."""

    bos, eos = 256, 257

    def encode(self, text: str) -> List[int]:
        return [self.bos] + list(text.encode("utf-8"))

    def decode(self, ids: Sequence[int]) -> str:
        return bytes(i for i in ids if 0 <= i < 256).decode("utf-8", errors="ignore")


class SentencePieceTokenizer:
    def __init__(self, path: str) -> None:
        import sentencepiece as spm
        self.sp = spm.SentencePieceProcessor(model_file=path)
        self.bos, self.eos = self.sp.bos_id(), self.sp.eos_id()

    def encode(self, text: str) -> List[int]:
        return [self.bos] + list(self.sp.encode(text))

    def decode(self, ids: Sequence[int]) -> str:
        return self.sp.decode([int(i) for i in ids])


def _randn(shape, std, gen, device, dtype) -> nn.Parameter:
    t = torch.empty(shape, device=device, dtype=dtype)
    t.normal_(0.0, std, generator=gen)
    return nn.Parameter(t, requires_grad=False)


class LMBlock(nn.Module):
    def __init__(self, c: CausalLMConfig, gen, device, dtype):
        super().__init__()
        hd = c.head_dim
        self.c = c
        self.attn_norm = nn.Parameter(torch.ones(c.dim, device=device, dtype=dtype), requires_grad=False)
        self.mlp_norm = nn.Parameter(torch.ones(c.dim, device=device, dtype=dtype), requires_grad=False)
        self.qkv = _randn(((c.heads + 2 * c.kv_heads) * hd, c.dim), 1.0 / math.sqrt(c.dim), gen, device, dtype)
        self.o = _randn((c.dim, c.heads * hd), 1.0 / math.sqrt(c.dim * 2 * c.layers), gen, device, dtype)
        self.gate_up = _randn((2 * c.ffn, c.dim), 1.0 / math.sqrt(c.dim), gen, device, dtype)  # [up; gate]
        self.down = _randn((c.dim, c.ffn), 1.0 / math.sqrt(c.ffn * 2 * c.layers), gen, device, dtype)

    def forward(self, x, kc, vc, pos0, lens, decode: bool):
        """x [B, T, dim]; kc/vc [B, L, Hk, hd] cache of this layer."""
        c = self.c
        B, T, _ = x.shape
        hd = c.head_dim
        qkv = ops.rms_linear(x, self.attn_norm, c.eps, self.qkv)
        q = torch.empty((B, T, c.heads, hd), device=x.device, dtype=x.dtype)
        ops.rope_kv(qkv, pos0, q, kc, vc, c.heads, c.kv_heads, c.rope_theta)
        if decode:
            o = ops.decode_attention(q.view(B, c.heads, hd), kc, vc, lens)
        else:
            # prefill from position 0: causal flash attention over the freshly written cache rows
            o = ops.attention(q, kc[:, :T], vc[:, :T], causal=True)
        x = ops.linear(o.reshape(B, T, c.heads * hd), self.o, residual=x)
        h = ops.rms_linear(x, self.mlp_norm, c.eps, self.gate_up, act="swiglu")
        return ops.linear(h, self.down, residual=x)


class CausalLM(nn.Module):
    def __init__(self, c: CausalLMConfig, device=None, dtype=torch.bfloat16, seed: int = 0):
        super().__init__()
        device = torch.device(device) if device is not None else torch.device("cpu")
        gen = torch.Generator(device=device).manual_seed(seed)
        self.c = c
        self.embed = _randn((c.vocab, c.dim), 1.0, gen, device, dtype)
        self.blocks = nn.ModuleList([LMBlock(c, gen, device, dtype) for _ in range(c.layers)])
        self.norm = nn.Parameter(torch.ones(c.dim, device=device, dtype=dtype), requires_grad=False)
        self.lm_head = _randn((c.vocab, c.dim), 1.0 / math.sqrt(c.dim), gen, device, dtype)

    def alloc_cache(self, B: int, L: int):
        c = self.c
        shape = (c.layers, B, L, c.kv_heads, c.head_dim)
        dev, dt = self.embed.device, self.embed.dtype
        return torch.zeros(shape, device=dev, dtype=dt), torch.zeros(shape, device=dev, dtype=dt)

    def forward(self, tokens: torch.Tensor, kcache, vcache, pos0: torch.Tensor,
                lens: Optional[torch.Tensor] = None, decode: bool = False) -> torch.Tensor:
        """tokens [B, T] -> logits of the last position [B, vocab] (bf16).  ``decode``: T == 1 at
        device positions ``pos0`` with ``lens = pos0 + 1`` valid keys; else prefill from 0."""
        B, T = tokens.shape
        x = self.embed.index_select(0, tokens.reshape(-1)).view(B, T, self.c.dim)
        for i, blk in enumerate(self.blocks):
            x = blk(x, kcache[i], vcache[i], pos0, lens, decode)
        return ops.rms_linear(x[:, -1], self.norm, self.c.eps, self.lm_head)

    @torch.no_grad()
    def full_logits(self, tokens: torch.Tensor) -> torch.Tensor:
        """Cache-free reference forward (all positions) -> [B, T, vocab] f32.  Test oracle."""
        from ..ops import reference as R
        c = self.c
        B, T = tokens.shape
        hd = c.head_dim
        x = self.embed.index_select(0, tokens.reshape(-1)).view(B, T, c.dim).float()
        pos = torch.arange(T, device=tokens.device)[None].expand(B, T)
        for blk in self.blocks:
            n = R.rms_norm(x, blk.attn_norm, c.eps).float()
            qkv = (n @ blk.qkv.float().t()).view(B, T, c.heads + 2 * c.kv_heads, hd)
            q = R.rope(qkv[:, :, :c.heads], pos, c.rope_theta).float()
            k = R.rope(qkv[:, :, c.heads:c.heads + c.kv_heads], pos, c.rope_theta).float()
            v = qkv[:, :, c.heads + c.kv_heads:]
            o = R.attention(q, k, v, causal=True).float()
            x = x + o.reshape(B, T, -1) @ blk.o.float().t()
            n = R.rms_norm(x, blk.mlp_norm, c.eps).float()
            hg = n @ blk.gate_up.float().t()
            h, g = hg.chunk(2, dim=-1)
            x = x + (h * torch.nn.functional.silu(g)) @ blk.down.float().t()
        x = R.rms_norm(x, self.norm, c.eps).float()
        return x @ self.lm_head.float().t()


class LMTextGenerator:
    """``generate_text(prompt, min_new_tokens, max_new_tokens)`` for
    :class:`~cassmantle_amd.game.prompts.LMPromptGenerator` (continuation only, no echo)."""

    def __init__(self, cfg: CausalLMConfig = TINY_LM, device=None, seed: int = 0, use_graphs: bool = True,
                 tokenizer=None, temperature: float = 0.8, top_k: int = 40, max_new_cap: int = 128) -> None:
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.cfg = cfg
        self.model = CausalLM(cfg, device=self.device, seed=seed)
        self.tok = tokenizer or ByteTokenizer()
        self.temperature, self.top_k = temperature, min(top_k, cfg.vocab)
        self.use_graphs = use_graphs and self.device.type == "cuda"
        self.max_new_cap = max_new_cap
        self.seed = seed
        L = cfg.max_ctx
        self.kc, self.vc = self.model.alloc_cache(1, L)
        dev = self.device
        self.tok_buf = torch.zeros((1,), device=dev, dtype=torch.long)
        self.pos = torch.zeros((1,), device=dev, dtype=torch.int32)
        self.lens = torch.ones((1,), device=dev, dtype=torch.int32)
        self.idx = torch.zeros((1,), device=dev, dtype=torch.long)
        self.noise = torch.zeros((max_new_cap, 1, cfg.vocab), device=dev, dtype=torch.float32)
        self.eos_bias = torch.zeros((max_new_cap,), device=dev, dtype=torch.float32)
        self.out = torch.zeros((max_new_cap, 1), device=dev, dtype=torch.long)
        self.graph = None
        self.calls = 0
        self._lock = threading.Lock()

    # one decode step entirely on device buffers (captured as a graph on GPU)
    def _step(self) -> None:
        logits = self.model(self.tok_buf.view(1, 1), self.kc, self.vc, self.pos, self.lens, decode=True)
        # top-k + Gumbel-max with this step's noise row, and the token / position / length / step
        # update: one in-tree kernel on the GPU (lm.hip lm_sample_kernel), no ATen sampling ops
        ops.lm_sample(logits, self.noise, self.eos_bias, self.tok.eos, self.temperature, self.top_k, self.idx,
                      self.out, self.tok_buf, self.pos, self.lens)

    def _capture(self) -> None:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        saved = [t.clone() for t in (self.tok_buf, self.pos, self.lens, self.idx)]
        with torch.cuda.stream(s):
            self._step()
        torch.cuda.current_stream().wait_stream(s)
        for t, v in zip((self.tok_buf, self.pos, self.lens, self.idx), saved):
            t.copy_(v)
        g = torch.cuda.CUDAGraph()
        with TRACER.capturing(), torch.cuda.graph(g, capture_error_mode="thread_local"):
            self._step()
        for t, v in zip((self.tok_buf, self.pos, self.lens, self.idx), saved):
            t.copy_(v)
        self.graph = g

    @torch.no_grad()
    def generate_ids(self, prompt_ids: Sequence[int], min_new: int, max_new: int) -> List[int]:
        max_new = max(1, min(max_new, self.max_new_cap))
        L = self.cfg.max_ctx
        ids = list(prompt_ids)[-(L - max_new):] or [self.tok.bos]
        dev = self.device
        T = len(ids)
        gen = torch.Generator(device="cpu").manual_seed(self.seed * 1000003 + self.calls)
        self.calls += 1
        u = torch.rand((max_new, 1, self.cfg.vocab), generator=gen).clamp_(1e-10, 1.0 - 1e-7)
        self.noise[:max_new].copy_((-torch.log(-torch.log(u))).to(dev))
        eb = torch.zeros((self.max_new_cap,))
        eb[:min(min_new, self.max_new_cap)] = float("-inf")
        self.eos_bias.copy_(eb.to(dev))
        self.idx.zero_()
        # prefill all but the last prompt token; the decode step consumes the last one
        self.pos.zero_()
        if T > 1:
            pre = torch.tensor([ids[:-1]], device=dev, dtype=torch.long)
            self.model(pre, self.kc, self.vc, self.pos, None, decode=False)
        self.pos.fill_(T - 1)
        self.lens.fill_(T)
        self.tok_buf.fill_(ids[-1])
        if self.use_graphs and self.graph is None:
            self._capture()
        for _ in range(max_new):
            if self.graph is not None:
                self.graph.replay()
            else:
                self._step()
        out = self.out[:max_new, 0].tolist()
        if self.tok.eos in out:
            out = out[:out.index(self.tok.eos)]
        return out

    def generate_text(self, prompt: str, min_new_tokens: int, max_new_tokens: int) -> str:
        # rooms call generators from worker threads; the static decode buffers are single-user
        with self._lock:
            ids = self.generate_ids(self.tok.encode(prompt), min_new_tokens, max_new_tokens)
        return self.tok.decode(ids)
