"""Text encoders: CLIP text transformer (SD conditioning) and MiniLM/BERT (guess scorer).

* CLIP (K13): SD-1.5 conditions on CLIP ViT-L/14's text tower [ext]: 49408-token vocab, 77
  positions, d=768, 12 pre-LN layers, 12 heads, quick-GELU MLP 3072, causal mask, final LN.
  SDXL adds OpenCLIP bigG (d=1280, 32 layers, 20 heads, GELU MLP 5120) and uses penultimate
  hidden states plus a pooled, projected EOS embedding.
* MiniLM (K16): all-MiniLM-L6-v2-shaped BERT [ext]: d=384, 6 post-LN layers, 12 heads
  (head dim 32), GELU MLP 1536, LN eps 1e-12, mean pooling + L2 normalisation — the scorer
  BASELINE config 1 names, replacing the reference's word2vec lookup
  (``src/backend.py:303-310``).

Tokenizers: the vocab files are not available offline, so :class:`HashTokenizer` maps
words deterministically into the vocab id range with the right special tokens and padding
(random-init weights make real ids meaningless anyway); a ``tokenizer.json`` is used through
the ``tokenizers`` library when one is configured.
"""
from __future__ import annotations

import hashlib
import re
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from .. import ops
from .layers import LayerNorm, Linear, SelfAttention, _param


class HashTokenizer:
    _pat = re.compile(r"[A-Za-z]+|[0-9]|[^\sA-Za-z0-9]")

    def __init__(self, vocab_size: int, bos: int, eos: int, pad: int, max_len: int,
                 first_regular: int = 0, json_path: Optional[str] = None) -> None:
        self.vocab_size, self.bos, self.eos, self.pad, self.max_len = vocab_size, bos, eos, pad, max_len
        self.first_regular = first_regular
        self._tok = None
        if json_path:
            from tokenizers import Tokenizer
            self._tok = Tokenizer.from_file(json_path)

    def _word_id(self, w: str) -> int:
        h = int.from_bytes(hashlib.blake2b(w.encode(), digest_size=8).digest(), "little")
        span = self.vocab_size - self.first_regular - 3
        return self.first_regular + (h % span)

    def encode(self, text: str) -> List[int]:
        if self._tok is not None:
            ids = self._tok.encode(text).ids
        else:
            ids = [self._word_id(w) for w in self._pat.findall(text.lower())]
        ids = [self.bos] + ids[: self.max_len - 2] + [self.eos]
        return ids

    def __call__(self, texts: Sequence[str], pad_to: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        enc = [self.encode(t) for t in texts]
        L = pad_to or max(len(e) for e in enc)
        ids = torch.full((len(enc), L), self.pad, dtype=torch.int64)
        lens = torch.zeros(len(enc), dtype=torch.int32)
        for i, e in enumerate(enc):
            ids[i, :len(e)] = torch.tensor(e)
            lens[i] = len(e)
        return ids, lens


def clip_tokenizer(max_len: int = 77, vocab: int = 49408) -> HashTokenizer:
    # SD pads with <|endoftext|> (49407)
    return HashTokenizer(vocab, bos=vocab - 2, eos=vocab - 1, pad=vocab - 1, max_len=max_len, first_regular=256)


def bert_tokenizer(max_len: int = 128, vocab: int = 30522) -> HashTokenizer:
    return HashTokenizer(vocab, bos=101, eos=102, pad=0, max_len=max_len, first_regular=1000)


@dataclass
class CLIPTextConfig:
    vocab_size: int = 49408
    max_positions: int = 77
    dim: int = 768
    layers: int = 12
    heads: int = 12
    mlp: int = 3072
    act: str = "quick_gelu"
    eps: float = 1e-5
    projection_dim: int = 0      # >0: pooled EOS projection (SDXL bigG: 1280)


CLIP_L = CLIPTextConfig()
CLIP_BIGG = CLIPTextConfig(dim=1280, layers=32, heads=20, mlp=5120, act="gelu", projection_dim=1280)
TINY_CLIP = CLIPTextConfig(dim=32, layers=2, heads=2, mlp=64)


class PreLNBlock(nn.Module):
    def __init__(self, dim, heads, mlp, act, eps, gen, dtype):
        super().__init__()
        self.layer_norm1 = LayerNorm(dim, eps, dtype)
        self.self_attn = SelfAttention(dim, heads, gen=gen, dtype=dtype, qkv_bias=True)
        self.layer_norm2 = LayerNorm(dim, eps, dtype)
        self.fc1 = Linear(dim, mlp, gen=gen, dtype=dtype)
        self.fc2 = Linear(mlp, dim, gen=gen, dtype=dtype)
        self.act = act

    def forward(self, x, causal=True):
        x = self.self_attn(self.layer_norm1(x), residual=x, causal=causal)
        return self.fc2(self.fc1(self.layer_norm2(x), act=self.act), residual=x)


class CLIPTextEncoder(nn.Module):
    def __init__(self, cfg: CLIPTextConfig = CLIP_L, seed: int = 0, dtype=torch.bfloat16):
        super().__init__()
        self.cfg = cfg
        gen = torch.Generator().manual_seed(seed + 101)
        self.token_embedding = _param((cfg.vocab_size, cfg.dim), 0.02, gen, dtype)
        self.position_embedding = _param((cfg.max_positions, cfg.dim), 0.01, gen, dtype)
        self.layers = nn.ModuleList([PreLNBlock(cfg.dim, cfg.heads, cfg.mlp, cfg.act, cfg.eps, gen, dtype)
                                     for _ in range(cfg.layers)])
        self.final_layer_norm = LayerNorm(cfg.dim, cfg.eps, dtype)
        self.text_projection = Linear(cfg.dim, cfg.projection_dim, bias=False, gen=gen, dtype=dtype) \
            if cfg.projection_dim else None
        self.tokenizer = clip_tokenizer(cfg.max_positions, cfg.vocab_size)

    def forward(self, ids: torch.Tensor, output_hidden: int = -1, eos_rows: Optional[torch.Tensor] = None):
        """ids [B, 77] -> (last/penultimate hidden [B,77,D], pooled [B,P] or None).
        ``eos_rows`` (int32 [B], = b * 77 + position of the first EOS, built on the host by
        :meth:`encode`) gathers the pooled rows without a device argmax."""
        B, L = ids.shape
        x = ops.gather_add(self.token_embedding, ids, self.position_embedding)   # token + position
        hidden = None
        n = len(self.layers)
        for i, blk in enumerate(self.layers):
            x = blk(x, causal=True)
            if output_hidden == -2 and i == n - 2:
                hidden = x
        last = self.final_layer_norm(x)
        if hidden is None:
            hidden = last
        pooled = None
        if self.text_projection is not None:
            if eos_rows is None:
                eos_pos = (ids == self.tokenizer.eos).int().argmax(dim=1)
                eos_rows = torch.arange(B, device=ids.device) * L + eos_pos
            pooled = self.text_projection(ops.gather_add(last.reshape(B * L, -1), eos_rows))
        return hidden, pooled

    def encode(self, texts: Sequence[str], device, output_hidden: int = -1, graphs: bool = False):
        """Tokenise on the host, encode on ``device``.  ``graphs`` (GPU): the encoder forward is
        captured once per (batch, output) shape and replayed -- ~12 (CLIP-L) / 32 (bigG) layers
        of launches per generation become one graph launch; the outputs are copied out of the
        graph's static buffers, so they outlive the next call."""
        ids, _ = self.tokenizer(texts, pad_to=self.cfg.max_positions)
        eos_rows = None
        if self.text_projection is not None:
            B, L = ids.shape
            eos_rows = (torch.arange(B) * L + (ids == self.tokenizer.eos).int().argmax(dim=1)).int()
        if not graphs or torch.device(device).type != "cuda" or ops.get_mode() != "hip":
            # int32 ids, converted on the host: the embedding gather takes them as they are
            return self.forward(ops.h2d(ids.int(), device), output_hidden,
                                None if eos_rows is None else ops.h2d(eos_rows, device))
        key = (tuple(ids.shape), output_hidden, str(device))
        g = self.__dict__.setdefault("_graphs", {}).get(key)
        if g is None:
            sid = ops.h2d(ids.int(), device)
            seos = None if eos_rows is None else ops.h2d(eos_rows, device)
            s = torch.cuda.Stream(device=device)
            s.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(s):
                self.forward(sid, output_hidden, seos)              # warm-up: allocator, GEMM plans
            torch.cuda.current_stream(device).wait_stream(s)
            from ..utils.tracing import TRACER
            graph = torch.cuda.CUDAGraph()
            with TRACER.capturing(), torch.cuda.graph(graph, capture_error_mode="thread_local"):
                out = self.forward(sid, output_hidden, seos)
            g = self._graphs[key] = (graph, sid, seos, out)
        graph, sid, seos, (hidden, pooled) = g
        sid.copy_(ids.int().pin_memory(), non_blocking=True)
        if seos is not None:
            seos.copy_(eos_rows.pin_memory(), non_blocking=True)
        graph.replay()
        h = ops.copy_(torch.empty_like(hidden), hidden)
        p = None if pooled is None else ops.copy_(torch.empty_like(pooled), pooled)
        return h, p


@dataclass
class BertConfig:
    vocab_size: int = 30522
    max_positions: int = 512
    type_vocab: int = 2
    dim: int = 384
    layers: int = 6
    heads: int = 12
    mlp: int = 1536
    eps: float = 1e-12


MINILM_L6 = BertConfig()
TINY_BERT = BertConfig(dim=32, layers=2, heads=2, mlp=64)


class PostLNBlock(nn.Module):
    def __init__(self, dim, heads, mlp, eps, gen, dtype):
        super().__init__()
        self.attention = SelfAttention(dim, heads, gen=gen, dtype=dtype, qkv_bias=True)
        self.attention_ln = LayerNorm(dim, eps, dtype)
        self.intermediate = Linear(dim, mlp, gen=gen, dtype=dtype)
        self.output = Linear(mlp, dim, gen=gen, dtype=dtype)
        self.output_ln = LayerNorm(dim, eps, dtype)

    def forward(self, x, lens):
        x = self.attention_ln(self.attention(x, residual=x, kv_lens=lens))
        return self.output_ln(self.output(self.intermediate(x, act="gelu"), residual=x))


class MiniLMEncoder(nn.Module):
    def __init__(self, cfg: BertConfig = MINILM_L6, seed: int = 0, dtype=torch.bfloat16, max_len: int = 32):
        super().__init__()
        self.cfg = cfg
        gen = torch.Generator().manual_seed(seed + 202)
        self.word_embeddings = _param((cfg.vocab_size, cfg.dim), 0.05, gen, dtype)
        self.position_embeddings = _param((cfg.max_positions, cfg.dim), 0.02, gen, dtype)
        self.token_type_embeddings = _param((cfg.type_vocab, cfg.dim), 0.02, gen, dtype)
        self.emb_ln = LayerNorm(cfg.dim, cfg.eps, dtype)
        self.layers = nn.ModuleList([PostLNBlock(cfg.dim, cfg.heads, cfg.mlp, cfg.eps, gen, dtype)
                                     for _ in range(cfg.layers)])
        self.tokenizer = bert_tokenizer(max_len, cfg.vocab_size)

    def forward(self, ids: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
        """ids [B, T], lens [B] -> L2-normalised mean-pooled embeddings [B, D] fp32."""
        # gather + position + token-type-0 add + LayerNorm in one kernel
        x = ops.embed_layer_norm(self.word_embeddings, ids, self.position_embeddings, self.token_type_embeddings[0],
                                 self.emb_ln.weight, self.emb_ln.bias, self.emb_ln.eps)
        for blk in self.layers:
            x = blk(x, lens)
        return ops.mean_pool_l2(x, lens)

    def embed(self, texts: Sequence[str], device, pad_to: Optional[int] = None) -> torch.Tensor:
        ids, lens = self.tokenizer(texts, pad_to=pad_to)
        return self.forward(ids.to(device), lens.to(device))
