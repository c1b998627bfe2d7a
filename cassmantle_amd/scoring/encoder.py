"""Sentence-embedding scorer (BASELINE config 1: MiniLM embed + cosine).

Replaces the reference's CPU word2vec cosine (``src/backend.py:303-310``).  All guesses of a
micro-batch (many sessions, see ``batcher.py``) and their answers are embedded by ONE MiniLM
forward on the GPU (fused-op encoder, mean-pool + L2 in one kernel) and compared by the fused
pair-cosine kernel.  Answer (secret-word) embeddings are cached for the round: a round has
only ``num_masked`` secrets, so steady-state batches embed guesses only.

BASELINE config 5 (live round: image generation and guess scoring on the same GPU): with
``stream_priority`` the scorer runs on its own high-priority HIP stream, so its small launches
are dispatched ahead of the queued denoise-graph kernels instead of behind them; the host sync
for the result waits on that stream only.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..game.scoring import SimilarityBackend
from ..models.text import MINILM_L6, BertConfig, MiniLMEncoder


class EncoderBackend(SimilarityBackend):
    def __init__(self, cfg: BertConfig = MINILM_L6, device: str = "cpu", seed: int = 0,
                 max_len: int = 16, dtype=torch.bfloat16, stream_priority: Optional[int] = None) -> None:
        self.device = torch.device(device)
        self.stream = None
        if stream_priority is not None and self.device.type == "cuda":
            self.stream = torch.cuda.Stream(device=self.device, priority=stream_priority)
        self.model = MiniLMEncoder(cfg, seed=seed, dtype=dtype, max_len=max_len).to(self.device).eval()
        self.max_len = max_len
        self._cache: Dict[str, torch.Tensor] = {}

    @torch.no_grad()
    def embed(self, texts: Sequence[str]) -> torch.Tensor:
        # pad to a fixed length so shapes repeat (allocator reuse, graph-friendly)
        return self.model.embed(list(texts), self.device, pad_to=self.max_len)

    def _ctx(self):
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    @torch.no_grad()
    def similarity(self, guesses: Sequence[str], answers: Sequence[str]) -> np.ndarray:
        with self._ctx():
            return self._similarity(guesses, answers)

    def _similarity(self, guesses: Sequence[str], answers: Sequence[str]) -> np.ndarray:
        missing = sorted({a for a in answers if a not in self._cache})
        uniq_g = sorted(set(guesses))
        emb = self.embed(uniq_g + missing)
        for j, a in enumerate(missing):
            self._cache[a] = emb[len(uniq_g) + j]
        if len(self._cache) > 4096:
            self._cache.clear()
        gi = {g: i for i, g in enumerate(uniq_g)}
        A = emb[[gi[g] for g in guesses]]
        Bm = torch.stack([self._cache[a] for a in answers]) if answers else A
        return ops.pair_cosine(A, Bm).float().cpu().numpy()

    @torch.no_grad()
    def embed_words(self, words: Sequence[str]) -> List[Optional[np.ndarray]]:
        if not words:
            return []
        with self._ctx():
            e = self.embed([w.lower() for w in words]).float().cpu().numpy()
        return [e[i] for i in range(len(words))]
