"""Word-vector table scorer (reference parity mode).

Reference: gensim ``KeyedVectors`` over word2vec-GoogleNews-300 (3M × 300 fp32, memory-mapped,
``src/backend.py:45``); ``wv.similarity`` = cosine of two rows (``:306``);
``most_similar`` = GEMV over the whole table + top-k (``:297-301``, unused by the game).

Here the table lives on the GPU (bf16 rows, sized for HBM: even a 3M × 300 table is 1.8 GB of
the 288 GB), and a *batch* of (guess, answer) pairs is scored by one fused HIP kernel
(``ops.gather_cosine``: row gather → L2 normalise → dot, K14).  ``most_similar`` is one
GEMV + top-k on device (K15).  Vectors come from a ``.npy`` + vocab file or a safetensors
file when provided, otherwise deterministic random vectors over the shipped word list
(``data/words.txt``) — random-init, as BASELINE.json specifies.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from ..game.scoring import SimilarityBackend

_DATA = os.path.join(os.path.dirname(os.path.dirname(__file__)), "data")


def load_vocab(path: Optional[str] = None) -> List[str]:
    path = path or os.path.join(_DATA, "words.txt")
    with open(path, encoding="utf-8") as f:
        return [ln.strip() for ln in f if ln.strip()]


class WordVectorBackend(SimilarityBackend):
    def __init__(self, vocab: Optional[Sequence[str]] = None, dim: int = 300,
                 vectors: Optional[np.ndarray] = None, device: str = "cpu",
                 dtype: torch.dtype = torch.float32, seed: int = 1234) -> None:
        self.vocab = list(vocab) if vocab is not None else load_vocab()
        self.index: Dict[str, int] = {w: i for i, w in enumerate(self.vocab)}
        if vectors is None:
            rng = np.random.default_rng(seed)
            vectors = rng.standard_normal((len(self.vocab), dim), dtype=np.float32)
        assert vectors.shape[0] == len(self.vocab)
        self.dim = vectors.shape[1]
        self.device = torch.device(device)
        self.table = torch.from_numpy(np.ascontiguousarray(vectors)).to(self.device, dtype)
        self._host = vectors

    @classmethod
    def from_files(cls, vectors_npy: str, vocab_txt: str, **kw) -> "WordVectorBackend":
        vecs = np.load(vectors_npy, allow_pickle=False)
        return cls(vocab=load_vocab(vocab_txt), vectors=vecs, **kw)

    def lookup(self, words: Sequence[str]) -> np.ndarray:
        return np.array([self.index.get(w, -1) for w in words], dtype=np.int64)

    def similarity(self, guesses: Sequence[str], answers: Sequence[str]) -> np.ndarray:
        ia = self.lookup([g.lower() for g in guesses])
        ib = self.lookup([a.lower() for a in answers])
        ta = torch.from_numpy(ia).to(self.device, torch.int32)
        tb = torch.from_numpy(ib).to(self.device, torch.int32)
        sims = ops.gather_cosine(self.table, ta, tb)  # NaN where an index is -1 (OOV)
        return sims.float().cpu().numpy()

    def embed_words(self, words: Sequence[str]) -> List[Optional[np.ndarray]]:
        # mask selection is case-sensitive in the reference (Appendix C.6); we look up
        # lower-case so that capitalised sentence-initial words are not OOV.
        out: List[Optional[np.ndarray]] = []
        for w in words:
            i = self.index.get(w.lower())
            out.append(None if i is None else self._host[i])
        return out

    def most_similar(self, word: str, topn: int = 50) -> List[Tuple[str, float]]:
        i = self.index.get(word.lower())
        if i is None:
            raise KeyError(f"Word not in dictionary: {word}")
        vals, idx = ops.cosine_topk(self.table, self.table[i], topn + 1)
        res = [(self.vocab[j], float(v)) for v, j in zip(vals.tolist(), idx.tolist()) if j != i]
        return res[:topn]
