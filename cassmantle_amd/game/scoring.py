"""Guess-scoring rules and the scorer interface.

Reference rules (``compute_score``, ``src/backend.py:303-310``): lower-case both strings;
exact match → 1.0; otherwise cosine similarity of the two word vectors; OOV → ``min_score``;
clamp below at ``min_score`` (negative cosines therefore read 0.01, Appendix C.7).
``compute_scores`` (``:312-317``) loops pair by pair and stringifies each float.

Here a :class:`SimilarityBackend` scores a whole *batch* of (guess, answer) pairs in one call
(one GPU launch for many players' guesses), and :func:`apply_rules` wraps it with the exact
reference rules so every backend shares them.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np


class SimilarityBackend:
    """Batched raw cosine similarity.  Returns NaN for a pair that has no embedding (OOV)."""

    def similarity(self, guesses: Sequence[str], answers: Sequence[str]) -> np.ndarray:  # pragma: no cover
        raise NotImplementedError

    def embed_words(self, words: Sequence[str]) -> List[Optional[np.ndarray]]:  # pragma: no cover
        """Vectors used by mask selection (``semantic_distance``)."""
        raise NotImplementedError

    def most_similar(self, word: str, topn: int = 50) -> List[Tuple[str, float]]:
        """``wv.most_similar`` parity (``src/backend.py:297-301``; unused by the game)."""
        raise NotImplementedError


def apply_rules(guesses: Sequence[str], answers: Sequence[str], raw: np.ndarray,
                min_score: float) -> List[float]:
    out: List[float] = []
    for g, a, s in zip(guesses, answers, np.asarray(raw, dtype=np.float64)):
        if g.lower() == a.lower():
            out.append(1.0)
        elif not np.isfinite(s):
            out.append(float(min_score))
        else:
            out.append(float(max(min_score, min(float(s), 1.0))))
    return out


def score_pairs(backend: SimilarityBackend, pairs: Sequence[Tuple[str, str]],
                min_score: float) -> List[float]:
    if not pairs:
        return []
    g = [p[0].lower() for p in pairs]
    a = [p[1].lower() for p in pairs]
    raw = backend.similarity(g, a)
    return apply_rules(g, a, raw, min_score)
