"""Sharded guess scoring across the ranks of a node: C1 broadcast + C3 score gather.

The reference scores every guess on the API worker that received it, one pair at a time
(``/root/reference/src/backend.py:303-317``, ``main.py:114-127``); with several uvicorn workers
the scoring load is spread over processes.  Here the front-end lives on rank 0, and there are
two topologies (``GameConfig.score_topology``):

* ``central`` (default): rank 0's micro-batching scorer (``scoring.batcher``) embeds every batch
  on its own GPU on a high-priority stream.  A 64-guess MiniLM batch is a few ms, so one GPU
  keeps up with any realistic player count and no collective sits on the request path.
* ``sharded``: each micro-batch that reaches ``score_shard_min`` pairs is split over all ranks.

  C1  rank 0 broadcasts the batch's (guess, answer) strings to every rank;
      every rank embeds and scores the contiguous slice ``[r*ceil(n/W), (r+1)*ceil(n/W))`` on
      its own device (its local backend, e.g. ``EncoderBackend`` on its GPU);
  C3  the per-rank float32 score slices, padded to ``ceil(n/W)``, are gathered to rank 0.

  The collectives run on a DEDICATED process group (created on every rank in the same order,
  right after the default group) from a dedicated thread on every rank, so they never interleave
  with the generation rounds' C1/C2/C4 on the default group.  The scoring group defaults to
  ``gloo``: its payload is host data at both ends (strings in, JSON floats out, a few KiB), so a
  host-side transport costs no H2D/D2H staging and cannot contend with RCCL's generation
  kernels for the device; ``score_group_backend="nccl"`` runs it over RCCL instead.

Failure handling mirrors ``parallel.rooms``: a collective that fails or outlives
``score_timeout_s``, or a generation coordinator that reports degraded (``healthy`` callback),
switches rank 0 to local scoring for good; the blocked collective thread is abandoned (it is a
daemon) and the process group is never used again from here.
"""
from __future__ import annotations

import concurrent.futures as cf
import logging
import threading
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from ..game.scoring import SimilarityBackend
from .dist import DistContext, broadcast_object

log = logging.getLogger("cassmantle")

STOP = "__stop__"


def shard_bounds(n: int, world: int, rank: int):
    """contiguous slice of an n-pair batch scored by ``rank`` (every rank gets ceil(n/W) but
    the last ones may get fewer or none)"""
    chunk = (n + world - 1) // world
    s = min(n, rank * chunk)
    return s, min(n, s + chunk), chunk


class ShardedSimilarity(SimilarityBackend):
    """``SimilarityBackend`` that spreads large batches over every rank (see module docstring).

    Rank 0 calls ``similarity`` (from the batching scorer's worker thread); every other rank runs
    ``serve_forever`` on a thread of its own.  ``embed_words`` / ``most_similar`` stay local."""

    def __init__(self, ctx: DistContext, local: SimilarityBackend, group=None, min_pairs: int = 256,
                 timeout_s: float = 30.0, healthy: Optional[Callable[[], bool]] = None) -> None:
        self.ctx = ctx
        self.local = local
        self.group = group
        self.min_pairs = min_pairs
        self.timeout = timeout_s
        self.healthy = healthy
        self.degraded: Optional[str] = None
        self.rounds = 0
        self.sharded_pairs = 0
        self.slice_failures = 0                      # consecutive rounds with a failed slice
        self.max_slice_failures = 3
        self._mu = threading.Lock()                  # one collective round at a time
        self._ex = cf.ThreadPoolExecutor(1, thread_name_prefix="score-collective") if ctx.rank == 0 else None
        self._closed = False

    # ------------------------------------------------------------------ helpers
    def _device(self) -> torch.device:
        be = dist.get_backend(self.group) if self.group is not None else self.ctx.backend
        return self.ctx.device if be == "nccl" else torch.device("cpu")

    def _score_slice(self, guesses: Sequence[str], answers: Sequence[str]) -> np.ndarray:
        if not guesses:
            return np.zeros((0,), np.float32)
        return np.asarray(self.local.similarity(list(guesses), list(answers)), dtype=np.float32)

    def _round(self, msg) -> Optional[np.ndarray]:
        """Collective on every rank: C1 broadcast, local slice, C3 gather.  Returns the whole
        batch's scores on rank 0, None elsewhere (or STOP)."""
        msg = broadcast_object(msg if self.ctx.rank == 0 else None, src=0, group=self.group)      # C1
        if msg == STOP:
            return STOP  # type: ignore[return-value]
        guesses, answers = msg
        W, rank = self.ctx.world_size, self.ctx.rank
        n = len(guesses)
        s, e, chunk = shard_bounds(n, W, rank)
        dev = self._device()
        buf = torch.full((max(chunk, 1),), float("nan"), dtype=torch.float32, device=dev)
        try:
            vals = self._score_slice(guesses[s:e], answers[s:e])
            if e > s:
                buf[: e - s].copy_(torch.from_numpy(vals).to(dev))
        except Exception as ex:  # noqa: BLE001 - a failed rank must still join the gather
            log.error("[ERROR] rank %d scoring failed: %s", rank, ex)
        if rank == 0:
            parts = [torch.empty_like(buf) for _ in range(W)]
            dist.gather(buf, parts, dst=0, group=self.group)                                       # C3
            self.rounds += 1
            out = torch.cat(parts)[:n].cpu().numpy()
            return self._repair(out, guesses, answers)
        dist.gather(buf, None, dst=0, group=self.group)
        self.rounds += 1
        return None

    def _repair(self, out: np.ndarray, guesses, answers) -> np.ndarray:
        """A rank whose local scoring raised leaves its slice NaN (the gather must still run):
        re-score those slices here, and stop sharding after ``max_slice_failures`` rounds in a
        row with a failed slice (a silently failing rank would otherwise turn 1/W of
        every sharded batch into min_score)."""
        W, n = self.ctx.world_size, len(guesses)
        bad_ranks = []
        for r in range(W):
            s, e, _ = shard_bounds(n, W, r)
            if e > s and not np.all(np.isfinite(out[s:e])):
                bad_ranks.append(r)
                out[s:e] = self._score_slice(guesses[s:e], answers[s:e])
        if bad_ranks:
            self.slice_failures += 1
            log.error("[ERROR] scoring slice(s) of rank(s) %s failed; re-scored on rank 0", bad_ranks)
            if self.slice_failures >= self.max_slice_failures:
                self.degrade(f"rank(s) {bad_ranks} failed their scoring slice {self.slice_failures} rounds in a row")
        else:
            self.slice_failures = 0
        return out

    def degrade(self, reason: str) -> None:
        if self.degraded is None:
            self.degraded = reason
            log.error("[ERROR] sharded scoring degraded to rank-0-local: %s", reason)

    # ------------------------------------------------------------------ rank 0
    def similarity(self, guesses: Sequence[str], answers: Sequence[str]) -> np.ndarray:
        n = len(guesses)
        if self.healthy is not None and self.degraded is None and not self.healthy():
            self.degrade("generation process group degraded")
        if (self.ctx.world_size == 1 or n < self.min_pairs or self.degraded is not None
                or self._closed or self._ex is None):
            return self.local.similarity(guesses, answers)
        with self._mu:
            fut = self._ex.submit(self._round, (list(guesses), list(answers)))
            try:
                out = fut.result(timeout=self.timeout)
            except cf.TimeoutError:
                self.degrade(f"scoring round exceeded {self.timeout:.0f} s")
                return self.local.similarity(guesses, answers)
            except Exception as ex:  # noqa: BLE001 - the group is unusable
                self.degrade(f"scoring collective failed: {type(ex).__name__}: {ex}")
                return self.local.similarity(guesses, answers)
        self.sharded_pairs += n
        return out

    def embed_words(self, words):
        return self.local.embed_words(words)

    def most_similar(self, word: str, topn: int = 50):
        return self.local.most_similar(word, topn)

    def close(self) -> None:
        """Rank 0: release the other ranks' ``serve_forever`` (skipped once degraded)."""
        if self._closed or self.ctx.rank != 0:
            return
        self._closed = True
        if self.degraded is None and self.ctx.world_size > 1:
            with self._mu:
                fut = self._ex.submit(self._round, STOP)
                try:
                    fut.result(timeout=self.timeout)
                except Exception as ex:  # noqa: BLE001
                    self.degrade(f"scoring stop failed: {ex}")
        self._ex.shutdown(wait=False)

    # ------------------------------------------------------------------ ranks != 0
    def serve_forever(self) -> None:
        """Follow rank 0's scoring rounds until STOP (or the group breaks)."""
        while True:
            try:
                if self._round(None) == STOP:
                    return
            except Exception as ex:  # noqa: BLE001 - rank 0 went away
                log.error("[ERROR] rank %d scoring loop ended: %s", self.ctx.rank, ex)
                return

    def start_serving(self) -> threading.Thread:
        t = threading.Thread(target=self.serve_forever, name="score-follower", daemon=True)
        t.start()
        return t


def new_scoring_group(backend: str = "gloo"):
    """Every rank must call this, in the same order relative to other group creations."""
    return dist.new_group(backend=backend)
