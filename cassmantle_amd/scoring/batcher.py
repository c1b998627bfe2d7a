"""Streaming guess scorer: micro-batches concurrent requests into one device launch.

Reference: ``compute_scores`` scores one pair at a time on the request path
(``src/backend.py:312-317``).  With many players in a round the GPU scorer is latency-bound
per launch, so requests arriving within ``window_ms`` are concatenated into a single batch
(one embedding/cosine kernel for every session's guesses), executed in a worker thread so
the event loop keeps serving, and the per-request slices are returned to their awaiting
coroutines.  Latencies are recorded for the p50/p99 metric (BASELINE config 1/5).
"""
from __future__ import annotations

import collections

import asyncio
import threading
import time
from typing import Deque, List, Optional, Sequence, Tuple

import numpy as np

from ..game.room import Scorer
from ..game.scoring import SimilarityBackend, score_pairs
from ..utils.tracing import TRACER


class DirectScorer(Scorer):
    def __init__(self, backend: SimilarityBackend, min_score: float) -> None:
        self.backend = backend
        self.min_score = min_score
        self.latencies: Deque[float] = collections.deque(maxlen=4096)   # bounded window

    async def score(self, pairs):
        t0 = time.perf_counter()
        out = score_pairs(self.backend, pairs, self.min_score)
        dt = time.perf_counter() - t0
        self.latencies.append(dt)
        TRACER.observe("score_request", dt * 1e3)
        return out

    def embed_words(self, words):
        return self.backend.embed_words(words)


class BatchingScorer(Scorer):
    def __init__(self, backend: SimilarityBackend, min_score: float, window_ms: float = 1.0,
                 max_batch: int = 4096) -> None:
        self.backend = backend
        self.min_score = min_score
        self.window = window_ms / 1000.0
        self.max_batch = max_batch
        self._queue: List[Tuple[Sequence[Tuple[str, str]], asyncio.Future, float]] = []
        self._flusher: Optional[asyncio.Task] = None
        self._lock = threading.Lock()  # one device batch at a time
        self.latencies: Deque[float] = collections.deque(maxlen=4096)   # bounded window
        self.batches = 0
        self.batched_pairs = 0

    def embed_words(self, words):
        return self.backend.embed_words(words)

    async def score(self, pairs):
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._queue.append((list(pairs), fut, time.perf_counter()))
        if sum(len(p) for p, _, _ in self._queue) >= self.max_batch:
            await self._flush()
        elif self._flusher is None or self._flusher.done():
            self._flusher = asyncio.ensure_future(self._delayed_flush())
        return await fut

    async def _delayed_flush(self):
        await asyncio.sleep(self.window)
        # drain: requests that arrived while a batch was on the device are flushed as soon as it
        # returns.  (A single flush stranded them until some later request started a new
        # flusher: a scorer tail of several ms at idle, and a hang once every player was waiting
        # on a stranded request -- tools/bench_live.py --switch-ms 0.5, profiles/r3_live_cumask.txt)
        while self._queue:
            await self._flush()

    def _run(self, flat):
        with self._lock:
            t0 = time.perf_counter()
            out = score_pairs(self.backend, flat, self.min_score)
            TRACER.observe("score_batch", (time.perf_counter() - t0) * 1e3)
            return out

    async def _flush(self):
        batch, self._queue = self._queue, []
        if not batch:
            return
        flat = [pr for p, _, _ in batch for pr in p]
        try:
            vals = await asyncio.to_thread(self._run, flat)
        except Exception as e:  # noqa: BLE001
            for _, fut, _ in batch:
                if not fut.done():
                    fut.set_exception(e)
            return
        self.batches += 1
        self.batched_pairs += len(flat)
        off = 0
        now = time.perf_counter()
        for p, fut, t0 in batch:
            n = len(p)
            if not fut.done():
                fut.set_result(vals[off:off + n])
            self.latencies.append(now - t0)
            TRACER.observe("score_request", (now - t0) * 1e3)
            off += n

    def latency_percentiles(self) -> dict:
        if not self.latencies:
            return {}
        a = np.asarray(self.latencies) * 1e3
        return {"p50_ms": float(np.percentile(a, 50)), "p99_ms": float(np.percentile(a, 99)), "n": len(a)}
