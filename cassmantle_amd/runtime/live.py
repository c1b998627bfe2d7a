"""Live-round load model (BASELINE config 5): simulated players streaming guesses through the
micro-batching scorer while the generation pipeline draws rooms' images back to back.

The reference scores each guess with a CPU word2vec lookup while its round timer keeps buffering
the next content as an asyncio task (``/root/reference/src/server.py:152-172``,
``src/backend.py:303-317``); here generation runs on the GPU's generation stream and scoring on
the scorer's own (high-priority) stream of the same device.  ``tools/bench_live.py`` (every
topology) and ``bench.py`` (the in-process extra of the headline record) share this core.
"""
from __future__ import annotations

import asyncio
import random
import threading
import time
from typing import Callable, Dict, List, Sequence

import numpy as np

WORDS = ("lantern river tower garden mirror orchard ancient crimson hollow silent glowing ember shadow "
         "velvet frozen radiant amber comet glacier harbor meadow falcon violin").split()


async def player(scorer, rng: random.Random, stop_at: float, lat: List[float], think_ms: float) -> None:
    """One player: submit both mask guesses, wait for the scores, think 0.5-1.5 x ``think_ms``."""
    while time.perf_counter() < stop_at:
        pairs = [(rng.choice(WORDS), rng.choice(WORDS)) for _ in range(2)]
        t0 = time.perf_counter()
        await scorer.score(pairs)
        lat.append((time.perf_counter() - t0) * 1e3)
        await asyncio.sleep(think_ms / 1e3 * rng.uniform(0.5, 1.5))


async def run_players(scorer, n: int, seconds: float, think_ms: float, seed: int) -> List[float]:
    lat: List[float] = []
    stop_at = time.perf_counter() + seconds
    rngs = [random.Random(seed * 1000 + i) for i in range(n)]
    await asyncio.gather(*(player(scorer, r, stop_at, lat, think_ms) for r in rngs))
    return lat


def pct(x: Sequence[float], q: float) -> float:
    return float(np.percentile(np.asarray(x), q)) if len(x) else float("nan")


def live_round_inprocess(generate: Callable[[int], int], scorer, players: int = 64, seconds: float = 8.0,
                         think_ms: float = 250.0, idle_s: float = 0.0, seed: int = 0) -> Dict[str, float]:
    """One process, one device: a generation thread calls ``generate(step)`` (returns the number
    of images it drew, host-complete) back to back while ``players`` simulated players score on
    this thread's event loop for ``seconds``.  Images counted are those finished when the scoring
    phase ends (a generation still running then is not counted).  ``idle_s`` > 0 first measures
    the scoring latency floor with no generation running."""
    asyncio.run(run_players(scorer, min(players, 4), 0.5, think_ms, seed + 99))      # warm shapes
    idle = asyncio.run(run_players(scorer, players, idle_s, think_ms, seed)) if idle_s > 0 else []
    done = {"images": 0, "generations": 0}
    stop = threading.Event()
    err: List[BaseException] = []

    def gen_loop() -> None:
        step = 1
        try:
            while not stop.is_set():
                k = generate(step)
                done["images"] += k
                done["generations"] += 1
                step += 1
        except BaseException as e:  # noqa: BLE001 - reported by the caller
            err.append(e)

    th = threading.Thread(target=gen_loop, name="live-gen", daemon=True)
    t0 = time.perf_counter()
    th.start()
    load = asyncio.run(run_players(scorer, players, seconds, think_ms, seed + 7))
    images, generations = done["images"], done["generations"]   # one snapshot: finished work only
    elapsed = time.perf_counter() - t0
    stop.set()
    th.join()
    if err:
        raise err[0]
    out = {"images_per_s": round(images / elapsed, 3), "generations": generations,
           "load_p50_ms": round(pct(load, 50), 3), "load_p99_ms": round(pct(load, 99), 3),
           "requests": len(load), "seconds": round(elapsed, 2), "players": players}
    if idle:
        out.update(idle_p50_ms=round(pct(idle, 50), 3), idle_p99_ms=round(pct(idle, 99), 3))
    return out
