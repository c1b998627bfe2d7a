"""Injectable clocks.

The reference's round scheduler reads wall time implicitly through Redis TTLs and
``asyncio.sleep`` (``src/server.py:139-172``).  Every time-dependent component here takes a
``Clock`` so tests can drive a whole 900 s round in microseconds with :class:`FakeClock`.
"""
from __future__ import annotations

import asyncio
import time
from typing import List, Tuple


class Clock:
    def now(self) -> float:
        return time.monotonic()

    async def sleep(self, seconds: float) -> None:
        await asyncio.sleep(max(0.0, seconds))


class FakeClock(Clock):
    """Manually advanced clock.  ``sleep`` parks the coroutine until ``advance`` passes its
    deadline, so ``global_timer`` style loops can be stepped deterministically."""

    def __init__(self, start: float = 1000.0) -> None:
        self._t = float(start)
        self._waiters: List[Tuple[float, asyncio.Future]] = []

    def now(self) -> float:
        return self._t

    async def sleep(self, seconds: float) -> None:
        if seconds <= 0:
            await asyncio.sleep(0)
            return
        fut = asyncio.get_event_loop().create_future()
        self._waiters.append((self._t + seconds, fut))
        await fut

    async def advance(self, seconds: float, step: float = 0.25) -> None:
        """Advance time in ``step`` increments, letting woken coroutines run at each tick."""
        end = self._t + seconds
        while self._t < end - 1e-12:
            self._t = min(end, self._t + step)
            due = [w for w in self._waiters if w[0] <= self._t + 1e-9]
            self._waiters = [w for w in self._waiters if w[0] > self._t + 1e-9]
            for _, fut in due:
                if not fut.done():
                    fut.set_result(None)
            # let woken tasks (and what they spawn) run until quiescent
            for _ in range(20):
                await asyncio.sleep(0)
