"""Per-client, per-route rate limiting (slowapi parity without the dependency).

Reference: ``Limiter(key_func=get_remote_address, default_limits=["3/second"])`` plus
per-route ``@limiter.limit("2/second")`` decorators and slowapi's 429 handler
(``main.py:19-21,43,48,82,96,114``).  slowapi's fixed-window strategy is modelled with a fixed
window per (client address, route); the 429 body matches slowapi's
``{"error": "Rate limit exceeded: N per 1 second"}``.
"""
from __future__ import annotations

import time
from typing import Callable, Dict, Tuple

from ..config import parse_rate


class RateLimiter:
    def __init__(self, enabled: bool = True, now: Callable[[], float] = time.monotonic) -> None:
        self.enabled = enabled
        self.now = now
        self._windows: Dict[Tuple[str, str], Tuple[float, int]] = {}
        self.rejected = 0

    def hit(self, key: str, route: str, rate: str) -> bool:
        """Returns True if the request is allowed."""
        if not self.enabled:
            return True
        n, per = parse_rate(rate)
        t = self.now()
        start, count = self._windows.get((key, route), (t, 0))
        if t - start >= per:
            start, count = t, 0
        if count >= n:
            self.rejected += 1
            self._windows[(key, route)] = (start, count)
            return False
        self._windows[(key, route)] = (start, count + 1)
        if len(self._windows) > 100_000:  # bound memory: drop expired windows
            cutoff = t - 3600
            self._windows = {k: v for k, v in self._windows.items() if v[0] > cutoff}
        return True

    @staticmethod
    def message(rate: str) -> str:
        n, per = parse_rate(rate)
        unit = {1.0: "second", 60.0: "minute", 3600.0: "hour"}.get(per, f"{per} seconds")
        return f"Rate limit exceeded: {n} per 1 {unit}"
