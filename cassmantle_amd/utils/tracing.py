"""Per-stage timing: histograms of encode / denoise / decode / score / blur+JPEG.

The reference has no tracing at all — only ``print`` lines around its HTTP calls and generation
phases (``/root/reference/src/utils.py:45,49``, ``/root/reference/src/backend.py:241,274``).
Here every stage of a round lands in a fixed-bucket histogram that ``/metrics`` renders in the
Prometheus text format and ``bench.py`` / ``/healthz`` can read as a dict.

GPU stages are timed with HIP events recorded on the stage's own stream (the pipeline's
generation stream, the scorer's high-priority stream).  Recording an event never blocks the
host, so the denoise hot loop gains no synchronisation: finished event pairs are resolved lazily
(``event.query()``) the next time anyone opens a span or reads the tracer.  Host stages use
``time.perf_counter``.  ``profile_to`` wraps ``torch.profiler`` (ROCm: roctracer activity) for
a one-off chrome trace of a region.
"""
from __future__ import annotations

import bisect
import contextlib
import os
import threading
import time
from collections import deque
from typing import Deque, Dict, Iterator, List, Optional, Sequence, Tuple

# milliseconds: sub-ms scorer batches up to a multi-second SDXL denoise loop
DEFAULT_BUCKETS_MS: Tuple[float, ...] = (0.25, 0.5, 1, 2.5, 5, 10, 25, 50, 100, 250, 500,
                                         1000, 2500, 5000, 10000, 30000)


class Histogram:
    """Cumulative-bucket histogram (Prometheus semantics: ``le`` upper bounds, +Inf last)."""

    def __init__(self, name: str, buckets: Sequence[float] = DEFAULT_BUCKETS_MS) -> None:
        self.name = name
        self.bounds: List[float] = sorted(float(b) for b in buckets)
        self.counts: List[int] = [0] * (len(self.bounds) + 1)
        self.sum = 0.0
        self.count = 0
        self.max = 0.0
        self._recent: Deque[float] = deque(maxlen=1024)   # for exact recent percentiles

    def observe(self, ms: float) -> None:
        self.counts[bisect.bisect_left(self.bounds, ms)] += 1
        self.sum += ms
        self.count += 1
        self.max = max(self.max, ms)
        self._recent.append(ms)

    def percentile(self, q: float) -> Optional[float]:
        if not self._recent:
            return None
        a = sorted(self._recent)
        return a[min(len(a) - 1, int(round(q / 100.0 * (len(a) - 1))))]

    def render(self, metric: str) -> List[str]:
        lines, acc = [], 0
        for b, c in zip(self.bounds, self.counts):
            acc += c
            lines.append(f'{metric}_bucket{{stage="{self.name}",le="{b:g}"}} {acc}')
        acc += self.counts[-1]
        lines.append(f'{metric}_bucket{{stage="{self.name}",le="+Inf"}} {acc}')
        lines.append(f'{metric}_sum{{stage="{self.name}"}} {self.sum:.6f}')
        lines.append(f'{metric}_count{{stage="{self.name}"}} {self.count}')
        return lines


class Tracer:
    """Process-wide registry of stage histograms plus pending GPU event pairs."""

    MAX_PENDING = 4096

    def __init__(self, enabled: bool = True) -> None:
        self.enabled = enabled
        self._hist: Dict[str, Histogram] = {}
        self._pending: Deque[Tuple[str, object, object]] = deque()
        self._lock = threading.Lock()
        self._capturing = 0

    # ---------------------------------------------------------------- recording
    def observe(self, stage: str, ms: float) -> None:
        if not self.enabled:
            return
        with self._lock:
            h = self._hist.get(stage)
            if h is None:
                h = self._hist[stage] = Histogram(stage)
            h.observe(float(ms))

    @contextlib.contextmanager
    def span(self, stage: str, stream=None) -> Iterator[None]:
        """Time the enclosed region.  With a ``torch.cuda.Stream`` the region is timed on the
        device (events on that stream, no host sync); otherwise wall-clock on the host."""
        if not self.enabled:
            yield
            return
        if stream is None:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self.observe(stage, (time.perf_counter() - t0) * 1e3)
            return
        import torch
        start = torch.cuda.Event(enable_timing=True)
        end = torch.cuda.Event(enable_timing=True)
        start.record(stream)
        try:
            yield
        finally:
            end.record(stream)
            with self._lock:
                self._pending.append((stage, start, end))
                while len(self._pending) > self.MAX_PENDING:   # nobody is reading: drop oldest
                    self._pending.popleft()
            self.poll()

    @contextlib.contextmanager
    def capturing(self):
        """Mark a hipGraph capture in progress: event queries from other threads (a /metrics
        scrape on the event loop) are then deferred, since a query during a global-mode
        capture is a prohibited call that can invalidate the capture."""
        with self._lock:
            self._capturing += 1
        try:
            yield
        finally:
            with self._lock:
                self._capturing -= 1

    def poll(self) -> int:
        """Resolve every completed GPU span (in order; stops at the first unfinished one).
        A no-op while any graph capture is in progress (see :meth:`capturing`)."""
        done = []
        with self._lock:
            if self._capturing:
                return 0
            while self._pending:
                stage, s, e = self._pending[0]
                if not e.query():
                    break
                self._pending.popleft()
                done.append((stage, s.elapsed_time(e)))
        for stage, ms in done:
            self.observe(stage, ms)
        return len(done)

    def flush(self) -> None:
        """Block until every pending GPU span has finished and record it (tests, bench end)."""
        with self._lock:
            pend = list(self._pending)
        for _, _, e in pend:
            e.synchronize()
        self.poll()

    # ---------------------------------------------------------------- reading
    def stages(self) -> List[str]:
        self.poll()
        with self._lock:
            return sorted(self._hist)

    def histogram(self, stage: str) -> Optional[Histogram]:
        self.poll()
        with self._lock:
            return self._hist.get(stage)

    def snapshot(self) -> Dict[str, Dict[str, float]]:
        self.poll()
        out = {}
        with self._lock:
            for k, h in sorted(self._hist.items()):
                out[k] = {"count": h.count, "sum_ms": round(h.sum, 4),
                          "mean_ms": round(h.sum / max(h.count, 1), 4),
                          "p50_ms": h.percentile(50), "p99_ms": h.percentile(99),
                          "max_ms": round(h.max, 4)}
        return out

    def render_prometheus(self, metric: str = "cassmantle_stage_ms") -> str:
        self.poll()
        lines = [f"# HELP {metric} Per-stage latency in milliseconds (device time for GPU stages).",
                 f"# TYPE {metric} histogram"]
        with self._lock:
            for _, h in sorted(self._hist.items()):
                lines.extend(h.render(metric))
        return "\n".join(lines) + "\n"

    def reset(self) -> None:
        with self._lock:
            self._hist.clear()
            self._pending.clear()


TRACER = Tracer(enabled=os.environ.get("CASSMANTLE_TRACE", "1") != "0")


def span(stage: str, stream=None):
    return TRACER.span(stage, stream)


@contextlib.contextmanager
def profile_to(path: str, cuda: bool = True) -> Iterator[object]:
    """One-off ``torch.profiler`` region exported as a chrome trace at ``path``."""
    import torch
    acts = [torch.profiler.ProfilerActivity.CPU]
    if cuda and torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        yield prof
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    prof.export_chrome_trace(path)
