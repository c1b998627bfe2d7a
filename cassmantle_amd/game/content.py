"""Image-generation interface used by the game layer.

Reference: ``generate_image`` (``src/backend.py:270-295``) POSTs the styled prompt + negative
prompt to the remote SDXL endpoint and returns ``PIL.Image``.  Implementations here:

* :class:`SolidImageGenerator` — deterministic placeholder (tests / no-GPU front-end), with
  fault injection (``fail`` / ``slow`` / ``nan``) for the failure-handling tests.
* ``cassmantle_amd.pipeline.DiffusionImageGenerator`` — on-device SD txt2img.
* ``cassmantle_amd.parallel.rooms.RankImageGenerator`` — forwards to the GPU rank that owns
  the room (data-parallel room sharding over RCCL).
"""
from __future__ import annotations

import hashlib
import threading
import time
from typing import List, Optional, Sequence

import numpy as np


class ImageGenerationError(RuntimeError):
    pass


class DeviceImage:
    """A generated ``uint8 [H, W, 3]`` image that stays in the front-end GPU's HBM: the supervised
    workers' images land there over xGMI (``parallel.supervisor``, transport ``ipc``) and the blur
    cache reads them in place.  ``np.asarray`` / :meth:`host` give the host copy (made once, for
    the JPEG encode), so the game layer treats it like the arrays other generators return."""

    __slots__ = ("tensor", "_host")

    def __init__(self, tensor) -> None:
        self.tensor = tensor
        self._host: Optional[np.ndarray] = None

    @property
    def shape(self):
        return tuple(self.tensor.shape)

    @property
    def dtype(self):
        return np.dtype(np.uint8)

    def host(self) -> np.ndarray:
        if self._host is None:
            self._host = self.tensor.cpu().numpy()
        return self._host

    def __array__(self, dtype=None, copy=None):
        h = self.host()
        return h if dtype is None else h.astype(dtype)

    def __getitem__(self, idx):
        return self.host()[idx]


class ImageGenerator:
    resolution: int = 512

    def generate(self, prompts: Sequence[str], negative_prompt: str,
                 seeds: Sequence[int]) -> List[np.ndarray]:  # pragma: no cover - interface
        """Returns one ``uint8 [H, W, 3]`` array per prompt."""
        raise NotImplementedError


class SolidImageGenerator(ImageGenerator):
    def __init__(self, resolution: int = 64, fault: Optional[str] = None, delay: float = 0.0) -> None:
        self.resolution = resolution
        self.fault = fault
        self.delay = delay
        self.calls = 0

    def generate(self, prompts, negative_prompt, seeds):
        self.calls += 1
        if self.fault == "fail":
            raise ImageGenerationError("injected failure")
        if self.fault == "slow" or self.delay:
            time.sleep(self.delay or 0.2)
        out = []
        r = self.resolution
        for p, s in zip(prompts, seeds):
            h = hashlib.sha256(f"{p}|{s}".encode()).digest()
            base = np.frombuffer(h[:3], dtype=np.uint8).astype(np.float32)
            yy, xx = np.mgrid[0:r, 0:r].astype(np.float32) / max(1, r - 1)
            img = base[None, None, :] * (0.5 + 0.5 * yy[..., None]) + 60.0 * xx[..., None]
            if self.fault == "nan":
                img[:] = np.nan
            if not np.all(np.isfinite(img)):
                raise ImageGenerationError("non-finite image")
            out.append(np.clip(img, 0, 255).astype(np.uint8))
        return out


class _GenRequest:
    __slots__ = ("prompts", "negative", "seeds", "done", "result", "error")

    def __init__(self, prompts, negative, seeds) -> None:
        self.prompts, self.negative, self.seeds = list(prompts), negative, list(seeds)
        self.done = threading.Event()
        self.result: Optional[List[np.ndarray]] = None
        self.error: Optional[BaseException] = None


class BatchingImageGenerator(ImageGenerator):
    """Serialises and BATCHES the generation requests of several rooms that share one device
    pipeline (single-GPU serving with ``num_rooms > 1``).

    Each room calls :meth:`generate` from its own worker thread (``asyncio.to_thread``).  The
    first caller to take the run lock becomes the leader: it waits ``window_s`` for concurrent
    requests, concatenates up to ``max_batch`` images' worth of them (same negative prompt, FIFO)
    into ONE ``inner.generate`` call (one UNet batch of 2 x images with CFG) and hands every
    request its slice; the others wait on their event and lead the next batch if theirs was not
    taken.  The reference's rooms would each POST to the remote endpoint
    (``src/backend.py:270-295``); here concurrent rooms become one batched denoise loop, and the
    device pipeline is never driven by two threads at once."""

    def __init__(self, inner: ImageGenerator, max_batch: int = 4, window_s: float = 0.02) -> None:
        self.inner = inner
        self.resolution = getattr(inner, "resolution", 512)
        self.max_batch = max(1, int(max_batch))
        self.window_s = window_s
        self._q: List[_GenRequest] = []
        self._qlock = threading.Lock()
        self._run = threading.Lock()
        self.batch_sizes: List[int] = []

    def _take(self) -> List[_GenRequest]:
        with self._qlock:
            if not self._q:
                return []
            neg = self._q[0].negative
            batch, n, rest = [], 0, []
            for r in self._q:
                if r.negative == neg and (not batch or n + len(r.prompts) <= self.max_batch):
                    batch.append(r)
                    n += len(r.prompts)
                else:
                    rest.append(r)
            self._q = rest
            return batch

    def generate(self, prompts, negative_prompt, seeds):
        req = _GenRequest(prompts, negative_prompt, seeds)
        with self._qlock:
            self._q.append(req)
        while not req.done.is_set():
            if not self._run.acquire(timeout=0.005):
                continue
            try:
                if req.done.is_set():
                    break
                if self.window_s > 0:
                    time.sleep(self.window_s)      # let concurrent rooms join this batch
                batch = self._take()
                if not batch:
                    continue
                self.batch_sizes.append(sum(len(r.prompts) for r in batch))
                try:
                    imgs = self.inner.generate([p for r in batch for p in r.prompts], batch[0].negative,
                                               [s for r in batch for s in r.seeds])
                    i = 0
                    for r in batch:
                        r.result = imgs[i:i + len(r.prompts)]
                        i += len(r.prompts)
                except BaseException as e:  # noqa: BLE001 - every room of the batch sees the failure
                    for r in batch:
                        r.error = e
                for r in batch:
                    r.done.set()
            finally:
                self._run.release()
        if req.error is not None:
            raise req.error
        return req.result
