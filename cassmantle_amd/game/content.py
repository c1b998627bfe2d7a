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
import time
from typing import List, Optional, Sequence

import numpy as np


class ImageGenerationError(RuntimeError):
    pass


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
