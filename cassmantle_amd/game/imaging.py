"""Image masking (score → blur) and JPEG transport.

Reference: ``score_to_blur`` = ``min + (1 - s²)(max - min)`` (``src/backend.py:319-320``) and
``mask_image`` = PIL ``GaussianBlur`` (``src/backend.py:322-324``), recomputed from the full
JPEG on every ``/fetch/contents`` (``src/server.py:129-133``, Appendix C.13), then JPEG +
base64 (``main.py:101-107``).  Here the blur radius is quantised into buckets and each
(content version, bucket) JPEG is cached, so a page view costs a dict lookup; the blur itself
runs on the GPU (``ops.gaussian_blur``, HIP separable kernel) when the content was generated
there, else PIL on the CPU.
"""
from __future__ import annotations

import io
import math
import threading
from collections import OrderedDict
from typing import Callable, Optional, Tuple

import numpy as np
from PIL import Image, ImageFilter

from ..utils.tracing import TRACER


def score_to_blur(score: float, min_blur: float = 0.0, max_blur: float = 15.0) -> float:
    return min_blur + (1.0 - score ** 2) * (max_blur - min_blur)


def encode_jpeg(img, quality: int = 75) -> bytes:
    """``encode_image`` parity (``src/utils.py:12-16``; PIL default quality is 75).  ``img``: a
    PIL image, a uint8 array, or anything ``np.asarray`` turns into one (``DeviceImage``)."""
    if not isinstance(img, Image.Image):
        img = Image.fromarray(np.asarray(img))
    if img.mode != "RGB":
        img = img.convert("RGB")
    buf = io.BytesIO()
    img.save(buf, format="JPEG", quality=quality)
    return buf.getvalue()


def decode_jpeg(data: bytes) -> np.ndarray:
    return np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))


def blur_pil(img: np.ndarray, radius: float) -> np.ndarray:
    img = np.asarray(img)
    if radius <= 0:
        return img
    return np.asarray(Image.fromarray(img).filter(ImageFilter.GaussianBlur(radius)))


def quantize_radius(radius: float, bucket: float) -> float:
    if bucket <= 0:
        return radius
    return round(radius / bucket) * bucket


BlurFn = Callable[[np.ndarray, float], np.ndarray]


class BlurCache:
    """LRU of blurred JPEGs keyed by (content version, radius bucket)."""

    def __init__(self, blur_fn: Optional[BlurFn] = None, bucket: float = 0.25,
                 quality: int = 75, capacity: int = 256) -> None:
        self.blur_fn = blur_fn or blur_pil
        self.bucket = bucket
        self.quality = quality
        self.capacity = capacity
        self._lru: "OrderedDict[Tuple[str, float], bytes]" = OrderedDict()
        self._decoded: Tuple[Optional[str], Optional[np.ndarray]] = (None, None)
        # version -> device-resident source image (DeviceImage) of content generated on a GPU:
        # the blur reads it in HBM instead of decoding the JPEG (bounded: current + next content)
        self._sources: "OrderedDict[str, object]" = OrderedDict()
        self._lock = threading.Lock()
        self.hits = 0
        self.misses = 0

    def __len__(self) -> int:
        with self._lock:
            return len(self._lru)

    def set_source(self, version: str, img) -> None:
        """Register the device-resident original of content ``version`` (see ``_sources``)."""
        with self._lock:
            self._sources[version] = img
            self._sources.move_to_end(version)
            while len(self._sources) > 4:
                self._sources.popitem(last=False)

    def get(self, version: str, jpeg: bytes, radius: float) -> bytes:
        r = quantize_radius(radius, self.bucket)
        key = (version, r)
        with self._lock:
            if key in self._lru:
                self._lru.move_to_end(key)
                self.hits += 1
                return self._lru[key]
            self.misses += 1
            arr = self._sources.get(version)
            if arr is None:
                ver, arr = self._decoded
                if ver != version:
                    arr = decode_jpeg(jpeg)
                    self._decoded = (version, arr)
        with TRACER.span("blur_jpeg"):
            out = encode_jpeg(self.blur_fn(arr, r), self.quality) if r > 0 else jpeg
        with self._lock:
            self._lru[key] = out
            while len(self._lru) > self.capacity:
                self._lru.popitem(last=False)
        return out

    def prewarm(self, version: str, jpeg: bytes, max_blur: float) -> int:
        """Precompute every bucket for a freshly promoted image (round boundary)."""
        n = 0
        steps = int(math.ceil(max_blur / self.bucket)) if self.bucket > 0 else 0
        for i in range(steps + 1):
            self.get(version, jpeg, i * self.bucket)
            n += 1
        return n
