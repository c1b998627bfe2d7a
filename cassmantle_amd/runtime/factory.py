"""Wiring: config -> GameService with the right scorer and image generator for this host.

* GPU present: on-device SD pipeline (``pipeline.DiffusionImageGenerator``) and the batched
  GPU scorer (MiniLM encoder or word-vector table, ``scoring``).
* CPU only (tests, dev): placeholder images, CPU scorer.
* Multi-GPU serving (``torchrun``): rank 0 builds the service with
  ``parallel.rooms.RankImageGenerator`` so each room's images come from its owner rank.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ..config import Config
from ..game.content import ImageGenerator, SolidImageGenerator
from ..game.service import GameService
from ..scoring.batcher import BatchingScorer


def build_scorer(cfg: Config, device: Optional[str] = None):
    dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
    if cfg.model.scorer == "wordvec":
        from ..scoring.wordvec import WordVectorBackend
        backend = WordVectorBackend(device=dev, dtype=torch.bfloat16 if dev.startswith("cuda") else torch.float32)
    else:
        from ..scoring.encoder import EncoderBackend
        backend = EncoderBackend(device=dev)
    return BatchingScorer(backend, cfg.game.min_score, window_ms=cfg.model.scorer_batch_window_ms)


def build_image_generator(cfg: Config, device: Optional[str] = None) -> ImageGenerator:
    m = cfg.model
    use_gpu = (m.device == "cuda") or (m.device == "auto" and torch.cuda.is_available())
    if m.image_model == "solid" or not use_gpu:
        return SolidImageGenerator(resolution=min(m.resolution, 256))
    from ..pipeline import DiffusionImageGenerator
    return DiffusionImageGenerator(m.image_model, device=device or "cuda", steps=m.steps,
                                   guidance=m.guidance_scale, scheduler=m.scheduler,
                                   use_graphs=m.use_graphs, fp8_attention=m.fp8_attention, seed=m.seed)


def build_service(cfg: Config, image_gen_for_room: Optional[Callable[[str], ImageGenerator]] = None,
                  **kw) -> GameService:
    scorer = build_scorer(cfg)
    if image_gen_for_room is None:
        gen = build_image_generator(cfg)
        image_gen_for_room = lambda rid: gen  # noqa: E731 - one device pipeline shared by rooms
    return GameService(cfg, scorer, image_gen_for_room=image_gen_for_room, **kw)
