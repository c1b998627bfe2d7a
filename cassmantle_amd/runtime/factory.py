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
        # high-priority stream: guess scoring is dispatched ahead of queued denoise kernels
        backend = EncoderBackend(device=dev, stream_priority=-1 if dev.startswith("cuda") else None)
    return BatchingScorer(backend, cfg.game.min_score, window_ms=cfg.model.scorer_batch_window_ms)


def build_prompt_generator(cfg: Config, device: Optional[str] = None):
    """synthetic (default, template grammar) | lm (local causal LM, models/lm.py) | remote
    (HF text-generation endpoint, reference parity).  ``None`` -> per-room synthetic."""
    m = cfg.model
    if m.prompt_generator == "lm":
        from ..game.prompts import LMPromptGenerator
        from ..models.lm import LM_CONFIGS, LMTextGenerator, SentencePieceTokenizer
        tok = SentencePieceTokenizer(m.lm_tokenizer) if m.lm_tokenizer else None
        gen = LMTextGenerator(LM_CONFIGS[m.lm_model], device=device, seed=m.seed, use_graphs=m.use_graphs,
                              tokenizer=tok)
        if m.lm_weights:
            from ..models.weights import load_causal_lm, read_safetensors
            load_causal_lm(gen.model, read_safetensors(m.lm_weights))
        return LMPromptGenerator(gen)
    if m.prompt_generator == "remote":
        if not m.remote_prompt_url:
            raise ValueError("prompt_generator=remote needs remote_prompt_url")
        from .remote import RemotePromptGenerator
        return RemotePromptGenerator(m.remote_prompt_url, token=m.remote_token, timeout_s=m.remote_timeout_s,
                                     max_retries=cfg.game.max_retries, retry_unit_s=m.remote_retry_s)
    return None


def build_image_generator(cfg: Config, device: Optional[str] = None) -> ImageGenerator:
    m = cfg.model
    use_gpu = (m.device == "cuda") or (m.device == "auto" and torch.cuda.is_available())
    if m.image_model == "remote":
        if not m.remote_image_url:
            raise ValueError("image_model=remote needs remote_image_url")
        from .remote import RemoteImageGenerator
        return RemoteImageGenerator(m.remote_image_url, resolution=m.resolution, token=m.remote_token,
                                    timeout_s=m.remote_timeout_s, max_retries=cfg.game.max_retries,
                                    retry_unit_s=m.remote_retry_s)
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
    if "prompt_gen" not in kw:
        kw["prompt_gen"] = build_prompt_generator(cfg)
    return GameService(cfg, scorer, image_gen_for_room=image_gen_for_room, **kw)
