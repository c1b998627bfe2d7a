"""Wiring: config -> GameService with the right scorer and image generator for this host.

* GPU present: on-device SD pipeline (``pipeline.DiffusionImageGenerator``) and the batched
  GPU scorer (MiniLM encoder or word-vector table, ``scoring``).
* CPU only (tests, dev): placeholder images, CPU scorer.
* Multi-GPU serving (``torchrun``): rank 0 builds the service with
  ``parallel.rooms.RankImageGenerator`` so each room's images come from its owner rank.
"""
from __future__ import annotations

import contextlib
import os

from typing import Callable, Optional

import numpy as np
import torch

from ..config import Config
from ..game.content import BatchingImageGenerator, ImageGenerator, SolidImageGenerator
from ..game.service import GameService
from ..scoring.batcher import BatchingScorer


_DTYPES = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32, "float32": torch.float32}


def model_dtype(cfg: Config, device: str) -> torch.dtype:
    """``ModelConfig.dtype``: the HIP kernels are bf16-only; fp32 selects the CPU reference path
    (tests / parity) and is rejected on a GPU rather than silently ignored."""
    dt = _DTYPES.get(cfg.model.dtype.lower())
    if dt is None:
        raise ValueError(f"dtype={cfg.model.dtype!r}: expected bf16 or fp32")
    if dt != torch.bfloat16 and str(device).startswith("cuda"):
        raise ValueError("dtype=fp32 runs only on the CPU reference path; the GPU kernels are bf16")
    return dt


_STREAMS: dict = {}


def reserved_streams(cfg: Config, device: str):
    """(scorer stream, generation stream) with ``scorer_reserved_cus`` CUs for the scorer, one
    pair per device and process; (None, None) when no reservation is configured."""
    n = cfg.model.scorer_reserved_cus
    if n <= 0 or not str(device).startswith("cuda"):
        return None, None
    key = (str(device), n)
    if key not in _STREAMS:
        from .cumask import reserved_streams as _rs
        _STREAMS[key] = _rs(device, n)
    return _STREAMS[key]


def build_scorer(cfg: Config, device: Optional[str] = None, wrap=None):
    """MiniLM-encoder (or word-vector) backend behind the micro-batching scorer.  ``wrap`` maps
    the local backend to the one the scorer calls (multi-GPU: ``parallel.scoring.ShardedSimilarity``)."""
    dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
    if cfg.model.scorer == "wordvec":
        from ..scoring.wordvec import WordVectorBackend
        backend = WordVectorBackend(device=dev, dtype=torch.bfloat16 if dev.startswith("cuda") else torch.float32)
    else:
        from ..scoring.encoder import EncoderBackend
        # high-priority stream: guess scoring is dispatched ahead of queued denoise kernels (the
        # supervised front-end sets cfg.model.scorer_stream_priority = 0, serve._serve_supervised)
        prio = cfg.model.scorer_stream_priority
        prio = (-1 if prio is None else prio) if dev.startswith("cuda") else None
        backend = EncoderBackend(device=dev, stream_priority=prio,
                                 dtype=model_dtype(cfg, dev), stream=reserved_streams(cfg, dev)[0])
        if cfg.model.scorer_weights:
            from ..models.weights import load_bert, read_safetensors
            missing = load_bert(backend.model, read_safetensors(cfg.model.scorer_weights))
            if missing:
                raise KeyError(f"scorer_weights: {len(missing)} tensors missing, e.g. {missing[:3]}")
    if wrap is not None:
        backend = wrap(backend)
    return BatchingScorer(backend, cfg.game.min_score, window_ms=cfg.model.scorer_batch_window_ms)


def build_blur_fn(cfg: Config, device: Optional[str] = None):
    """The /fetch/contents blur (``mask_image``, ``src/backend.py:322-324``) on the GPU: the HIP
    LDS-tiled Gaussian (ops.gaussian_blur) on its own stream.  ``None`` -> PIL on the CPU."""
    dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
    if not cfg.model.gpu_blur or not dev.startswith("cuda"):
        return None
    from .. import ops
    # the blur runs on the calling thread's current stream: a stream of its own in a process that
    # shares its GPU with a generation worker cost that worker 14 % of its images/s
    # (profiles/r6_live_ipc_stream_ab.txt); CASSMANTLE_BLUR_STREAM=own restores one
    stream = torch.cuda.Stream(device=dev) if os.environ.get("CASSMANTLE_BLUR_STREAM") == "own" else None

    def blur(img, radius: float):
        with (torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()):
            t = getattr(img, "tensor", None)        # DeviceImage: already in this GPU's HBM
            if t is not None and t.device.type == "cuda":
                x = t.to(dev, non_blocking=False)
            else:
                x = torch.from_numpy(np.ascontiguousarray(np.asarray(img))).to(dev, non_blocking=False)
            y = ops.gaussian_blur(x, radius)
            return y.cpu().numpy()
    return blur


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
    dev = device or "cuda"
    return DiffusionImageGenerator(m.image_model, device=dev, steps=m.steps,
                                   guidance=m.guidance_scale, scheduler=m.scheduler,
                                   use_graphs=m.use_graphs, fp8_attention=m.fp8_attention, seed=m.seed,
                                   dtype=model_dtype(cfg, dev), weights_path=m.weights_path,
                                   stream=reserved_streams(cfg, dev)[1])


def build_service(cfg: Config, image_gen_for_room: Optional[Callable[[str], ImageGenerator]] = None,
                  scorer=None, **kw) -> GameService:
    scorer = scorer if scorer is not None else build_scorer(cfg)
    if image_gen_for_room is None:
        # one device pipeline shared by every room: requests are serialised and batched
        gen = BatchingImageGenerator(build_image_generator(cfg), max_batch=cfg.model.gen_batch_max,
                                     window_s=cfg.model.gen_batch_window_ms / 1e3 if cfg.game.num_rooms > 1 else 0.0)
        image_gen_for_room = lambda rid: gen  # noqa: E731
    if "prompt_gen" not in kw:
        kw["prompt_gen"] = build_prompt_generator(cfg)
    if "blur_fn" not in kw:
        kw["blur_fn"] = build_blur_fn(cfg)
    return GameService(cfg, scorer, image_gen_for_room=image_gen_for_room, **kw)
