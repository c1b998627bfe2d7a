"""Typed configuration for the whole framework.

The reference hard-codes every knob in constructor defaults:
``main.py:23`` (round length 900 s), ``src/server.py:15-24`` (min_score 0.01),
``src/backend.py:20-50`` (retries, lock timeouts, masks per prompt, episodes per story),
``src/server.py:162`` (buffer trigger at 0.7 T), ``src/backend.py:319`` (blur range),
``main.py:19,43,48,82,96,114`` (rate limits).  Here they live in one dataclass with the same
defaults, overridable from the environment (``CASSMANTLE_<FIELD>``) or a CLI ``--key value``.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, List, Optional, Sequence

_ENV_PREFIX = "CASSMANTLE_"


def _coerce(value: str, typ: Any) -> Any:
    if typ in (bool, "bool"):
        return value.strip().lower() in ("1", "true", "yes", "on")
    if typ in (int, "int"):
        return int(value)
    if typ in (float, "float"):
        return float(value)
    if typ in (str, "str"):
        return value
    if typ in ("Optional[str]",):
        return None if value.lower() in ("", "none", "null") else value
    if typ in ("Optional[int]",):
        return None if value.lower() in ("", "none", "null") else int(value)
    # lists / dicts as JSON
    return json.loads(value)


@dataclass
class GameConfig:
    # --- round / scoring rules (reference defaults in effect) ---
    time_per_prompt: int = 900            # main.py:23 (Server default 600 overridden)
    min_score: float = 0.01               # src/server.py:17
    max_retries: int = 5                  # src/backend.py:23
    retry_backoff: float = 0.5            # s; reference sleeps 10*(retry+1) s on HTTP 503 (src/utils.py:57)
    lock_timeout: float = 120.0           # src/backend.py:47
    acquire_timeout: float = 2.0          # src/backend.py:48
    num_masked: int = 2                   # src/backend.py:49
    episode_per_story: int = 20           # src/backend.py:50
    buffer_trigger_frac: float = 0.7      # src/server.py:162
    min_blur: float = 0.0                 # src/backend.py:319
    max_blur: float = 15.0                # src/backend.py:319
    chapter_header: str = "\nChapter 1\n\n"   # src/backend.py:80,91
    negative_prompt: str = "blurry, distorted, fake, abstract, negative"  # src/backend.py:284
    style_template: str = "A {style} style piece depicting the following: "  # src/backend.py:272
    llm_min_new_tokens: int = 32          # src/backend.py:252
    llm_max_new_tokens: int = 96          # src/backend.py:253
    # Quirk decisions.  True = keep reference behaviour.
    quirk_exact_second_trigger: bool = False   # C.8: exact-second equality can miss; we use a latch
    quirk_duplicate_masks: bool = False        # C.4: words.index() duplicates; we pick distinct indices
    quirk_reset_story_on_restart: bool = False # C.9: restart re-inits story even if content exists
    quirk_validate_indices: bool = True        # C.3: reject indices that are not masks (False = reference)
    blur_bucket: float = 0.25             # per-score-bucket blur cache granularity (C.13 fix)
    jpeg_quality: int = 75                # PIL default quality (src/utils.py:14)
    # --- API ---
    rate_default: str = "3/second"        # main.py:19
    rate_root: str = "3/second"           # main.py:43
    rate_game: str = "2/second"           # main.py:48,82,96,114
    rate_limit_enabled: bool = True
    clock_period: float = 1.0             # main.py:63
    metrics_enabled: bool = False
    num_rooms: int = 1
    snapshot_path: Optional[str] = None   # JSON snapshot at round boundaries
    # --- multi-GPU serving ---
    # gpus > 1 without torchrun: the front-end supervises one worker process per GPU
    # (parallel/supervisor.py): a dead / wedged GPU is retired and the rooms re-sharded over the
    # survivors.  Under torchrun the legacy layout (front-end inside rank 0) is used instead.
    gpus: int = 1
    # --- multi-GPU failure handling (parallel/rooms.py; reference analog: 120 s lock TTL) ---
    rank_heartbeat_s: float = 1.0         # period of every rank's heartbeat in the PG store
    rank_stale_s: float = 30.0            # a heartbeat older than this marks the rank dead
    round_timeout_s: float = 600.0        # a generation round running longer degrades to local
    exit_on_rank_failure: bool = False    # after degrading: snapshot + exit 3 for a supervisor
    # supervised groups: once EVERY device is retired, rounds repeat (the reference's fallback,
    # src/backend.py:211-215) and the retired devices are re-probed after this long (doubling
    # per failed probe, capped at 1 h) instead of being lost for the life of the process
    device_reprobe_s: float = 120.0
    # supervised groups: "async" hands each worker its rooms' next batch as soon as THAT worker
    # is idle (a slow GPU holds only its own rooms); "lockstep" runs C1/C2/C4 collective rounds
    supervisor_dispatch: str = "async"
    # supervised async groups: how a worker's images reach the front-end.  "ipc": they stay in
    # HBM -- the worker copies them into an outbox buffer shared once through a HIP IPC handle and
    # the front-end lands them on ITS GPU with one device-to-device copy (xGMI between GPUs), where
    # the blur cache reads them; "pipe": host uint8 arrays pickled through the worker's pipe
    supervisor_transport: str = "ipc"
    # ipc landing on the front-end: "device" (copy of the worker's HBM outbox onto the front-end
    # GPU, where the blur cache reads it) or "host" (DMA into pinned memory); both at pipe speed
    supervisor_land: str = "device"
    # share of the rooms owned by the GPU the front-end's guess scorer also runs on (GPU 0);
    # the other GPUs have weight 1 (parallel.rooms.RoomSharding)
    frontend_device_weight: float = 0.85
    # --- multi-GPU guess scoring (parallel/scoring.py) ---
    score_topology: str = "central"       # central (rank 0 scores) | sharded (C1 broadcast + C3 gather)
    score_shard_min: int = 256            # sharded: smaller micro-batches are still scored on rank 0
    score_timeout_s: float = 30.0         # sharded: a slower scoring round degrades to rank-0-local
    score_group_backend: str = "gloo"     # sharded: transport of the scoring group (gloo | nccl)


@dataclass
class ModelConfig:
    # --- on-device generation (BASELINE.json configs) ---
    image_model: str = "sd15"            # sd15 | sdxl | tiny | solid
    resolution: int = 512
    steps: int = 50
    guidance_scale: float = 7.5
    scheduler: str = "pndm"               # pndm | ddim | euler
    # rooms that share one device pipeline have their concurrent generation requests batched
    # into one denoise loop (game/content.BatchingImageGenerator): up to gen_batch_max images,
    # collected for gen_batch_window_ms
    gen_batch_max: int = 4
    gen_batch_window_ms: float = 50.0
    dtype: str = "bf16"                   # bf16 (HIP kernels) | fp32 (CPU reference path only)
    device: str = "auto"                  # auto | cpu | cuda
    gpu_blur: bool = True                 # /fetch/contents blur on the GPU (HIP kernel) when present
    use_graphs: bool = True               # hipGraph-captured denoise loop
    fp8_attention: bool = False           # BASELINE config 4 (SDXL)
    weights_path: Optional[str] = None    # diffusers-layout dir (unet/ vae/ text_encoder[_2]/ *.safetensors)
    seed: int = 0
    scorer: str = "minilm"               # minilm | wordvec
    scorer_weights: Optional[str] = None  # BertModel / sentence-transformers MiniLM safetensors
    scorer_batch_window_ms: float = 1.0   # micro-batch window for streaming guess scoring
    # scorer stream priority (-1 high, 0 normal); None = high when this process also generates, normal
    # in the supervised front-end, whose GPU-0 neighbour is a worker PROCESS: there a high-priority
    # scorer cost generation 6 % more at no gain in scoring p99 (profiles/r4_live_topologies.txt)
    scorer_stream_priority: Optional[int] = None
    # CUs reserved for guess scoring on a GPU that also generates (runtime/cumask.py): the scorer
    # stream runs on these CUs only, the generation stream on the rest (0 = no reservation)
    scorer_reserved_cus: int = 0
    prompt_generator: str = "synthetic"   # synthetic | lm | remote
    lm_model: str = "tiny-lm"             # tiny-lm | mistral-7b (models/lm.py)
    lm_weights: Optional[str] = None      # HF-layout safetensors dir/file for the LM
    lm_tokenizer: Optional[str] = None    # sentencepiece model (else byte-level tokenizer)
    # --- remote generation (reference parity: HF inference endpoints, src/backend.py:24-25) ---
    remote_prompt_url: Optional[str] = None
    remote_image_url: Optional[str] = None
    remote_token: Optional[str] = None    # bearer token (reference reads it from a file)
    remote_timeout_s: float = 60.0        # src/backend.py:99,175
    remote_retry_s: float = 10.0          # backoff unit: sleep 10*(retry+1) on 503 (src/utils.py:55-57)


@dataclass
class Config:
    game: GameConfig = field(default_factory=GameConfig)
    model: ModelConfig = field(default_factory=ModelConfig)

    # ------------------------------------------------------------------
    @staticmethod
    def _apply(obj: Any, key: str, raw: str) -> bool:
        for f in fields(obj):
            if f.name == key:
                setattr(obj, key, _coerce(raw, f.type))
                return True
        return False

    def set(self, key: str, raw: str) -> None:
        key = key.replace("-", "_")
        if "." in key:
            sect, sub = key.split(".", 1)
            if not self._apply(getattr(self, sect), sub, raw):
                raise KeyError(key)
            return
        if not (self._apply(self.game, key, raw) or self._apply(self.model, key, raw)):
            raise KeyError(key)

    @classmethod
    def from_env(cls, environ: Optional[Dict[str, str]] = None) -> "Config":
        cfg = cls()
        env = os.environ if environ is None else environ
        for k, v in env.items():
            if k.startswith(_ENV_PREFIX):
                try:
                    cfg.set(k[len(_ENV_PREFIX):].lower(), v)
                except KeyError:
                    pass
        return cfg

    @classmethod
    def from_args(cls, argv: Sequence[str], base: Optional["Config"] = None) -> "Config":
        cfg = base or cls.from_env()
        it = iter(list(argv))
        for tok in it:
            if not tok.startswith("--"):
                continue
            tok = tok[2:]
            if "=" in tok:
                k, v = tok.split("=", 1)
            else:
                k, v = tok, next(it, "true")
            cfg.set(k, v)
        return cfg

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


def parse_rate(rate: str) -> tuple:
    """'3/second' -> (3, 1.0).  Accepts second/minute/hour (slowapi syntax subset)."""
    n, per = rate.split("/")
    per = per.strip().lower()
    unit = {"second": 1.0, "s": 1.0, "minute": 60.0, "m": 60.0, "hour": 3600.0, "h": 3600.0}
    if per not in unit:
        raise ValueError(f"bad rate {rate}")
    return int(n), unit[per]
