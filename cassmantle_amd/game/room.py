"""One game room: round content pipeline + session logic + round scheduler.

This is the behaviour of the reference's ``Backend`` (``src/backend.py``) and ``Server``
(``src/server.py``) classes, which at runtime are one object (``Server(Backend)``,
``src/server.py:10``).  Differences by design:

* State lives in the front-end process (:class:`~.store.StateStore`), not Redis; one writer
  per room *by ownership*, so the three Redis locks become in-process locks that still
  expire (``lock_timeout``) like the reference's.
* Content comes from pluggable generators (on-device SD pipeline, rank workers, or a
  placeholder) instead of remote HTTP; failures keep the reference's graceful degradation:
  if buffering fails the current round repeats (``src/backend.py:211-215``).
* Scoring goes through a batched scorer (many sessions' guesses per GPU launch).
* Each quirk listed in SURVEY Appendix C is either kept or fixed behind a config flag.

Key layout (Appendix B) is kept, namespaced per room: ``prompt``, ``image``, ``story``,
``sessions``, ``<session_id>``, ``countdown``, ``reset``.
"""
from __future__ import annotations

import asyncio
import hashlib
import json
import logging
import random
from typing import Any, Awaitable, Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..config import GameConfig
from .clock import Clock
from .content import ImageGenerator, SolidImageGenerator
from .imaging import BlurCache, encode_jpeg, score_to_blur
from .nlp import construct_prompt_dict, format_seconds_to_time
from .prompts import PromptGenerator, SyntheticPromptGenerator, image_prompt, load_seeds, load_styles
from .store import LockError, StateStore

log = logging.getLogger("cassmantle")


class Scorer:
    """Async scorer interface: ``await score([(guess, answer), ...]) -> [float, ...]``."""

    async def score(self, pairs: Sequence[Tuple[str, str]]) -> List[float]:  # pragma: no cover
        raise NotImplementedError

    def embed_words(self, words):  # pragma: no cover
        raise NotImplementedError


class GameRoom:
    def __init__(self, cfg: GameConfig, store: StateStore, scorer: Scorer,
                 prompt_gen: Optional[PromptGenerator] = None,
                 image_gen: Optional[ImageGenerator] = None,
                 room_id: str = "", clock: Optional[Clock] = None,
                 rng: Optional[random.Random] = None,
                 blur_fn=None) -> None:
        self.cfg = cfg
        self.store = store
        self.scorer = scorer
        self.prompt_gen = prompt_gen or SyntheticPromptGenerator()
        self.image_gen = image_gen or SolidImageGenerator()
        self.room_id = room_id
        self.clock = clock or store.clock
        self.rng = rng or random.Random()
        self.seeds = load_seeds()          # src/backend.py:31-34
        self.styles = load_styles()        # src/backend.py:36-39
        self.blur_cache = BlurCache(blur_fn=blur_fn, bucket=cfg.blur_bucket, quality=cfg.jpeg_quality)
        self._buffer_task: Optional[asyncio.Task] = None
        self._buffer_latched = False
        self.generation_errors = 0
        self.rounds = 0
        self.on_round: List[Callable[["GameRoom"], Any]] = []

    # ------------------------------------------------------------------ keys
    def k(self, name: str) -> str:
        return name if not self.room_id else f"room:{self.room_id}:{name}"

    # ------------------------------------------------------------------ story (backend.py:52-68)
    def select_style(self) -> str:
        return self.styles[self.rng.randint(0, len(self.styles) - 1)]

    def select_seed(self) -> str:
        return self.seeds[self.rng.randint(0, len(self.seeds) - 1)]

    def init_story(self, seed: str) -> None:
        self.store.hset(self.k("story"), mapping={"title": seed, "episode": 0})

    def set_next_story(self, seed: str) -> None:
        self.store.hset(self.k("story"), "next", seed)

    def reset_story(self) -> None:
        seed = self.store.hget(self.k("story"), "next")
        self.init_story(seed)
        self.store.hdel(self.k("story"), "next")

    # ------------------------------------------------------------------ generation
    async def generate_prompt(self, seed: str, is_seed: bool) -> Optional[str]:
        """``generate_prompt`` (``src/backend.py:240-268``) with the reference's retry budget."""
        self.store.hset(self.k("prompt"), "status", "busy")
        try:
            for attempt in range(self.cfg.max_retries):
                try:
                    text = await asyncio.to_thread(self.prompt_gen.generate, seed, is_seed)
                    if text:
                        return text
                except Exception as e:  # noqa: BLE001 - mirror reference's broad handling
                    log.error("[ERROR] prompt generation failed: %s", e)
                if attempt + 1 < self.cfg.max_retries:
                    # linear backoff like api_call (src/utils.py:57), in wall time: a
                    # generator failure is not a function of the game clock
                    await asyncio.sleep(self.cfg.retry_backoff * (attempt + 1))
            return None
        finally:
            self.store.hset(self.k("prompt"), "status", "idle")

    async def generate_image(self, prompt: str, seed: Optional[int] = None) -> Optional[np.ndarray]:
        """``generate_image`` (``src/backend.py:270-295``): styled prompt + negative prompt."""
        style = self.select_style()
        text = image_prompt(style, prompt, self.cfg.style_template)
        if seed is None:
            seed = int.from_bytes(hashlib.sha256(text.encode()).digest()[:4], "little")
        self.store.hset(self.k("image"), "status", "busy")
        try:
            for attempt in range(self.cfg.max_retries):
                try:
                    imgs = await asyncio.to_thread(self.image_gen.generate, [text], self.cfg.negative_prompt, [seed])
                    return imgs[0]
                except Exception as e:  # noqa: BLE001
                    log.error("[ERROR] image generation failed: %s", e)
                if attempt + 1 < self.cfg.max_retries:
                    # linear backoff like api_call (src/utils.py:57), in wall time: a
                    # generator failure is not a function of the game clock
                    await asyncio.sleep(self.cfg.retry_backoff * (attempt + 1))
            return None
        finally:
            self.store.hset(self.k("image"), "status", "idle")

    def _prompt_dict(self, prompt: str) -> Dict[str, List]:
        return construct_prompt_dict(self.scorer.embed_words, prompt, self.cfg.num_masked,
                                     distinct=not self.cfg.quirk_duplicate_masks)

    async def _make_content(self, seed: str, is_seed: bool) -> Optional[Tuple[str, str, bytes]]:
        prompt = await self.generate_prompt(seed, is_seed)
        if prompt is None:
            log.error("[ERROR] Prompt generation failed")
            return None
        image = await self.generate_image(prompt)
        if image is None:
            log.error("[ERROR] Image generation failed")
            return None
        pdict = await asyncio.to_thread(self._prompt_dict, prompt)
        jpeg = await asyncio.to_thread(encode_jpeg, image, self.cfg.jpeg_quality)
        if hasattr(image, "tensor"):           # landed in HBM (DeviceImage): blur it there
            self.blur_cache.set_source(self._version(jpeg), image)
        return prompt, json.dumps(pdict), jpeg

    # ------------------------------------------------------------------ startup (backend.py:73-129)
    async def startup(self) -> bool:
        st = self.store
        st.hset(self.k("prompt"), "status", "idle")
        st.hset(self.k("image"), "status", "idle")
        try:
            async with st.lock(self.k("startup_lock"), self.cfg.lock_timeout, self.cfg.acquire_timeout):
                has_content = st.hget(self.k("prompt"), "current") is not None and \
                    st.hget(self.k("image"), "current") is not None
                seed = self.select_seed()
                # Appendix C.9: the reference re-inits the story even when content exists.
                if self.cfg.quirk_reset_story_on_restart or not has_content or not st.exists(self.k("story")):
                    self.init_story(seed)
                seed += self.cfg.chapter_header
                if not has_content:
                    made = await self._make_content(seed, True)
                    if made is None:
                        self.generation_errors += 1
                        return False
                    prompt, pjson, jpeg = made
                    st.hset(self.k("prompt"), "seed", prompt)
                    st.hset(self.k("prompt"), "current", pjson)
                    st.hset(self.k("image"), "current", jpeg)
                    st.hset(self.k("image"), "version", self._version(jpeg))
                    st.hincrby(self.k("story"), "episode", 1)
                    log.info("[INFO] Content initialization complete")
                return True
        except LockError:
            log.info("[INFO] Worker could not acquire lock, moving on.")
            return False

    @staticmethod
    def _version(jpeg: bytes) -> str:
        return hashlib.sha1(jpeg).hexdigest()[:16]

    # ------------------------------------------------------------------ double buffering
    def random_seed(self) -> Tuple[bool, str]:
        """Story continuation policy (``src/backend.py:137-150``)."""
        eps = int(self.store.hget(self.k("story"), "episode") or 0)
        if eps < self.cfg.episode_per_story:
            seed = self.store.hget(self.k("prompt"), "seed")
            if seed is not None:
                return False, seed
        return True, self.select_seed()

    async def buffer_contents(self) -> bool:
        """``buffer_contents`` (``src/backend.py:152-202``)."""
        st = self.store
        try:
            async with st.lock(self.k("buffer_lock"), self.cfg.lock_timeout, self.cfg.acquire_timeout):
                is_seed, seed = self.random_seed()
                if is_seed:
                    log.info("[INFO] Restarting storyline.")
                    self.set_next_story(seed)
                    seed += self.cfg.chapter_header
                if st.hget(self.k("prompt"), "next") is None and st.hget(self.k("image"), "next") is None:
                    made = await self._make_content(seed, is_seed)
                    if made is None:
                        self.generation_errors += 1
                        return False
                    prompt, pjson, jpeg = made
                    st.hset(self.k("prompt"), "seed", prompt)
                    st.hset(self.k("prompt"), "next", pjson)
                    st.hset(self.k("image"), "next", jpeg)
                    log.info("[INFO] Content buffering complete")
                return True
        except LockError:
            return False
        except Exception as e:  # noqa: BLE001 - reference swallows and prints (backend.py:200-202)
            log.error("[ERROR] An unexpected error occurred: %s", e)
            self.generation_errors += 1
            return False

    async def promote_buffer(self) -> bool:
        """``promote_buffer`` (``src/backend.py:204-238``).  No buffer ⇒ round repeats."""
        st = self.store
        try:
            async with st.lock(self.k("promotion_lock"), self.cfg.lock_timeout, self.cfg.acquire_timeout):
                img = st.hget(self.k("image"), "next")
                pj = st.hget(self.k("prompt"), "next")
                if img is None or pj is None:
                    return False
                st.hset(self.k("image"), "current", img)
                st.hset(self.k("image"), "version", self._version(img))
                st.hset(self.k("prompt"), "current", pj)
                st.hdel(self.k("image"), "next")
                st.hdel(self.k("prompt"), "next")
                if st.hget(self.k("story"), "next") is not None:
                    self.reset_story()
                st.hincrby(self.k("story"), "episode", 1)
                log.info("[INFO] Buffer promotion complete")
                return True
        except LockError:
            return False

    # ------------------------------------------------------------------ sessions (server.py:26-51)
    def fetch_current_prompt(self) -> Dict[str, Any]:
        raw = self.store.hget(self.k("prompt"), "current")
        if raw is None:
            return {"tokens": [], "masks": []}
        return json.loads(raw)

    def _skey(self, session: str) -> str:
        return self.k(session) if self.room_id else session

    def session_exists(self, session: Optional[str]) -> bool:
        return bool(session) and bool(self.store.exists(self._skey(session)))

    def reset_client(self, session: str) -> None:
        prompt = self.fetch_current_prompt()
        contents: Dict[str, Any] = {"max": self.cfg.min_score, "won": 0, "attempts": 0}
        for m in prompt["masks"]:
            contents[str(m)] = 0.0
        key = self._skey(session)
        self.store.delete(key)  # stale mask keys of the previous round must not leak into the view
        self.store.hset(key, mapping=contents)
        self.store.expire(key, self.cfg.time_per_prompt)

    def init_client(self, session: str) -> None:
        self.reset_client(session)
        self.store.sadd(self.k("sessions"), session)

    def add_client(self, session: str) -> None:
        # Appendix C.1: the reference checks the misspelt key 'session'; membership add is idempotent.
        self.store.sadd(self.k("sessions"), session)

    def remove_connection(self, session: str) -> None:
        self.store.srem(self.k("sessions"), session)

    def player_count(self) -> int:
        return self.store.scard(self.k("sessions"))

    def increment_attempt(self, session: str) -> None:
        self.store.hincrby(self._skey(session), "attempts", 1)

    def fetch_client_scores(self, session: str) -> Dict[str, str]:
        return {k: (v.decode() if isinstance(v, bytes) else v)
                for k, v in self.store.hgetall(self._skey(session)).items()}

    async def compute_client_scores(self, session: str, inputs: Dict[str, str]) -> Dict[str, Any]:
        """``compute_client_scores`` + ``set_client_scores`` (``src/server.py:63-89``)."""
        prompt = self.fetch_current_prompt()
        tokens, masks = prompt["tokens"], prompt["masks"]
        keys, pairs = [], []
        for m, guess in inputs.items():
            try:
                idx = int(m)
            except (TypeError, ValueError):
                continue
            if not (0 <= idx < len(tokens)):
                continue
            if self.cfg.quirk_validate_indices and idx not in masks:
                continue  # Appendix C.3 fix: only mask positions can be probed
            keys.append(str(m))
            pairs.append((str(guess), tokens[idx]))
        if not pairs:
            # Appendix C.2: reference divides by zero (HTTP 500) on empty input.
            return {"won": int(self.fetch_client_scores(session).get("won", "0"))}
        vals = await self.scorer.score(pairs)
        scores: Dict[str, Any] = {k: str(v) for k, v in zip(keys, vals)}
        async with self.store.critical(self._skey(session)):  # atomic read-modify-write (§5.2)
            cur = self.fetch_client_scores(session)
            mean = sum(float(s) for s in scores.values()) / len(scores)
            if mean > float(cur.get("max", self.cfg.min_score)):
                self.store.hset(self._skey(session), "max", mean)
            for key, v in scores.items():
                self.store.hset(self._skey(session), key, v)
            won = int(mean == 1)
            self.store.hset(self._skey(session), "won", won)
            self.increment_attempt(session)
        scores["won"] = won
        return scores

    def fetch_prompt_json(self, session: str) -> Dict[str, Any]:
        """Per-player prompt view (``src/server.py:96-123``)."""
        prompt = self.fetch_current_prompt()
        scores = self.fetch_client_scores(session)
        attempts = int(scores.get("attempts", "0"))
        prompt["correct"] = []
        if scores.get("won") == "1":
            prompt["masks"] = []
        else:
            og = list(prompt["masks"])
            for i, mask in enumerate(og):
                s = scores.get(str(mask))
                if s and float(s) == 1.0:
                    prompt["masks"][i] = -1
                    prompt["correct"].append(mask)
                else:
                    prompt["tokens"][mask] = "*"
        prompt["scores"] = scores
        prompt["attempts"] = attempts
        return prompt

    def fetch_story(self) -> Dict[str, str]:
        return self.store.hgetall(self.k("story"))

    def masked_image_request(self, session: str) -> Optional[Tuple[str, bytes, float]]:
        """The store reads of :meth:`fetch_masked_image` — (image version, JPEG, blur radius) —
        done on the event loop so only the pure blur/encode work moves to a worker thread."""
        scores = self.fetch_client_scores(session)
        jpeg = self.store.hget(self.k("image"), "current")
        if jpeg is None:
            return None
        version = self.store.hget(self.k("image"), "version") or self._version(jpeg)
        radius = score_to_blur(float(scores.get("max", self.cfg.min_score)), self.cfg.min_blur, self.cfg.max_blur)
        return version, jpeg, radius

    def render_masked_image(self, req: Optional[Tuple[str, bytes, float]]) -> bytes:
        return b"" if req is None else self.blur_cache.get(*req)

    def fetch_masked_image(self, session: str) -> bytes:
        """Blurred JPEG by the session's best score (``src/server.py:129-133``)."""
        return self.render_masked_image(self.masked_image_request(session))

    def reset_sessions(self) -> None:
        for s in self.store.smembers(self.k("sessions")):
            self.reset_client(s)

    # ------------------------------------------------------------------ clock (server.py:139-172)
    def start_countdown(self) -> None:
        self.store.setex(self.k("countdown"), self.cfg.time_per_prompt, "active")

    def fetch_countdown(self) -> float:
        return float(self.store.ttl(self.k("countdown")))

    def fetch_clock(self) -> str:
        return format_seconds_to_time(int(self.fetch_countdown()))

    def reset_flag(self) -> bool:
        return bool(self.store.exists(self.k("reset")))

    async def tick(self) -> None:
        """One iteration of ``global_timer``'s loop body."""
        remaining = self.fetch_countdown()
        trigger = int(self.cfg.time_per_prompt * self.cfg.buffer_trigger_frac)
        if self.cfg.quirk_exact_second_trigger:
            fire = int(remaining) == trigger
        else:  # Appendix C.8 fix: latch instead of exact-second equality
            fire = (not self._buffer_latched) and 0.5 < remaining <= trigger
        if fire:
            self._buffer_latched = True
            self._buffer_task = asyncio.ensure_future(self.buffer_contents())
        if remaining <= 0.5:
            await self.end_round()

    async def end_round(self) -> None:
        await self.promote_buffer()
        self.reset_sessions()
        self.start_countdown()
        self.store.setex(self.k("reset"), 1, 1)
        self._buffer_latched = False
        self.rounds += 1
        jpeg = self.store.hget(self.k("image"), "current")
        if jpeg is not None:
            version = self.store.hget(self.k("image"), "version") or self._version(jpeg)
            # precompute blur buckets off the event loop (C.13)
            asyncio.ensure_future(asyncio.to_thread(self.blur_cache.prewarm, version, jpeg, self.cfg.max_blur))
        for cb in self.on_round:
            r = cb(self)
            if asyncio.iscoroutine(r):
                await r

    async def global_timer(self, stop: Optional[asyncio.Event] = None) -> None:
        self.start_countdown()
        await self.clock.sleep(1)
        while stop is None or not stop.is_set():
            await self.tick()
            await self.clock.sleep(1)
