"""GameService: the front-end process's owner of all rooms, their round timers and persistence.

Reference: one module-level ``Server`` per uvicorn worker (``main.py:23``), each running
``startup`` + ``global_timer`` (``main.py:37-40``) against shared Redis.  Here ONE front-end
process owns every room (single writer by ownership).  The legacy endpoints serve
the default room ``""``; extra rooms (BASELINE config 3/5: concurrent rooms sharded over the
node's GPUs) are addressed with ``?room=<id>``.  Image generation for a room is delegated to
whatever :class:`~.content.ImageGenerator` the service was built with — locally on one GPU,
or to the rank worker that owns the room (``parallel.rooms``).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import random
from typing import Callable, Dict, List, Optional

from ..config import Config
from .clock import Clock
from .content import ImageGenerator, SolidImageGenerator
from .prompts import PromptGenerator, SyntheticPromptGenerator
from .room import GameRoom, Scorer
from .store import StateStore

log = logging.getLogger("cassmantle")


class GameService:
    def __init__(self, cfg: Config, scorer: Scorer,
                 image_gen_for_room: Optional[Callable[[str], ImageGenerator]] = None,
                 prompt_gen: Optional[PromptGenerator] = None,
                 clock: Optional[Clock] = None, store: Optional[StateStore] = None,
                 room_ids: Optional[List[str]] = None, seed: Optional[int] = None,
                 blur_fn=None) -> None:
        self.cfg = cfg
        self.clock = clock or Clock()
        self.store = store or StateStore(self.clock)
        self.scorer = scorer
        gen_for = image_gen_for_room or (lambda rid: SolidImageGenerator())
        ids = room_ids if room_ids is not None else [""] + [str(i) for i in range(1, cfg.game.num_rooms)]
        rng = random.Random(seed)
        self.rooms: Dict[str, GameRoom] = {}
        for rid in ids:
            self.rooms[rid] = GameRoom(cfg.game, self.store, scorer,
                                       prompt_gen=prompt_gen or SyntheticPromptGenerator(salt=hash(rid) & 0xffff),
                                       image_gen=gen_for(rid), room_id=rid, clock=self.clock,
                                       rng=random.Random(rng.random()), blur_fn=blur_fn)
        self._tasks: List[asyncio.Task] = []
        self._stop: Optional[asyncio.Event] = None
        if cfg.game.snapshot_path:
            for r in self.rooms.values():
                r.on_round.append(lambda _r: self.save_snapshot())

    def room(self, rid: Optional[str]) -> GameRoom:
        rid = rid or ""
        if rid not in self.rooms:
            raise KeyError(rid)
        return self.rooms[rid]

    # ------------------------------------------------------------------ lifecycle
    async def start(self, run_timers: bool = True) -> None:
        self.load_snapshot()
        self._stop = asyncio.Event()
        await asyncio.gather(*(r.startup() for r in self.rooms.values()))
        if run_timers:
            for r in self.rooms.values():
                self._tasks.append(asyncio.ensure_future(r.global_timer(self._stop)))

    async def stop(self) -> None:
        if self._stop is not None:
            self._stop.set()
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        self._tasks.clear()
        self.save_snapshot()

    # ------------------------------------------------------------------ checkpoint / resume (§5.4)
    def save_snapshot(self) -> None:
        path = self.cfg.game.snapshot_path
        if not path:
            return
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(self.store.dumps())
        os.replace(tmp, path)

    def load_snapshot(self) -> bool:
        path = self.cfg.game.snapshot_path
        if not path or not os.path.exists(path):
            return False
        with open(path) as f:
            self.store.loads(f.read())
        log.info("[INFO] restored state snapshot from %s", path)
        return True

    # ------------------------------------------------------------------ metrics
    def stats(self) -> dict:
        lat = getattr(self.scorer, "latency_percentiles", lambda: {})()
        return {
            "rooms": len(self.rooms),
            "players": sum(r.player_count() for r in self.rooms.values()),
            "rounds": sum(r.rounds for r in self.rooms.values()),
            "generation_errors": sum(r.generation_errors for r in self.rooms.values()),
            "score_latency": lat,
        }
