"""HTTP/WebSocket API — the exact contract of the reference.

Reference: ``main.py`` (FastAPI app, ``main.py:18-120``).  Routes, cookie, JSON shapes and
quirks kept byte-compatible so the browser client works unchanged:

=================  ======  ==================================================================
route              method  behaviour (reference cite)
=================  ======  ==================================================================
``/``              GET     ``static/index.html`` (``main.py:42-45``)
``/init``          GET     new uuid4 ``session_id`` cookie + session hash (``main.py:47-53``)
``/clock``         WS      every ~1 s ``{"time","reset","conns"}`` (``main.py:55-79``)
``/client/status`` GET     ``{"needInitialization":true}`` / ``{"won","needInitialization"}``
``/fetch/contents``GET     ``{"image": b64 JPEG, "prompt": view, "story": hash}`` (``:95-111``)
``/compute_score`` POST    ``{"inputs":{idx:guess}}`` -> ``{idx: "score", ..., "won"}``
``/static|/data|/media``   static files (``main.py:25-27``)
=================  ======  ==================================================================

Additions (not part of the public contract): ``?room=<id>`` on every route selects a room
(default room ``""`` = the reference's single global round); ``/metrics`` (Prometheus text,
off unless ``metrics_enabled``); ``/healthz``.
``GET /spell?word=w`` -> ``{"word","ok","suggestions"}``: the affix spell check + suggestions
of the client (static/spell.js, reference Typo.js check/suggest) on the server (game/spell.py).
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import base64
import contextlib
import logging
import os
import time
import uuid
from typing import Optional

from fastapi import Cookie, FastAPI, Request, WebSocket, WebSocketDisconnect
from fastapi.middleware.cors import CORSMiddleware
from fastapi.responses import FileResponse, JSONResponse, PlainTextResponse, Response
from fastapi.staticfiles import StaticFiles

from ..config import Config
from ..game.service import GameService
from ..utils.tracing import TRACER
from .ratelimit import RateLimiter

log = logging.getLogger("cassmantle")
PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def create_app(service: GameService, cfg: Optional[Config] = None, run_timers: bool = True,
               static_dir: Optional[str] = None) -> FastAPI:
    cfg = cfg or service.cfg
    gcfg = cfg.game
    limiter = RateLimiter(enabled=gcfg.rate_limit_enabled)

    @contextlib.asynccontextmanager
    async def lifespan(app: FastAPI):
        await service.start(run_timers=run_timers)
        try:
            yield
        finally:
            await service.stop()

    app = FastAPI(docs_url=None, redoc_url=None, lifespan=lifespan)
    app.state.service = service
    app.state.limiter = limiter
    sdir = static_dir or os.path.join(PKG, "static")
    app.mount("/static", StaticFiles(directory=sdir), name="static")
    app.mount("/data", StaticFiles(directory=os.path.join(PKG, "data")), name="data")
    app.mount("/media", StaticFiles(directory=os.path.join(PKG, "media")), name="media")
    app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=True,
                       allow_methods=["GET", "POST"], allow_headers=["*"])

    counters = {"requests": 0, "fetch_ms": 0.0, "score_ms": 0.0, "fetches": 0, "scores": 0}

    def client_key(request: Request) -> str:
        return request.client.host if request.client else "unknown"

    def limited(request: Request, route: str, rate: str) -> Optional[Response]:
        counters["requests"] += 1
        # the reference applies both the global default limit and the route's own limit
        if not limiter.hit(client_key(request), "*", gcfg.rate_default) or \
                not limiter.hit(client_key(request), route, rate):
            return JSONResponse({"error": limiter.message(rate)}, status_code=429)
        return None

    def room_of(request: Request):
        try:
            return service.room(request.query_params.get("room"))
        except KeyError:
            return None

    @app.get("/")
    async def read_root(request: Request):
        if (r := limited(request, "/", gcfg.rate_root)) is not None:
            return r
        return FileResponse(os.path.join(sdir, "index.html"))

    @app.get("/init")
    async def initialize_session(request: Request, response: Response):
        if (r := limited(request, "/init", gcfg.rate_game)) is not None:
            return r
        room = room_of(request)
        if room is None:
            return JSONResponse({"error": "unknown room"}, status_code=404)
        sid = str(uuid.uuid4())
        response.set_cookie(key="session_id", value=sid)
        room.init_client(sid)
        return {"message": "Session initialized", "session_id": sid}

    @app.websocket("/clock")
    async def connect_clock(websocket: WebSocket, session_id: Optional[str] = Cookie(None)):
        await websocket.accept()
        try:
            room = service.room(websocket.query_params.get("room"))
        except KeyError:
            await websocket.close(code=1008)
            return
        log.info("[INFO] Client %s Connected.", session_id)
        try:
            while True:
                if session_id:
                    room.add_client(session_id)
                await service.clock.sleep(gcfg.clock_period)
                await websocket.send_json({"time": room.fetch_clock(), "reset": room.reset_flag(),
                                           "conns": room.player_count()})
        except (WebSocketDisconnect, RuntimeError, asyncio.CancelledError):
            log.info("[INFO] Client Disconnected.")
        finally:
            if session_id:
                room.remove_connection(session_id)

    spell_pool = concurrent.futures.ThreadPoolExecutor(2, thread_name_prefix="spell")

    @app.get("/spell")
    async def spell(request: Request, word: str = ""):
        """server twin of the client's affix spell check (game/spell.py == static/spell.js)"""
        if (r := limited(request, "/spell", gcfg.rate_game)) is not None:
            return r
        from ..game.spell import spell_report
        w = word.strip()[:32]
        if not w.isalpha():
            return JSONResponse({"word": w, "ok": False, "suggestions": []})
        # a small executor of its own: suggestion searches never queue in front of the
        # /fetch/contents blur + JPEG work on asyncio's default executor
        loop = asyncio.get_running_loop()
        return JSONResponse(await loop.run_in_executor(spell_pool, spell_report, w, 5))

    @app.get("/client/status")
    async def check_status(request: Request, session_id: Optional[str] = Cookie(None)):
        if (r := limited(request, "/client/status", gcfg.rate_game)) is not None:
            return r
        room = room_of(request)
        if room is None or not room.session_exists(session_id):
            return JSONResponse(content={"needInitialization": True})
        scores = room.fetch_client_scores(session_id)
        return JSONResponse(content={"won": int(scores.get("won", 0)), "needInitialization": False})

    @app.get("/fetch/contents")
    async def fetch_contents(request: Request, session_id: Optional[str] = Cookie(None)):
        if (r := limited(request, "/fetch/contents", gcfg.rate_game)) is not None:
            return r
        room = room_of(request)
        if room is None:
            return JSONResponse({"error": "unknown room"}, status_code=404)
        t0 = time.perf_counter()
        minted = None
        if not session_id:
            # the reference keys such a request on a None session; here the caller gets a real
            # session AND its cookie, so repeated cookie-less calls do not pile up orphans
            session_id = minted = str(uuid.uuid4())
        if not room.session_exists(session_id):
            room.init_client(session_id)
        # store reads on the loop; only the blur + JPEG encode runs in a worker thread
        jpeg = await asyncio.to_thread(room.render_masked_image, room.masked_image_request(session_id))
        content = {
            "image": base64.b64encode(jpeg).decode(),
            "prompt": room.fetch_prompt_json(session_id),
            "story": room.fetch_story(),
        }
        counters["fetch_ms"] += (time.perf_counter() - t0) * 1e3
        counters["fetches"] += 1
        resp = JSONResponse(content=content)
        if minted:
            resp.set_cookie(key="session_id", value=minted)
        return resp

    @app.post("/compute_score")
    async def compute_score(request: Request, session_id: Optional[str] = Cookie(None)):
        if (r := limited(request, "/compute_score", gcfg.rate_game)) is not None:
            return r
        room = room_of(request)
        if room is None:
            return JSONResponse({"error": "unknown room"}, status_code=404)
        t0 = time.perf_counter()
        minted = None
        if not session_id:
            session_id = minted = str(uuid.uuid4())
        if not room.session_exists(session_id):
            room.init_client(session_id)
        try:
            data = await request.json()
            inputs = data["inputs"]
            if not isinstance(inputs, dict):
                raise TypeError("inputs must be an object")
        except Exception:  # noqa: BLE001
            return JSONResponse({"error": "body must be {\"inputs\": {index: guess}}"}, status_code=422)
        scores = await room.compute_client_scores(session_id, {str(k): str(v) for k, v in inputs.items()})
        counters["score_ms"] += (time.perf_counter() - t0) * 1e3
        counters["scores"] += 1
        resp = JSONResponse(scores)
        if minted:
            resp.set_cookie(key="session_id", value=minted)
        return resp

    @app.get("/healthz")
    async def healthz():
        sup = getattr(app.state, "supervisor", None)       # supervised multi-GPU worker group
        extra = {"workers": sup.status()} if sup is not None else {}
        return {"ok": True, **service.stats(), "stages": TRACER.snapshot(), **extra}

    @app.get("/metrics")
    async def metrics():
        if not gcfg.metrics_enabled:
            return JSONResponse({"error": "metrics disabled"}, status_code=404)
        st = service.stats()
        lines = [
            f"cassmantle_requests_total {counters['requests']}",
            f"cassmantle_rate_limited_total {limiter.rejected}",
            f"cassmantle_players {st['players']}",
            f"cassmantle_rounds_total {st['rounds']}",
            f"cassmantle_generation_errors_total {st['generation_errors']}",
            f"cassmantle_fetch_ms_sum {counters['fetch_ms']:.3f}",
            f"cassmantle_fetch_count {counters['fetches']}",
            f"cassmantle_score_ms_sum {counters['score_ms']:.3f}",
            f"cassmantle_score_count {counters['scores']}",
        ]
        for k, v in (st.get("score_latency") or {}).items():
            lines.append(f"cassmantle_score_latency_{k} {v}")
        return PlainTextResponse("\n".join(lines) + "\n" + TRACER.render_prometheus())

    return app


def build_default_app(cfg: Optional[Config] = None) -> FastAPI:
    """App wired from config: GPU pipeline + GPU scorer when a device is present, CPU
    placeholders otherwise."""
    from ..runtime.factory import build_service
    cfg = cfg or Config.from_env()
    return create_app(build_service(cfg), cfg)
