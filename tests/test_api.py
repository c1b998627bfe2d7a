"""API contract tests with Starlette's in-process TestClient: every route,
the cookie, the JSON shapes (scores as strings, won as int, masks -1 for solved ones, '*'
tokens), the /clock WebSocket message schema, static mounts, rate limiting and rooms."""
import base64
import json
import random

import numpy as np
import pytest
from fastapi.testclient import TestClient

from cassmantle_amd.api.app import create_app
from cassmantle_amd.config import Config
from cassmantle_amd.game.content import SolidImageGenerator
from cassmantle_amd.game.service import GameService
from cassmantle_amd.scoring.batcher import BatchingScorer
from cassmantle_amd.scoring.wordvec import WordVectorBackend


def make_client(rate_limit=False, rooms=1, clock_period=0.02):
    cfg = Config()
    cfg.game.rate_limit_enabled = rate_limit
    cfg.game.num_rooms = rooms
    cfg.game.clock_period = clock_period
    cfg.game.metrics_enabled = True
    vocab = ["lantern", "tower", "river", "ancient", "lamp"]
    backend = WordVectorBackend(vocab=vocab, vectors=np.random.default_rng(0).standard_normal((5, 8)).astype(np.float32))
    svc = GameService(cfg, BatchingScorer(backend, cfg.game.min_score, window_ms=0.5),
                      image_gen_for_room=lambda rid: SolidImageGenerator(48), seed=0)
    return TestClient(create_app(svc, cfg, run_timers=False)), svc


def test_full_contract_flow():
    client, svc = make_client()
    with client:
        r = client.get("/client/status")
        assert r.json() == {"needInitialization": True}
        r = client.get("/init")
        body = r.json()
        assert body["message"] == "Session initialized"
        sid = body["session_id"]
        assert client.cookies.get("session_id") == sid
        assert client.get("/client/status").json() == {"won": 0, "needInitialization": False}
        c = client.get("/fetch/contents").json()
        assert set(c) == {"image", "prompt", "story"}
        assert base64.b64decode(c["image"])[:2] == b"\xff\xd8"
        p = c["prompt"]
        assert set(p) == {"tokens", "masks", "correct", "scores", "attempts"}
        assert p["attempts"] == 0 and p["correct"] == []
        assert all(p["tokens"][m] == "*" for m in p["masks"])
        assert p["scores"]["won"] == "0" and p["scores"]["attempts"] == "0"
        st = c["story"]
        assert st["episode"] == "1" and isinstance(st["title"], str)
        # guess: wrong then exact
        room = svc.room("")
        secret = room.fetch_current_prompt()
        m0, m1 = secret["masks"]
        r = client.post("/compute_score", json={"inputs": {str(m0): "zzz", str(m1): "qqq"}}).json()
        assert r == {str(m0): "0.01", str(m1): "0.01", "won": 0}
        r = client.post("/compute_score", json={"inputs": {str(m0): secret["tokens"][m0]}}).json()
        assert r[str(m0)] == "1.0" and r["won"] == 1
        p = client.get("/fetch/contents").json()["prompt"]
        assert p["masks"] == [] and p["attempts"] == 2
        assert client.get("/client/status").json()["won"] == 1


def test_partial_solve_view():
    client, svc = make_client()
    with client:
        client.get("/init")
        room = svc.room("")
        secret = room.fetch_current_prompt()
        m0, m1 = secret["masks"]
        # solving one of two masks with a wrong second guess: mean < 1, view marks solved -1
        client.post("/compute_score", json={"inputs": {str(m0): secret["tokens"][m0], str(m1): "zzz"}})
        p = client.get("/fetch/contents").json()["prompt"]
        assert p["masks"] == [-1, m1] and p["correct"] == [m0]
        assert p["tokens"][m0] == secret["tokens"][m0] and p["tokens"][m1] == "*"


def test_clock_websocket_schema():
    client, svc = make_client()
    with client:
        client.get("/init")
        with client.websocket_connect("/clock") as ws:
            msg = ws.receive_json()
            assert set(msg) == {"time", "reset", "conns"}
            assert isinstance(msg["reset"], bool) and msg["conns"] >= 1
            assert len(msg["time"]) == 5 and msg["time"][2] == ":"


def test_static_mounts_and_root():
    client, _ = make_client()
    with client:
        assert "CassMantle" in client.get("/").text
        assert client.get("/static/script.js").status_code == 200
        assert client.get("/data/seeds.txt").status_code == 200
        assert "lantern" in client.get("/data/words.txt").text
        assert client.get("/media/logo.svg").status_code == 200


def test_rate_limit_429():
    client, _ = make_client(rate_limit=True)
    with client:
        codes = [client.get("/client/status").status_code for _ in range(5)]
        assert codes[:2] == [200, 200] and 429 in codes
        r = [client.get("/client/status") for _ in range(3)][-1]
        assert r.json()["error"].startswith("Rate limit exceeded")


def test_rooms_are_isolated():
    client, svc = make_client(rooms=3)
    with client:
        a = client.get("/init?room=1").json()["session_id"]
        c = client.get("/fetch/contents?room=2").json()
        assert c["story"]["episode"] == "1"
        assert client.get("/fetch/contents?room=9").status_code == 404
        assert svc.room("1").player_count() == 1 and svc.room("2").player_count() == 1
        assert svc.room("").player_count() == 0


def test_bad_score_body():
    client, _ = make_client()
    with client:
        client.get("/init")
        assert client.post("/compute_score", json={"nope": 1}).status_code == 422


def test_metrics_and_health():
    client, _ = make_client()
    with client:
        assert client.get("/healthz").json()["ok"] is True
        assert "cassmantle_requests_total" in client.get("/metrics").text


def test_cookieless_requests_get_a_session_cookie_not_orphans():
    """a request without the cookie is served as a fresh session AND gets the cookie, so
    repeated calls reuse it instead of piling up orphan session members"""
    client, svc = make_client()
    with client:
        room = svc.room("")
        r = client.get("/fetch/contents")
        sid = r.cookies.get("session_id")
        assert sid and room.session_exists(sid)
        n = room.player_count()
        for _ in range(3):                  # the client now sends the cookie
            client.get("/fetch/contents")
            client.post("/compute_score", json={"inputs": {}})
        assert room.player_count() == n


def test_round_boundary_prewarms_blur_cache_1024():
    """end_round promotes the buffered 1024^2 image and precomputes every blur bucket off the
    event loop; a page view at any score is then a cache hit (Appendix C.13 fix)"""
    import asyncio
    import time
    cfg = Config()
    cfg.game.rate_limit_enabled = False
    cfg.game.blur_bucket = 1.0
    backend = WordVectorBackend(vocab=["lantern", "tower"], vectors=np.eye(2, dtype=np.float32))
    svc = GameService(cfg, BatchingScorer(backend, cfg.game.min_score),
                      image_gen_for_room=lambda rid: SolidImageGenerator(1024), seed=0)
    client = TestClient(create_app(svc, cfg, run_timers=False))
    with client:
        room = svc.room("")
        client.portal.call(room.buffer_contents)
        client.portal.call(room.end_round)
        cache = room.blur_cache
        deadline = time.time() + 60
        while len(cache) < 16 and time.time() < deadline:     # 0..15 in 1.0 buckets
            time.sleep(0.05)
        assert cache.misses == 16 and len(cache) == 16
        client.get("/init")
        hits = cache.hits
        img = base64.b64decode(client.get("/fetch/contents").json()["image"])
        assert img[:2] == b"\xff\xd8" and cache.hits == hits + 1


def test_media_assets_served():
    """procedurally generated media (tools/make_media.py) stand in for the reference's media/"""
    client, _ = make_client()
    with client:
        png = client.get("/media/background.png")
        assert png.status_code == 200 and png.content[:8] == b"\x89PNG\r\n\x1a\n"
        ico = client.get("/media/icon.ico")
        assert ico.status_code == 200 and ico.content[:4] == b"\x00\x00\x01\x00"
        for name in ("person-circle.svg", "code-mark.svg", "logo.svg"):
            assert client.get(f"/media/{name}").status_code == 200
        page = client.get("/").text
        assert "/static/spell.js" in page and "/media/icon.ico" in page
