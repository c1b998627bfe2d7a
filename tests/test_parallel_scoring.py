"""Sharded guess scoring (parallel/scoring.py): C1 broadcast of the batch, per-rank slice
scoring, C3 gather of the scores to rank 0 -- gloo, world sizes 2 and 3, on the CPU.

Reference behaviour being distributed: ``compute_scores`` (``/root/reference/src/backend.py:303-317``),
which scores on whichever API worker received the guess."""
import os
import tempfile
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cassmantle_amd.game.scoring import SimilarityBackend, score_pairs
from cassmantle_amd.parallel.dist import DistContext
from cassmantle_amd.parallel.scoring import ShardedSimilarity, shard_bounds
from tests.test_parallel import free_port


class _TagBackend(SimilarityBackend):
    """value = computing rank + 0.001 * local index: shows which rank scored which pair"""

    def __init__(self, rank):
        self.rank = rank
        self.calls = 0

    def similarity(self, guesses, answers):
        self.calls += 1
        return np.array([self.rank + 0.001 * i for i in range(len(guesses))], np.float32)

    def embed_words(self, words):
        return [None for _ in words]


class _HashBackend(SimilarityBackend):
    """deterministic content-only similarity (identical on every rank)"""

    def similarity(self, guesses, answers):
        return np.array([((sum(map(ord, g)) * 31 + sum(map(ord, a))) % 97) / 97.0 for g, a in zip(guesses, answers)],
                        np.float32)

    def embed_words(self, words):
        return [None for _ in words]


def _rank_main(rank, world, port, path, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = DistContext(rank, world, rank, torch.device("cpu"), "gloo")
    group = dist.new_group(backend="gloo")
    local = _HashBackend() if mode == "hash" else _TagBackend(rank)
    sh = ShardedSimilarity(ctx, local, group=group, min_pairs=8, timeout_s=2.0 if mode == "dead" else 30.0)
    if rank != 0:
        if mode == "dead":                       # never joins a scoring round, then leaves
            time.sleep(6.0)
            os._exit(0)
        sh.serve_forever()
        dist.barrier()
        dist.destroy_process_group()
        return
    out = {}
    if mode == "tag":
        for n in (8, 9, 10, 64, 100):
            g = [f"w{i}" for i in range(n)]
            out[n] = sh.similarity(g, g).tolist()
        out["small"] = sh.similarity(["a", "b"], ["c", "d"]).tolist()        # below min_pairs: local
        out["rounds"] = sh.rounds
    elif mode == "hash":
        rng = np.random.default_rng(0)
        words = ["lantern", "ember", "tower", "crystal", "river", "shadow", "glow", "stone"]
        pairs = [(words[rng.integers(8)], words[rng.integers(8)]) for _ in range(77)]
        out["sharded"] = score_pairs(sh, pairs, 0.01)
        out["local"] = score_pairs(_HashBackend(), pairs, 0.01)
    else:                                        # dead follower: timeout -> local, degraded for good
        g = [f"w{i}" for i in range(16)]
        t0 = time.monotonic()
        out["first"] = sh.similarity(g, g).tolist()
        out["t_first"] = time.monotonic() - t0
        t0 = time.monotonic()
        out["second"] = sh.similarity(g, g).tolist()
        out["t_second"] = time.monotonic() - t0
        out["degraded"] = sh.degraded
        with open(path, "w") as f:
            f.write(repr(out))
        os._exit(0)                              # the group is broken: no barrier / destroy
    sh.close()
    with open(path, "w") as f:
        f.write(repr(out))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, mode):
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "out.txt")
        mp.spawn(_rank_main, args=(world, free_port(), path, mode), nprocs=world, join=True)
        return eval(open(path).read())


def test_shard_bounds_cover_the_batch():
    for n in range(0, 40):
        for w in (1, 2, 3, 8):
            got = []
            for r in range(w):
                s, e, chunk = shard_bounds(n, w, r)
                assert e - s <= chunk
                got += list(range(s, e))
            assert got == list(range(n))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_scores_come_from_every_rank(world):
    out = _run(world, "tag")
    for n in (8, 9, 10, 64, 100):
        exp = []
        for r in range(world):
            s, e, _ = shard_bounds(n, world, r)
            exp += [r + 0.001 * i for i in range(e - s)]
        np.testing.assert_allclose(out[n], exp, rtol=0, atol=1e-6)
    assert out["small"] == pytest.approx([0.0, 0.001])       # rank 0 alone
    assert out["rounds"] == 5


def test_sharded_scoring_matches_local_scoring():
    out = _run(2, "hash")
    assert out["sharded"] == out["local"]


def test_dead_follower_degrades_to_local_scoring():
    out = _run(2, "dead")
    assert out["degraded"] and "exceeded" in out["degraded"]
    assert out["first"] == pytest.approx([0.001 * i for i in range(16)])    # rank 0 scored all of it
    assert out["second"] == out["first"]
    assert out["t_first"] < 10 and out["t_second"] < 1.0                    # no further collectives
