"""Room sharding over ranks (BASELINE configs 3/5) on CPU with gloo, world_size 2 and 3:
ownership table, the broadcast(C1)/gather(C2)/barrier(C4) generation round, the rank-0
coordinator that batches rooms' requests, heartbeat-based dead-rank reassignment."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cassmantle_amd.game.content import SolidImageGenerator
from cassmantle_amd.parallel.dist import DistContext
from cassmantle_amd.parallel.rooms import (STOP, GenerationCoordinator, GenJob, HeartbeatMonitor,
                                           RankImageGenerator, RankWorker, RoomSharding)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharding_table_and_reassign():
    sh = RoomSharding(["", "1", "2", "3", "4"], 3)
    assert [sh.owner(r) for r in ["", "1", "2", "3", "4"]] == [0, 1, 2, 0, 1]
    assert sh.rooms_of(2) == ["2"]
    sh.mark_dead([1])
    assert all(sh.owner(r) in (0, 2) for r in sh.room_ids)
    assert sh.state() == (1,)


class _TaggedGen(SolidImageGenerator):
    """Marks each image with the generating rank so the test can check ownership."""

    def __init__(self, rank, res=16, fail_rank=None):
        super().__init__(res)
        self.rank = rank
        self.fail_rank = fail_rank

    def generate(self, prompts, negative, seeds):
        if self.rank == self.fail_rank:
            raise RuntimeError("injected")
        out = super().generate(prompts, negative, seeds)
        for im in out:
            im[0, 0, 0] = 100 + self.rank
        return out


def _worker(rank, world, port, rooms, result_path, fail_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = DistContext(rank, world, rank, torch.device("cpu"), "gloo")
    sh = RoomSharding(rooms, world)
    w = RankWorker(ctx, _TaggedGen(rank, fail_rank=fail_rank), sh)
    if rank == 0:
        coord = GenerationCoordinator(w, window_s=0.2)
        gens = {r: RankImageGenerator(coord, r) for r in rooms}
        import concurrent.futures as cf
        with cf.ThreadPoolExecutor(len(rooms)) as ex:
            futs = {r: ex.submit(gens[r].generate, [f"prompt {r} a", f"prompt {r} b"], "neg", [1, 2]) for r in rooms}
            res = {}
            for r, f in futs.items():
                try:
                    res[r] = [int(im[0, 0, 0]) for im in f.result(timeout=60)]
                except Exception as e:  # noqa: BLE001
                    res[r] = str(type(e).__name__)
        coord.close()
        # heartbeat monitor over the default store
        store = dist.distributed_c10d._get_default_store()
        hb = HeartbeatMonitor(store, 0, world, stale_s=5.0)
        hb.beat()
        dead = hb.dead_ranks()
        with open(result_path, "w") as f:
            f.write(repr((res, dead, w.rounds)))
    else:
        w.serve_forever()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_rank", [(2, None), (3, None), (2, 1)])
def test_generation_rounds_gloo(world, fail_rank):
    rooms = ["", "1", "2", "3"]
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "res.txt")
        mp.spawn(_worker, args=(world, free_port(), rooms, path, fail_rank), nprocs=world, join=True)
        res, dead, rounds = eval(open(path).read())
    sh = RoomSharding(rooms, world)
    for i, r in enumerate(rooms):
        owner = sh.owner(r)
        if owner == fail_rank:
            assert res[r] == "ImageGenerationError"     # failed room keeps its old content
        else:
            assert res[r] == [100 + owner, 100 + owner]
    assert rounds >= 1
    # only rank 0 heart-beat in this test -> the others are reported
    assert 0 not in dead
