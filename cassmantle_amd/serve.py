"""Server entry point.

Single GPU / CPU (reference equivalent of ``uvicorn main:app``)::

    python -m cassmantle_amd.serve --port 8000 [--num_rooms 4] [--image_model sd15] ...

Whole node, rooms data-parallel over the GPUs (one worker process per GPU, RCCL over xGMI),
supervised by the front-end (``parallel.supervisor``; a dead or wedged GPU is retired and its
rooms move to the survivors)::

    python -m cassmantle_amd.serve --gpus 8 --num_rooms 8

Legacy layout, the front-end inside rank 0 of a ``torchrun`` group (a dead rank degrades the
node to rank 0's GPU)::

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m cassmantle_amd.serve --num_rooms 8

Every worker owns the rooms ``i mod W`` and generates their images when the coordinator opens a
generation round (``parallel.rooms``).  Any ``GameConfig``/``ModelConfig`` field can be passed as
``--field value`` or ``CASSMANTLE_FIELD`` in the environment.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

WS_PROTOCOL = "cassmantle_amd.api.wsproto:RFC6455Protocol"


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if os.environ.get("CASSMANTLE_DIAG_TWICE", "0") == "1":
        print("[serve] CASSMANTLE_DIAG_TWICE=1 (a timing diagnostic with WRONG results) refused", file=sys.stderr)
        return 2
    ap = argparse.ArgumentParser(add_help=True)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--log-level", default="info")
    args, rest = ap.parse_known_args(argv)
    logging.basicConfig(level=getattr(logging, args.log_level.upper(), logging.INFO),
                        format="[%(levelname)s] %(message)s")

    from .config import Config
    cfg = Config.from_args(rest)
    world = int(os.environ.get("WORLD_SIZE", "1"))

    import uvicorn
    from .api.app import create_app
    from .runtime.factory import build_image_generator, build_service

    if world == 1 and cfg.game.gpus > 1:
        return _serve_supervised(cfg, args)
    if world == 1:
        app = create_app(build_service(cfg), cfg)
        uvicorn.run(app, host=args.host, port=args.port, ws=WS_PROTOCOL, log_level=args.log_level)
        return 0

    from .parallel import dist as cdist
    from .parallel.rooms import GenerationCoordinator, HeartbeatMonitor, RankImageGenerator, RankWorker, RoomSharding
    ctx = cdist.init_from_env()
    room_ids = [""] + [str(i) for i in range(1, max(cfg.game.num_rooms, world))]
    cfg.game.num_rooms = len(room_ids)
    gen = build_image_generator(cfg, device=str(ctx.device))
    worker = RankWorker(ctx, gen, RoomSharding(room_ids, ctx.world_size), cfg.game.negative_prompt)
    import torch.distributed as tdist
    store = tdist.distributed_c10d._get_default_store()
    hb = HeartbeatMonitor(store, ctx.rank, ctx.world_size, period_s=cfg.game.rank_heartbeat_s,
                          stale_s=cfg.game.rank_stale_s).start()
    g = cfg.game
    if g.score_topology not in ("central", "sharded"):
        raise ValueError(f"score_topology must be central or sharded, got {g.score_topology!r}")
    sharded = None
    holder = {}
    if g.score_topology == "sharded":                  # C1 + C3 on a scoring group of its own
        from .parallel.scoring import ShardedSimilarity, new_scoring_group
        from .runtime.factory import build_scorer
        sgroup = new_scoring_group(g.score_group_backend)

        def wrap(local):
            nonlocal sharded
            sharded = ShardedSimilarity(ctx, local, group=sgroup, min_pairs=g.score_shard_min,
                                        timeout_s=g.score_timeout_s,
                                        healthy=lambda: holder.get("coord") is None or holder["coord"].degraded is None)
            return sharded
        scorer = build_scorer(cfg, device=str(ctx.device), wrap=wrap)
    if ctx.rank != 0:
        st = sharded.start_serving() if sharded is not None else None
        worker.serve_forever()
        if st is not None:
            st.join(timeout=g.score_timeout_s)
        hb.stop()
        cdist.shutdown()
        return 0

    def on_degraded(reason: str) -> None:
        # rooms keep serving from rank 0's GPU; optionally hand over to a supervisor restart
        svc_ = holder.get("svc")
        if svc_ is not None:
            svc_.save_snapshot()
        if cfg.game.exit_on_rank_failure:
            logging.getLogger("cassmantle").error("[ERROR] exiting for a supervisor restart: %s", reason)
            os._exit(3)   # the collectives are unusable; no barrier / destroy on a dead group

    coord = GenerationCoordinator(worker, monitor=hb, round_timeout_s=cfg.game.round_timeout_s,
                                  on_degraded=on_degraded)
    holder["coord"] = coord
    svc = build_service(cfg, image_gen_for_room=lambda rid: RankImageGenerator(coord, rid), room_ids=room_ids,
                        scorer=scorer if sharded is not None else None)
    holder["svc"] = svc
    app = create_app(svc, cfg)
    try:
        uvicorn.run(app, host=args.host, port=args.port, ws=WS_PROTOCOL, log_level=args.log_level)
    finally:
        if sharded is not None:
            sharded.close()
        coord.close()
        hb.stop()
        if coord.degraded is None:
            cdist.shutdown()
    return 0 if coord.degraded is None else 3


def _serve_supervised(cfg, args) -> int:
    """Front-end process + supervised worker group (``parallel.supervisor``).  The group is
    spawned before this process touches the GPU (the scorer and the blur run here, on GPU 0)."""
    import uvicorn
    import torch
    from .api.app import create_app
    from .parallel.supervisor import GroupSupervisor, SupervisedImageGenerator
    from .runtime.factory import build_service
    n = cfg.game.gpus
    room_ids = [""] + [str(i) for i in range(1, max(cfg.game.num_rooms, n))]
    cfg.game.num_rooms = len(room_ids)
    devices = [f"cuda:{i}" for i in range(n)]
    # no ``local`` generator: with every GPU retired the rounds repeat (the reference's fallback)
    # until a re-probe brings devices back (cfg.game.device_reprobe_s)
    sup = GroupSupervisor(cfg, devices, room_ids, round_timeout_s=cfg.game.round_timeout_s,
                          stale_s=cfg.game.rank_stale_s, heartbeat_s=cfg.game.rank_heartbeat_s,
                          reprobe_s=cfg.game.device_reprobe_s, dispatch=cfg.game.supervisor_dispatch,
                          weights={devices[0]: cfg.game.frontend_device_weight},
                          transport=cfg.game.supervisor_transport, frontend_device=devices[0],
                          land=cfg.game.supervisor_land)
    sup.wait_ready()
    if cfg.model.scorer_stream_priority is None:
        cfg.model.scorer_stream_priority = 0      # no generation in this process (config.py)
    svc = build_service(cfg, image_gen_for_room=lambda rid: SupervisedImageGenerator(sup, rid), room_ids=room_ids)
    app = create_app(svc, cfg)
    app.state.supervisor = sup
    try:
        uvicorn.run(app, host=args.host, port=args.port, ws=WS_PROTOCOL, log_level=args.log_level)
    finally:
        sup.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
