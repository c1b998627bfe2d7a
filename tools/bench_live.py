"""BASELINE config 5: a live round — image generation and streaming guess scoring overlapped.

The SERVING topology (``serve.py``): every rank (one per GPU, ``torchrun`` for N > 1) generates
its rooms' content; guess scoring runs on rank 0, next to the front-end that owns every session
(a guess costs microseconds of GPU time, so a cross-rank hop would only add latency), unless
``--score-topology sharded`` (serve.py's ``score_topology=sharded``) splits large micro-batches
over every rank with a C1 broadcast + C3 score gather (``parallel/scoring.py``):

* on every rank a generation thread replays the hipGraph-captured SD-1.5 denoise loop back to
  back (batch 4 images per room, 512², 50 PNDM steps) on the pipeline's own stream;
* on rank 0 an asyncio loop runs ``--players`` simulated players; each submits its two mask
  guesses, waits for the scores, "thinks" for a random 0.5–1.5 × ``--think-ms`` and repeats.
  Requests go through the micro-batching scorer (``scoring.batcher``), whose graph-replayed
  MiniLM embed + cosine runs on a HIGH-PRIORITY stream (``EncoderBackend(stream_priority=-1)``)
  so scoring kernels are dispatched ahead of queued denoise kernels.

Phases: ``--idle-s`` seconds of scoring alone (latency floor), then ``--seconds`` with both.
Rank 0 prints one JSON line: whole-job images/s during the overlapped phase, p50/p99 guess
latency idle vs under load (max over ranks), and requests served.

    python tools/bench_live.py --seconds 30
    python tools/bench_live.py --gpus 8 --players 64          # the supervised topology serve.py uses
    torchrun --nproc-per-node 8 tools/bench_live.py --players 64   # the legacy torchrun layout

``--gpus N`` (no torchrun environment) runs the topology ``serve.py --gpus N`` really uses: this
process is the front-end; it spawns one supervised worker process per GPU BEFORE it touches a
GPU (``parallel.supervisor.GroupSupervisor``), then scores on GPU 0 beside worker 0.  Every
generation round gives each of the N rooms (one per GPU) its ``--batch`` images: C1 job list to
the workers, local generation, C2 device-resident gather to the group leader, one pipe hop of
uint8 images to the front-end.  ``--model tiny`` runs the same topology on the CPU (gloo).
"""
import argparse
import asyncio
import json
import os
import random
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--players", type=int, default=64, help="total over all ranks")
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--idle-s", type=float, default=8.0)
    ap.add_argument("--think-ms", type=float, default=250.0)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--model", default="sd15")
    ap.add_argument("--priority", type=int, default=None,
                    help="scorer stream priority (lower = higher); default -1 in-process, 0 in the supervised "
                         "front-end (as serve.py: config.ModelConfig.scorer_stream_priority)")
    ap.add_argument("--no-priority", action="store_true",
                    help="A/B: score on a normal-priority side stream (the scorer always owns a stream: "
                         "on the legacy default stream it queued behind whole generations, "
                         "pipeline.StableDiffusion.generate_tensor docstring)")
    ap.add_argument("--window-ms", type=float, default=1.0)
    ap.add_argument("--switch-ms", type=float, default=None,
                    help="sys.setswitchinterval for the process (ms); default: Python's 5 ms")
    ap.add_argument("--exclusive-scorer", action="store_true",
                    help="mask the scorer to the reserved CUs too (default: scorer on all CUs)")
    ap.add_argument("--reserve-cus", type=int, default=0,
                    help="CUs reserved for the scorer (CU-masked streams, runtime/cumask.py); 0 = none")
    ap.add_argument("--score-topology", choices=("central", "sharded"), default="central",
                    help="as serve.py's GameConfig.score_topology: rank-0 scoring, or micro-batches of "
                         ">= --shard-min pairs split over every rank (C1 broadcast + C3 gather, parallel/scoring.py)")
    ap.add_argument("--shard-min", type=int, default=256)
    ap.add_argument("--dispatch", choices=("async", "lockstep"), default="async",
                    help="supervised topology: per-worker (async) or collective (lockstep) rounds")
    ap.add_argument("--transport", choices=("ipc", "pipe"), default="ipc",
                    help="supervised async data plane: images land on GPU 0 from the workers' HBM "
                         "outboxes (ipc) or travel as host arrays through the pipes (pipe)")
    ap.add_argument("--land", choices=("host", "device"), default="device",
                    help="ipc transport: land each round in pinned host memory (DMA) or on GPU 0")
    ap.add_argument("--weight0", type=float, default=None,
                    help="room share of GPU 0 (the scorer's device); default config.frontend_device_weight")
    ap.add_argument("--slots-per-gpu", type=int, default=1,
                    help="supervised workers per GPU (>1 runs gloo; a one-GPU rehearsal of several workers)")
    ap.add_argument("--gpus", type=int, default=None,
                    help="supervised topology on this many devices (front-end + one worker process each)")
    return ap.parse_args()


from cassmantle_amd.runtime.live import pct, run_players  # noqa: E402  (shared with bench.py)


def main_supervised(a) -> None:
    """The serving topology of ``serve.py --gpus N``: front-end (scoring, game state) plus a
    supervised worker group (generation), see the module docstring."""
    from cassmantle_amd.config import Config
    from cassmantle_amd.game.prompts import SyntheticPromptGenerator, image_prompt, load_seeds, load_styles
    from cassmantle_amd.parallel.supervisor import GroupSupervisor
    from cassmantle_amd.pipeline import SPECS
    from cassmantle_amd.scoring.batcher import BatchingScorer
    from cassmantle_amd.scoring.encoder import EncoderBackend

    gpu = torch.cuda.device_count() > 0          # (does not initialise the GPU on this image)
    n = a.gpus
    devices = ([f"cuda:{i}" + (f"#{k}" if k else "") for i in range(n) for k in range(a.slots_per_gpu)] if gpu
               else [f"cpu:{i}" for i in range(n * a.slots_per_gpu)])
    n = len(devices)
    spec = SPECS[a.model]
    cfg = Config()
    cfg.model.image_model = a.model
    cfg.model.resolution = spec.resolution
    cfg.model.steps = spec.steps
    cfg.model.scheduler = spec.scheduler
    cfg.model.guidance_scale = spec.guidance
    cfg.model.device = "cuda" if gpu else "cpu"
    rooms = [""] + [str(i) for i in range(1, n)]
    t_start = time.perf_counter()
    w0 = cfg.game.frontend_device_weight if a.weight0 is None else a.weight0
    sup = GroupSupervisor(cfg, devices, rooms, window_s=0.05, start_timeout_s=1200, dispatch=a.dispatch,
                          weights={devices[0]: w0}, transport=a.transport,
                          frontend_device="cuda:0" if gpu else None, land=a.land)
    if not sup.wait_ready(1500) or not sup.live_devices():
        raise SystemExit(f"worker group did not start: {sup.status()}")
    print(f"[live] worker group up on {sup.live_devices()} in {time.perf_counter() - t_start:.1f} s",
          file=sys.stderr, flush=True)
    dev = torch.device("cuda:0" if gpu else "cpu")
    prio = 0 if a.no_priority else (0 if a.priority is None else a.priority)
    backend = EncoderBackend(device=str(dev), stream_priority=prio)
    scorer = BatchingScorer(backend, 0.01, window_ms=a.window_ms)
    gen = SyntheticPromptGenerator(salt=0)
    seeds_txt, styles = load_seeds(), load_styles()

    def prompts(step, r):
        return [image_prompt(styles[(step + j) % len(styles)],
                             gen.generate(seeds_txt[(r + step + j) % len(seeds_txt)] + "\n", True),
                             "A {style} style piece depicting the following: ") for j in range(a.batch)]

    def one_round(step) -> int:
        futs = [sup.submit(room, prompts(step, i), [i * 10000 + step * 10 + j for j in range(a.batch)])
                for i, room in enumerate(rooms)]
        return sum(len(f.result(timeout=1800)) for f in futs)

    one_round(0)                                   # warm: graph capture on every worker
    print("[live] warm round done", file=sys.stderr, flush=True)
    asyncio.run(run_players(scorer, min(a.players, 4), 1.0, a.think_ms, 99))
    idle = asyncio.run(run_players(scorer, a.players, a.idle_s, a.think_ms, 0))
    print(f"[live] idle phase done: {len(idle)} requests", file=sys.stderr, flush=True)
    done = {"images": 0, "rounds": 0}
    stop = threading.Event()
    mu = threading.Lock()

    def room_loop(i, room):
        # every room runs its own rounds (as the game's rooms do: each buffers its next content on
        # its own timer), so a room on a fast GPU is never held by a room on a slow one
        step = 1
        while not stop.is_set():
            f = sup.submit(room, prompts(step, i), [i * 10000 + step * 10 + j for j in range(a.batch)])
            k = len(f.result(timeout=1800))
            with mu:
                done["images"] += k
                done["rounds"] += 1
                if i == 0:
                    print(f"[live] {done['images']} images", file=sys.stderr, flush=True)
            step += 1

    ths = [threading.Thread(target=room_loop, args=(i, room), daemon=True) for i, room in enumerate(rooms)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    load = asyncio.run(run_players(scorer, a.players, a.seconds, a.think_ms, 7))
    with mu:
        imgs_at_stop = done["images"]
    elapsed = time.perf_counter() - t0
    stop.set()
    for th in ths:
        th.join()
    st = sup.status()
    sup.close()

    print(json.dumps({
        "metric": "live round: images/s with overlapped streaming guess scoring (BASELINE config 5)",
        "topology": "supervised", "images_per_s": round(imgs_at_stop / elapsed, 3), "n_gpus": a.gpus, "workers": n,
        "devices": st["live_devices"], "players": a.players, "think_ms": a.think_ms,
        "idle_p50_ms": round(pct(idle, 50), 3), "idle_p99_ms": round(pct(idle, 99), 3),
        "load_p50_ms": round(pct(load, 50), 3), "load_p99_ms": round(pct(load, 99), 3), "requests": len(load),
        "rounds": done["rounds"], "gather_us_p50": st["gather_us_p50"], "retired": st["retired"],
        "scorer_stream_priority": prio, "seconds": a.seconds, "dispatch": a.dispatch,
        "worker_rounds": st.get("worker_rounds"), "transport": st.get("transport"),
        "land_us_p50": st.get("land_us_p50"),
        "config": {"model": a.model, "batch_per_room": a.batch, "rooms": len(rooms)}}), flush=True)


def main():
    a = parse()
    if a.gpus is not None and "WORLD_SIZE" not in os.environ:
        return main_supervised(a)
    from cassmantle_amd.game.prompts import SyntheticPromptGenerator, image_prompt, load_seeds, load_styles
    from cassmantle_amd.parallel import dist as cdist
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    from cassmantle_amd.scoring.batcher import BatchingScorer
    from cassmantle_amd.scoring.encoder import EncoderBackend

    if a.switch_ms is not None:
        sys.setswitchinterval(a.switch_ms / 1e3)
    ctx = cdist.init_from_env()
    rank, world, dev = ctx.rank, ctx.world_size, ctx.device
    n_players = a.players if rank == 0 else 0          # rank-0-central scoring, as serve.py
    s_score = s_gen = None
    if a.reserve_cus > 0:
        from cassmantle_amd.runtime.cumask import reserved_streams
        s_score, s_gen = reserved_streams(dev, a.reserve_cus, exclusive=a.exclusive_scorer)
    sd = StableDiffusion(SPECS[a.model], device=dev, seed=0, stream=s_gen)
    prio = 0 if a.no_priority else (-1 if a.priority is None else a.priority)
    backend = EncoderBackend(device=str(dev), stream_priority=prio, stream=s_score)
    sharded = follower = None
    if a.score_topology == "sharded" and world > 1:
        from cassmantle_amd.parallel.scoring import ShardedSimilarity, new_scoring_group
        sharded = ShardedSimilarity(ctx, backend, group=new_scoring_group("gloo"), min_pairs=a.shard_min)
        backend = sharded
        if rank != 0:
            follower = sharded.start_serving()
    scorer = BatchingScorer(backend, 0.01, window_ms=a.window_ms)
    gen = SyntheticPromptGenerator(salt=rank)
    seeds_txt, styles = load_seeds(), load_styles()
    neg = "blurry, distorted, fake, abstract, negative"

    def prompts(step):
        return [image_prompt(styles[(step + j) % len(styles)],
                             gen.generate(seeds_txt[(rank + step + j) % len(seeds_txt)] + "\n", True),
                             "A {style} style piece depicting the following: ") for j in range(a.batch)]

    # warm everything (graph capture, allocator, scorer shapes)
    sd.generate_tensor(prompts(0), neg, list(range(a.batch))).cpu()
    print(f"[live] warm generation done", file=sys.stderr, flush=True)
    if n_players:
        asyncio.run(run_players(scorer, min(n_players, 4), 1.0, a.think_ms, rank + 99))
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()

    idle = asyncio.run(run_players(scorer, n_players, a.idle_s, a.think_ms, rank)) if n_players else []
    print(f"[live] idle phase done: {len(idle)} requests", file=sys.stderr, flush=True)

    done = {"images": 0}
    stop = threading.Event()

    def gen_loop():
        step = 1
        while not stop.is_set():
            # numpy result copied on the generation stream: never waits on the legacy stream
            sd.generate(prompts(step), neg, [rank * 10000 + step * 10 + j for j in range(a.batch)])
            done["images"] += a.batch
            step += 1
            print(f"[live] {done['images']} images", file=sys.stderr, flush=True)

    if world > 1:
        torch.distributed.barrier()
    th = threading.Thread(target=gen_loop, daemon=True)
    t0 = time.perf_counter()
    th.start()
    if n_players:
        load = asyncio.run(run_players(scorer, n_players, a.seconds, a.think_ms, rank + 7))
    else:
        load = []
        time.sleep(a.seconds)
    imgs_at_stop = done["images"]
    elapsed = time.perf_counter() - t0
    stop.set()
    th.join()
    if sharded is not None:
        sharded.close()                                # rank 0: STOP to the followers
        if follower is not None:
            follower.join(timeout=60)

    stats = torch.tensor([imgs_at_stop / elapsed, pct(idle, 50), pct(idle, 99), pct(load, 50), pct(load, 99),
                          float(len(load))], dtype=torch.float64, device=dev)
    if world > 1:
        allv = [torch.zeros_like(stats) for _ in range(world)]
        torch.distributed.all_gather(allv, stats)
        m = torch.stack(allv)
        agg = [m[:, 0].sum(), m[0, 1], m[0, 2], m[0, 3], m[0, 4], m[:, 5].sum()]   # latencies: rank 0 scores
        stats = torch.stack(agg)
    if rank == 0:
        s = [float(x) for x in stats.tolist()]
        print(json.dumps({
            "metric": "live round: images/s with overlapped streaming guess scoring (BASELINE config 5)",
            "images_per_s": round(s[0], 3), "n_gpus": world, "players": a.players,
            "think_ms": a.think_ms, "idle_p50_ms": round(s[1], 3), "idle_p99_ms": round(s[2], 3),
            "load_p50_ms": round(s[3], 3), "load_p99_ms": round(s[4], 3), "requests": int(s[5]),
            "scorer_stream_priority": prio, "seconds": a.seconds,
            "score_topology": a.score_topology, "reserved_cus": a.reserve_cus, "exclusive_scorer": a.exclusive_scorer,
            "switch_ms": sys.getswitchinterval() * 1e3,
            "sharded_pairs": sharded.sharded_pairs if sharded is not None else 0,
            "config": {"model": a.model, "batch_per_room": a.batch, "graphs": bool(sd.use_graphs)}}), flush=True)
    cdist.shutdown()


if __name__ == "__main__":
    main()
