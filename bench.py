#!/usr/bin/env python
"""Headline benchmark: SD-1.5 512² 50-step images/sec (whole node) + p50 guess-score latency.

BASELINE.json config 3: concurrent rooms data-parallel over the node's GPUs, one process per
GPU, SD-1.5 512×512, 50 PNDM steps (51 UNet evaluations, SD-1.5's default scheduler),
classifier-free guidance 7.5 (UNet batch 2×4), batch = 4 images per room, bf16, random-init
weights, synthetic ``seeds.txt`` story prompts.  One benchmark *step* = every rank generates
its room's 4 images end to end (CLIP encode → hipGraph-replayed denoise loop → VAE decode →
uint8) and the images are GATHERED to rank 0 over RCCL (C2: what the front-end needs at a round
boundary; device-resident, on a dedicated comm stream fenced by the decode event, no host hop).
Whole-job images/s = N·4·K / max-over-ranks(time of K steps); ``per_rank`` reports each rank's
step time and device time of its gather (µs).

Rank 0 also measures the streaming guess scorer (BASELINE config 1/5): MiniLM-L6 embed +
cosine for a 64-player micro-batch, p50 latency in ms (reported as ``p50_score_ms``).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 4] [--baseline]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_IMAGES_PER_SEC = None  # BASELINE.json "published": {} — no reference number
METRICS = {"sd15": "SD-1.5 512^2 50-step images/sec (whole node) + p50 guess-score latency",
           "sdxl": "SDXL-base 1024^2 30-step images/sec (BASELINE config 4)"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--batch", type=int, default=4, help="images per room (per GPU)")
    p.add_argument("--model", default="sd15")
    p.add_argument("--denoise-steps", type=int, default=None, help="default: the model spec's (sd15: 50)")
    p.add_argument("--scheduler", default=None, help="default: the model spec's (sd15: pndm)")
    p.add_argument("--baseline", action="store_true", help="stock PyTorch ops, no graphs (eager baseline)")
    p.add_argument("--no-graphs", action="store_true")
    p.add_argument("--no-score", action="store_true")
    p.add_argument("--fp8-attention", action="store_true")
    p.add_argument("--overlap", action="store_true", help="VAE decode on a side stream, overlapped with the next step's denoise")
    p.add_argument("--no-batch1", action="store_true", help="skip the batch-1 latency (s/image one room waits)")
    p.add_argument("--profile-steps", type=int, default=0)
    p.add_argument("--oversubscribe", action="store_true",
                   help="allow --gpus N above the visible GPU count: the N ranks share the GPUs "
                        "(rank r on GPU r mod visible) over gloo with a host gather; RCCL refuses "
                        "two ranks on one device, so nccl is refused here")
    return p.parse_args()


def scorer_bench(device) -> dict:
    """BASELINE config 1 / 5 scorer latency: every timed micro-batch holds DISTINCT guesses drawn
    from the 49k-word list (no dedup shortcut), against the round's 2 secret words; p50/p99 at
    batch 1 / 64 / 256 on the GPU (graph-replayed MiniLM), plus the two CPU baselines: the same
    MiniLM on the CPU for one pair, and the reference-equivalent numpy cosine of 300-d word
    vectors one pair at a time (``src/backend.py:303-317``)."""
    import random
    import numpy as np
    import torch
    from cassmantle_amd.scoring.wordvec import load_vocab
    from cassmantle_amd.game.scoring import score_pairs
    from cassmantle_amd.scoring.encoder import EncoderBackend
    words = [w for w in load_vocab() if w.isalpha()]
    rng = random.Random(0)
    secrets = ["lantern", "tower"]
    be = EncoderBackend(device=str(device), stream_priority=-1)

    def run(batch, iters):
        lat = []
        for it in range(iters + 3):
            guesses = rng.sample(words, batch)
            pairs = [(g, secrets[i % 2]) for i, g in enumerate(guesses)]
            t1 = time.perf_counter()
            score_pairs(be, pairs, 0.01)
            if it >= 3:
                lat.append((time.perf_counter() - t1) * 1e3)
        return float(np.percentile(lat, 50)), float(np.percentile(lat, 99))
    out = {}
    for b in (1, 64, 256):
        p50, p99 = run(b, 50)
        out[f"b{b}"] = {"p50_ms": round(p50, 3), "p99_ms": round(p99, 3)}
    # the reference-equivalent word-vector scorer (K14 gather + normalise + cosine on the GPU,
    # ops.gather_cosine; reference: wv.similarity per pair, src/backend.py:303-317), 300-d table
    # over the 49k-word list (random-init vectors, as BASELINE specifies)
    from cassmantle_amd.scoring.wordvec import WordVectorBackend
    be_wv = WordVectorBackend(device=str(device), dtype=torch.bfloat16)
    wv = {}
    for b in (1, 64, 256):
        lat = []
        for it in range(53):
            guesses = rng.sample(words, b)
            pairs = [(g, secrets[i % 2]) for i, g in enumerate(guesses)]
            t1 = time.perf_counter()
            score_pairs(be_wv, pairs, 0.01)
            if it >= 3:
                lat.append((time.perf_counter() - t1) * 1e3)
        wv[f"b{b}"] = {"p50_ms": round(float(np.percentile(lat, 50)), 3), "p99_ms": round(float(np.percentile(lat, 99)), 3)}
    # CPU baselines (config 1)
    cpu = EncoderBackend(device="cpu")
    lat = []
    for _ in range(20):
        g = rng.choice(words)
        t1 = time.perf_counter()
        score_pairs(cpu, [(g, "lantern")], 0.01)
        lat.append((time.perf_counter() - t1) * 1e3)
    vec = {w: np.random.default_rng(hash(w) & 0xffff).standard_normal(300).astype(np.float32) for w in words[:2000]}
    keys = list(vec)
    lat_np = []
    for i in range(2000):
        a, b = vec[keys[i % 2000]], vec[keys[(i * 7 + 1) % 2000]]
        t1 = time.perf_counter()
        float(np.dot(a, b) / (np.linalg.norm(a) * np.linalg.norm(b)))
        lat_np.append((time.perf_counter() - t1) * 1e3)
    return {"p50_score_ms": out["b64"]["p50_ms"], "p99_score_ms": out["b64"]["p99_ms"], "score_batch": 64,
            "score_latency": out, "score_latency_wordvec": wv, "cpu_minilm_1pair_p50_ms": round(float(np.percentile(lat, 50)), 3),
            "cpu_numpy_cosine_1pair_p50_ms": round(float(np.percentile(lat_np, 50)), 5)}


def _visible_gpus() -> int:
    """Device count WITHOUT initialising the GPU (on this ROCm image ``device_count`` does not
    create a HIP context, so the launcher may still start fresh rank processes afterwards)."""
    import torch
    return torch.cuda.device_count()


def launch_ranks(args) -> int:
    """``bench.py --gpus N`` with no torchrun environment: start N fresh rank processes (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set; RCCL on GPUs, gloo on the CPU) before
    this process makes any GPU call, relay rank 0's JSON line and fail if any rank fails.
    Every rank's stdout/stderr is inherited; only rank 0 prints the result line."""
    import signal
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if args.oversubscribe:
            env["CASSMANTLE_DIST_BACKEND"] = "gloo"
        # host threads per rank (torchrun's default is 1): N ranks must not each spin up a
        # thread per core of the machine
        env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // args.gpus)))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    print(f"[bench] rank {procs.index(p)} exited with {code}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in live:           # peers would block in a collective forever
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def main() -> int:
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) != args.gpus:
        print(f"[bench] WORLD_SIZE={env_world} disagrees with --gpus {args.gpus}", file=sys.stderr)
        return 2
    if args.oversubscribe:
        if os.environ.get("CASSMANTLE_DIST_BACKEND", "gloo") != "gloo":
            print("[bench] --oversubscribe runs gloo (RCCL refuses two ranks on one GPU); "
                  f"CASSMANTLE_DIST_BACKEND={os.environ['CASSMANTLE_DIST_BACKEND']} refused", file=sys.stderr)
            return 2
        os.environ["CASSMANTLE_DIST_BACKEND"] = "gloo"
    if env_world is None and args.gpus > 1:
        n_vis = _visible_gpus()
        if n_vis and args.gpus > n_vis and not args.oversubscribe:
            print(f"[bench] --gpus {args.gpus} exceeds the {n_vis} visible GPU(s) "
                  "(--oversubscribe shares them over gloo)", file=sys.stderr)
            return 2
        return launch_ranks(args)
    if env_world is None and args.gpus < 1:
        print("[bench] --gpus must be >= 1", file=sys.stderr)
        return 2
    if args.baseline:
        os.environ["CASSMANTLE_OPS"] = "torch"
    import numpy as np
    import torch
    import torch.distributed as dist

    from cassmantle_amd import ops
    from cassmantle_amd.parallel import dist as cdist
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    from cassmantle_amd.game.prompts import SyntheticPromptGenerator, image_prompt, load_seeds, load_styles

    ctx = cdist.init_from_env()
    rank, world = ctx.rank, ctx.world_size
    device = ctx.device
    if args.baseline:
        ops.set_mode("torch")
    torch.manual_seed(0)

    spec = SPECS[args.model]
    args.denoise_steps = args.denoise_steps or spec.steps
    args.scheduler = args.scheduler or spec.scheduler
    sd = StableDiffusion(spec, device=device, use_graphs=not (args.baseline or args.no_graphs),
                         fp8_attention=args.fp8_attention, seed=0, overlap_decode=args.overlap)
    gen = SyntheticPromptGenerator(salt=rank)
    seeds_txt, styles = load_seeds(), load_styles()
    negative = "blurry, distorted, fake, abstract, negative"

    def room_prompts(step: int):
        out = []
        for j in range(args.batch):
            title = seeds_txt[(rank * 7 + step * 3 + j) % len(seeds_txt)]
            text = gen.generate(title + "\nChapter 1\n\n", True)
            out.append(image_prompt(styles[(step + j) % len(styles)], text, "A {style} style piece depicting the following: "))
        return out

    H = spec.resolution
    gather_buf = None
    gather_ms = []
    comm = torch.cuda.Stream(device=device) if device.type == "cuda" else None
    # gloo (the one-GPU multi-rank rehearsal) gathers host tensors; RCCL gathers in HBM
    host_gather = world > 1 and dist.get_backend() == "gloo"

    def one_step(step: int):
        nonlocal gather_buf
        prompts = room_prompts(step)
        seeds = [1000 * rank + 10 * step + j for j in range(args.batch)]
        # sync_caller=False: nothing is enqueued on this thread's stream; the images are ordered
        # on the pipeline's output stream only
        img = sd.generate_tensor(prompts, negative, seeds, steps=args.denoise_steps, scheduler=args.scheduler,
                                 sync_caller=False)
        if world > 1 and comm is None:                      # CPU rehearsal (gloo)
            if gather_buf is None and rank == 0:
                gather_buf = [torch.empty_like(img) for _ in range(world)]
            dist.gather(img, gather_buf if rank == 0 else None, dst=0)
        elif world > 1:
            # C2 on the comm stream, fenced by the decode event: the next step's encode/denoise
            # on the generation stream is not ordered behind the collective
            ev = torch.cuda.Event()
            ev.record(sd.out_stream)
            comm.wait_event(ev)
            with torch.cuda.stream(comm):
                img.record_stream(comm)
                src = img.cpu() if host_gather else img
                if gather_buf is None and rank == 0:
                    gather_buf = [torch.empty_like(src) for _ in range(world)]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(comm)
                dist.gather(src, gather_buf if rank == 0 else None, dst=0)
                e1.record(comm)
            gather_ms.append((e0, e1))
        return img

    for w in range(args.warmup):
        one_step(w)
    torch.cuda.synchronize(device) if device.type == "cuda" else None
    if world > 1:
        dist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    from cassmantle_amd.utils.tracing import TRACER
    TRACER.flush()
    TRACER.reset()                      # stage means over the timed generations only
    t0 = time.perf_counter()
    for k in range(args.steps):
        img = one_step(args.warmup + k)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    mine = elapsed
    # finiteness of the final LATENTS of the last TIMED generation (the uint8 image is finite by
    # construction); read before the batch-1 runs below replace it
    finite = bool(sd.last_finite.item()) if sd.last_finite is not None else None
    TRACER.flush()
    stage_ms = {k: v["mean_ms"] for k, v in TRACER.snapshot().items()
                if k in ("encode", "denoise", "decode")}
    # per-rank scalars: host tensors over gloo (no GPU all_gather there), device tensors over RCCL
    cdev = device if (world == 1 or dist.get_backend() != "gloo") else torch.device("cpu")
    t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    per_rank = None
    if world > 1:
        # per-rank step time and device time of its image gather (C2, RCCL over xGMI), to rank 0
        ag = [a.elapsed_time(b) for a, b in gather_ms[args.warmup:]] or [0.0]   # ms
        mine_t = torch.tensor([mine / args.steps * 1e3, float(np.mean(ag)) * 1e3], dtype=torch.float64, device=cdev)
        allv = [torch.zeros_like(mine_t) for _ in range(world)]
        dist.all_gather(allv, mine_t)
        per_rank = [{"rank": i, "ms_per_step": round(float(v[0]), 2), "gather_us": round(float(v[1]), 1)}
                    for i, v in enumerate(allv)]
    # batch-1 latency: one room's single image end to end (prompt -> uint8 on host), what a
    # serving room waits on; one warm-up generation (graph capture for batch 1), then 2 timed
    b1 = None
    if not args.no_batch1 and device.type == "cuda":
        p1 = room_prompts(10_000)[:1]
        sd.generate(p1, negative, [7], steps=args.denoise_steps, scheduler=args.scheduler)
        lat1 = []
        for i in range(2):
            t1 = time.perf_counter()
            sd.generate(p1, negative, [8 + i], steps=args.denoise_steps, scheduler=args.scheduler)
            lat1.append(time.perf_counter() - t1)
        b1 = round(float(np.median(lat1)), 4)

    score = {}
    if rank == 0 and not args.no_score:
        score = scorer_bench(device)    # noqa: F841 - reported below


    if rank == 0:
        images = world * args.batch * args.steps
        value = images / elapsed
        out = {
            "metric": METRICS.get(args.model, f"{args.model} images/sec"),
            "value": round(value, 4),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (value / BASELINE_IMAGES_PER_SEC) if BASELINE_IMAGES_PER_SEC else None,
            "dtype": "bf16",
            "data": "synthetic (seeds.txt template prompts, random-init weights)",
            "config": {"model": f"{args.model} UNet/VAE/CLIP ({spec.resolution}x{spec.resolution}, "
                                f"{args.denoise_steps} steps {args.scheduler}, cfg {spec.guidance})"
                                + (", fp8 attention" if args.fp8_attention else ""),
                       "global_batch": world * args.batch, "seq_len": (spec.resolution // 8) ** 2,
                       "parallelism": f"dp{world} (rooms)"},
            "ops": ("torch-eager" if args.baseline else "hip") if device.type == "cuda" else "cpu-reference",
            "graphs": bool(sd.use_graphs),
            "finite": finite,
            "s_per_image_per_gpu": round(elapsed / (args.steps * args.batch), 4),
            "batch1_s_per_image": b1,       # one room, one image, prompt -> host uint8
            "stage_overlap": sd.decode_stream is not None,
            "stage_mean_ms": stage_ms,      # device time per timed generation
            **score,
        }
        if per_rank is not None:
            out["per_rank"] = per_rank
            out["comm"] = {"backend": dist.get_backend(), "world_size": world,
                           "oversubscribed": bool(args.oversubscribe)}
        print(json.dumps(out), flush=True)
    cdist.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
