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

After the headline timed region (its fields unchanged), a 1-GPU run also records BASELINE
configs 4 and 5 (skippable): ``sdxl_fp8_s_per_image`` (SDXL-base 1024², 30 Euler steps, batch 1,
fp8 attention; one warm-up + 2 timed generations, prompt -> host uint8, with its own ``finite``)
and a short in-process live round (``live_images_per_s``, ``live_score_p50_ms`` /
``live_score_p99_ms``: 64 simulated players scoring while the same pipeline draws 4-image rooms
back to back, ``runtime/live.py``).

Failure handling (a first multi-GPU run must end with a diagnosable record, not a silent hang):
the launcher counts GPUs without touching HIP (visibility variables, KFD sysfs topology); the
process-group init and every blocking collective of a rank are bounded by ``--comm-timeout-s``
(a watchdog thread ends the rank with an error record); the launcher has an overall
``--deadline-s``.  On a failure ONE JSON line is printed (by the launcher, or by rank 0 under
torchrun) with ``value`` null, ``error`` and, for a collective / init failure, ``comm.error``.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 4] [--baseline]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import threading
import time
import traceback

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
    p.add_argument("--no-sdxl", action="store_true", help="skip the SDXL fp8 extra (BASELINE config 4)")
    p.add_argument("--no-live", action="store_true", help="skip the in-process live-round extra (config 5)")
    p.add_argument("--live-seconds", type=float, default=12.0)
    p.add_argument("--live-players", type=int, default=64)
    p.add_argument("--comm-timeout-s", type=float, default=180.0,
                   help="bound on the process-group init and on every blocking collective of a rank")
    p.add_argument("--deadline-s", type=float, default=1500.0, help="launcher: overall deadline of the job")
    p.add_argument("--oversubscribe", action="store_true",
                   help="allow --gpus N above the visible GPU count: the N ranks share the GPUs "
                        "(rank r on GPU r mod visible) over gloo with a host gather; RCCL refuses "
                        "two ranks on one device, so nccl is refused here")
    return p.parse_args()


_ENCODERS: dict = {}


def shared_encoder(device):
    """ONE graph-replayed MiniLM backend (and so one high-priority scorer stream) per process for
    the scorer measurements and the live round: every further stream of a process shares the
    GPU's hardware queues with the generation stream (supervisor.py, profiles/r6_live_ipc_stream_ab.txt)."""
    from cassmantle_amd.scoring.encoder import EncoderBackend
    key = str(device)
    if key not in _ENCODERS:
        _ENCODERS[key] = EncoderBackend(device=key, stream_priority=-1)
    return _ENCODERS[key]


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
    be = shared_encoder(device)

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
    """GPU count WITHOUT any HIP call (the launcher starts fresh rank processes afterwards and
    must never initialise the GPU itself; ``torch.cuda.device_count`` may fall back to a HIP
    runtime init when amdsmi is unavailable).  A visibility variable wins; otherwise the GPU
    nodes of the KFD topology (``simd_count`` > 0; CPU nodes report 0) are counted."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() not in ("", "-1")])
    n = 0
    for prop in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(prop) as f:
                kv = dict(line.split(None, 1) for line in f if len(line.split(None, 1)) == 2)
            n += int(kv.get("simd_count", "0")) > 0
        except (OSError, ValueError):
            continue
    return n


def _config_of(args, world: int) -> dict:
    return {"model": args.model, "global_batch": world * args.batch, "parallelism": f"dp{world} (rooms)"}


def error_record(args, world: int, error: str, comm_error: str = None, backend: str = None) -> dict:
    """The one JSON line of a failed job: the headline keys with ``value`` null."""
    out = {"metric": METRICS.get(args.model, f"{args.model} images/sec"), "value": None, "unit": "images/s",
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": None,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
           "data": "synthetic (seeds.txt template prompts, random-init weights)",
           "config": _config_of(args, world), "error": error}
    if comm_error is not None:
        out["comm"] = {"backend": backend, "world_size": world, "error": comm_error}
    return out


class RankFailure(Exception):
    def __init__(self, kind: str, msg: str) -> None:
        super().__init__(msg)
        self.kind = kind                    # "comm-init" | "comm" | "rank"


def report_failure(args, rank: int, world: int, kind: str, msg: str, backend: str = None) -> None:
    """Launched by our launcher: a per-rank record for it to relay.  Under torchrun: rank 0
    prints the job's one JSON line itself."""
    rec = {"rank": rank, "kind": kind, "error": msg[-2000:], "backend": backend}
    errdir = os.environ.get("CASSMANTLE_BENCH_ERRDIR")
    if errdir:
        try:
            with open(os.path.join(errdir, f"rank{rank}.json"), "w") as f:
                json.dump(rec, f)
        except OSError:
            pass
    elif rank == 0:
        comm = msg if kind.startswith("comm") else None
        print(json.dumps(error_record(args, world, f"rank 0 {kind}: {msg[-500:]}", comm, backend)), flush=True)
    print(f"[bench] rank {rank} failed ({kind}): {msg[-2000:]}", file=sys.stderr, flush=True)


class Watchdog:
    """Bounds the blocking phases of a rank: ``arm(stage, s)`` before a process-group init or a
    blocking collective / device sync behind collectives, ``disarm()`` after.  A stage still
    armed at its deadline (a dead or wedged peer: RCCL would wait forever) ends THIS process
    with a failure record (``os._exit``: the main thread is stuck inside the runtime)."""

    def __init__(self, args, rank: int, world: int) -> None:
        self.args, self.rank, self.world = args, rank, world
        self.backend = None
        self._stage, self._deadline = None, None
        self._mu = threading.Lock()
        threading.Thread(target=self._run, name="bench-watchdog", daemon=True).start()

    def arm(self, stage: str, seconds: float) -> None:
        with self._mu:
            self._stage, self._deadline = stage, time.monotonic() + seconds

    def disarm(self) -> None:
        with self._mu:
            self._stage, self._deadline = None, None

    def _run(self) -> None:
        while True:
            time.sleep(0.25)
            with self._mu:
                stage, dl = self._stage, self._deadline
            if dl is not None and time.monotonic() > dl:
                kind = "comm-init" if stage == "comm-init" else "comm"
                report_failure(self.args, self.rank, self.world, kind,
                               f"{stage} did not finish within its bound (a peer rank died or hung)", self.backend)
                sys.stdout.flush()
                sys.stderr.flush()
                os._exit(3)


def launch_ranks(args) -> int:
    """``bench.py --gpus N`` with no torchrun environment: start N fresh rank processes (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set; RCCL on GPUs, gloo on the CPU) before
    this process makes any GPU call, relay rank 0's JSON line and fail if any rank fails.
    Every rank's stdout/stderr is inherited; rank 0 prints the result line.  On a failure (a
    rank exits non-zero, or the job passes ``--deadline-s``) the other ranks are stopped within
    seconds and THIS process prints the job's one JSON line with the ranks' failure records."""
    import signal
    import socket
    import subprocess
    import tempfile
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    errdir = tempfile.mkdtemp(prefix="cassmantle-bench-")
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   CASSMANTLE_BENCH_ERRDIR=errdir)
        if args.oversubscribe:
            env["CASSMANTLE_DIST_BACKEND"] = "gloo"
        # host threads per rank (torchrun's default is 1): N ranks must not each spin up a
        # thread per core of the machine
        env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // args.gpus)))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    why = None
    t_end = time.monotonic() + args.deadline_s
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
                    why = f"rank {procs.index(p)} exited with {code}"
                    print(f"[bench] {why}; stopping the other ranks", file=sys.stderr, flush=True)
                    for q in live:           # peers would block in a collective forever
                        q.send_signal(signal.SIGTERM)
                    t_end = min(t_end, time.monotonic() + 10.0)
            if live and time.monotonic() > t_end:
                if rc == 0:
                    rc = 124
                    why = f"job exceeded the launcher deadline of {args.deadline_s:.0f} s"
                    print(f"[bench] {why}; killing the ranks", file=sys.stderr, flush=True)
                for q in live:
                    q.kill()
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    if rc != 0:
        recs = []
        for f in sorted(glob.glob(os.path.join(errdir, "rank*.json"))):
            try:
                with open(f) as fh:
                    recs.append(json.load(fh))
            except (OSError, ValueError):
                pass
        comm = [r for r in recs if str(r.get("kind", "")).startswith("comm")]
        backend = next((r.get("backend") for r in recs if r.get("backend")), None)
        detail = "; ".join(f"rank {r['rank']} {r['kind']}: {r['error'][-300:]}" for r in recs)
        out = error_record(args, args.gpus, why + (f" ({detail})" if detail else ""),
                           "; ".join(f"rank {r['rank']}: {r['error'][-300:]}" for r in comm) if comm
                           else (why if rc == 124 else None), backend)
        print(json.dumps(out), flush=True)
    for f in glob.glob(os.path.join(errdir, "*")):
        os.remove(f)
    os.rmdir(errdir)
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
    if (os.environ.get("CASSMANTLE_DIAG_TWICE", "0") == "1"
            and os.environ.get("CASSMANTLE_DIAG_TWICE_ACK") != "wrong-results"):
        # (tools/diag_twice.py traces set the acknowledgement; a record of such a run is invalid)
        print("[bench] CASSMANTLE_DIAG_TWICE=1 (a timing diagnostic with WRONG results) refused", file=sys.stderr)
        return 2
    if args.baseline:
        os.environ["CASSMANTLE_OPS"] = "torch"
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    wd = Watchdog(args, rank, world)
    try:
        return run_rank(args, wd)
    except RankFailure as e:
        report_failure(args, rank, world, e.kind, str(e), wd.backend)
    except BaseException as e:  # noqa: BLE001 - one record, then a non-zero exit
        report_failure(args, rank, world, "rank", "".join(traceback.format_exception(type(e), e, e.__traceback__)),
                       wd.backend)
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(3)          # no collective teardown: a peer may be gone


def run_rank(args, wd: "Watchdog") -> int:
    import numpy as np
    import torch
    import torch.distributed as dist

    from cassmantle_amd import ops
    from cassmantle_amd.parallel import dist as cdist
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    from cassmantle_amd.game.prompts import SyntheticPromptGenerator, image_prompt, load_seeds, load_styles

    wd.backend = os.environ.get("CASSMANTLE_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    wd.arm("comm-init", args.comm_timeout_s)
    try:
        ctx = cdist.init_from_env(timeout_s=args.comm_timeout_s)
    except Exception as e:  # noqa: BLE001
        raise RankFailure("comm-init", f"{type(e).__name__}: {e}") from e
    wd.disarm()
    rank, world = ctx.rank, ctx.world_size
    device = ctx.device
    if world > 1:
        wd.backend = dist.get_backend()
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
    # the C2 gather's stream exists only when there is a gather (a 1-GPU run creates no stream
    # beyond the pipeline's)
    comm = torch.cuda.Stream(device=device) if device.type == "cuda" and world > 1 else None
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

    # the warm-up (graph capture) and timed steps enqueue C2 gathers that wait for the peers:
    # every host wait behind them is bounded (a dead peer would block RCCL forever)
    wd.arm("warm-up steps + barrier", args.comm_timeout_s + 120.0 * max(1, args.warmup))
    for w in range(args.warmup):
        one_step(w)
    torch.cuda.synchronize(device) if device.type == "cuda" else None
    if world > 1:
        dist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    wd.arm("timed steps + barrier", args.comm_timeout_s + 60.0 * args.steps)
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
    wd.arm("timing collectives", args.comm_timeout_s)
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
    wd.disarm()
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

    # BASELINE configs 5 and 4 as extras of a 1-GPU record, after every headline measurement
    extras = {}
    use_graphs, overlap = bool(sd.use_graphs), sd.decode_stream is not None
    if world == 1 and device.type == "cuda" and args.model == "sd15" and not args.baseline:
        if not args.no_live:
            extras.update(live_extra(args, sd, device, room_prompts, negative))
        if not args.no_sdxl:
            del sd
            torch.cuda.empty_cache()
            extras.update(sdxl_extra(device, negative))


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
            "graphs": use_graphs,
            "finite": finite,
            "s_per_image_per_gpu": round(elapsed / (args.steps * args.batch), 4),
            "batch1_s_per_image": b1,       # one room, one image, prompt -> host uint8
            "stage_overlap": overlap,
            "stage_mean_ms": stage_ms,      # device time per timed generation
            **score,
            **extras,
        }
        if per_rank is not None:
            out["per_rank"] = per_rank
            out["comm"] = {"backend": dist.get_backend(), "world_size": world,
                           "oversubscribed": bool(args.oversubscribe)}
        print(json.dumps(out), flush=True)
    wd.arm("shutdown barrier", args.comm_timeout_s + 300.0)
    cdist.shutdown()
    wd.disarm()
    return 0


def live_extra(args, sd, device, room_prompts, negative) -> dict:
    """BASELINE config 5 (in-process, this GPU): ``--live-players`` players stream guesses through
    the micro-batching scorer (graph-replayed MiniLM on a high-priority stream) while the
    headline pipeline draws 4-image rooms back to back (prompt -> host uint8)."""
    from cassmantle_amd.runtime.live import live_round_inprocess
    from cassmantle_amd.scoring.batcher import BatchingScorer
    from cassmantle_amd.scoring.encoder import EncoderBackend
    scorer = BatchingScorer(shared_encoder(device), 0.01, window_ms=1.0)

    def gen(step: int) -> int:
        imgs = sd.generate(room_prompts(20_000 + step), negative,
                           [500_000 + 10 * step + j for j in range(args.batch)],
                           steps=args.denoise_steps, scheduler=args.scheduler)
        return len(imgs)
    # an idle scoring phase first (as tools/bench_live.py): every micro-batch shape the players
    # produce is graph-captured before generation runs (a capture under load was the p99)
    r = live_round_inprocess(gen, scorer, players=args.live_players, seconds=args.live_seconds, seed=3, idle_s=3.0)
    return {"live_images_per_s": r["images_per_s"], "live_score_p50_ms": r["load_p50_ms"],
            "live_score_p99_ms": r["load_p99_ms"],
            "live": {"players": r["players"], "requests": r["requests"], "seconds": r["seconds"],
                     "generations": r["generations"], "batch_per_room": args.batch, "topology": "in-process",
                     "idle_p50_ms": r.get("idle_p50_ms"), "idle_p99_ms": r.get("idle_p99_ms")}}


def sdxl_extra(device, negative) -> dict:
    """BASELINE config 4: SDXL-base 1024², 30 Euler steps, batch 1, fp8 (OCP e4m3) UNet
    attention on this GPU; one warm-up generation (graph capture), then 2 timed, each prompt ->
    host uint8 (the median is reported), with the finiteness of the timed latents."""
    import numpy as np
    from cassmantle_amd.game.prompts import SyntheticPromptGenerator, image_prompt, load_seeds, load_styles
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    spec = SPECS["sdxl"]
    t_build = time.perf_counter()
    xl = StableDiffusion(spec, device=device, fp8_attention=True, seed=0)
    gen = SyntheticPromptGenerator(salt=11)
    seeds_txt, styles = load_seeds(), load_styles()

    def prompt(i):
        text = gen.generate(seeds_txt[i % len(seeds_txt)] + "\nChapter 1\n\n", True)
        return [image_prompt(styles[i % len(styles)], text, "A {style} style piece depicting the following: ")]
    xl.generate(prompt(0), negative, [1])
    warm_s = time.perf_counter() - t_build
    lat, finite = [], True
    for i in range(2):
        t1 = time.perf_counter()
        try:
            xl.generate(prompt(1 + i), negative, [2 + i])
        except Exception as e:  # noqa: BLE001 - non-finite latents raise ImageGenerationError
            if "non-finite" not in str(e):
                raise
            finite = False
        lat.append(time.perf_counter() - t1)
    return {"sdxl_fp8_s_per_image": round(float(np.median(lat)), 4),
            "sdxl": {"resolution": spec.resolution, "steps": spec.steps, "scheduler": spec.scheduler,
                     "guidance": spec.guidance, "batch": 1, "attention": "fp8 (e4m3, block-scaled MFMA)",
                     "timed": len(lat), "s_per_image_each": [round(x, 4) for x in lat], "finite": finite,
                     "build_and_warmup_s": round(warm_s, 1)}}


if __name__ == "__main__":
    sys.exit(main())
