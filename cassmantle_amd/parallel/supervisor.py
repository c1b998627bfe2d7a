"""Supervised worker groups: the front-end process owns HTTP + game state and runs the GPU
rank workers as CHILD processes, so a dead or wedged GPU costs one GPU, not the node.

Reference analog: every uvicorn worker runs the round timer and whichever one holds the Redis
lock generates; a crashed holder's lock expires (120 s TTL) and any surviving worker takes over
(``/root/reference/src/backend.py:47,83-87,155-159,206-210``; ``main.py:37-40``).  Here
(SURVEY §7.1 design stance, §5.3):

* the front-end (this module, in the HTTP process) launches one worker process per healthy
  device as a fresh ``spawn`` child (never a re-exec of a process that touched the GPU).  The
  workers form their own ``torch.distributed`` group (RCCL over xGMI on GPUs, gloo on the CPU)
  and run ``parallel.rooms.RankWorker`` generation rounds: C1 broadcast of the job list from
  the group leader (worker rank 0), C2 device-resident gather of the images to the leader, C4
  barrier.  The leader talks to the front-end over one pipe: job lists in, uint8 images out;
* every worker publishes a wall-clock heartbeat and the id of the last round whose LOCAL
  generation it finished into shared memory;
* the front-end's coordinator thread batches the rooms' requests into rounds and, while a
  round runs, watches the group: a worker process that exited, a stale heartbeat, or a round
  past ``round_timeout_s`` (the culprits are the workers that never finished their local part:
  RCCL would block the others forever) fails the round — its rooms keep their content, the
  reference's "round repeats" fallback (``src/backend.py:211-215``) — and the whole group is
  torn down (SIGKILL: a collective with a dead peer cannot be cancelled in-process) and
  respawned on the remaining healthy devices, with the rooms re-sharded over the survivors;
* a device is retired when its worker died or hung; a failure no worker can be blamed for
  restarts the group on the same devices (``max_restarts_without_culprit`` times);
* with every device retired the rooms' rounds repeat (the reference's fallback), or a ``local``
  generator serves them, and the retired devices are re-probed with a fresh group after
  ``reprobe_s`` (doubling per failed probe): a transient fault does not cost the GPUs forever.

The legacy ``torchrun`` layout (front-end inside rank 0, ``serve.py`` under torchrun) is still
supported; there a dead rank can only degrade the node to rank 0's GPU.
"""
from __future__ import annotations

import concurrent.futures as cf
import importlib
import logging
import multiprocessing as pymp
import os
import queue
import signal
import socket
import threading
import time
import traceback
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..game.content import ImageGenerationError, ImageGenerator

log = logging.getLogger("cassmantle")


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@dataclass
class WorkerSpec:
    rank: int
    world: int
    port: int
    device: str                     # "cuda:3" | "cpu"
    backend: str                    # "nccl" (RCCL) | "gloo"
    room_ids: List[str]
    negative: str
    gen_factory: str                # "module:function", called as fn(cfg, device, spec) -> ImageGenerator
    cfg: Any                        # config.Config (picklable dataclass)
    epoch: int
    slot: str = ""                  # the device label the front-end knows this worker by
    heartbeat_s: float = 0.5
    env: Dict[str, str] = field(default_factory=dict)


def default_generator(cfg, device: str, spec: WorkerSpec) -> ImageGenerator:
    from ..runtime.factory import build_image_generator
    return build_image_generator(cfg, device=device)


def _resolve(path: str):
    mod, fn = path.split(":")
    return getattr(importlib.import_module(mod), fn)


def worker_main(spec: WorkerSpec, conn, hb, progress) -> None:
    """Entry point of one worker process (spawned child)."""
    os.environ.update(spec.env)
    logging.basicConfig(level=logging.INFO, format=f"[%(levelname)s] w{spec.rank}e{spec.epoch} %(message)s")
    import datetime

    import torch
    import torch.distributed as dist

    from .dist import DistContext
    from .rooms import STOP, RankWorker, RoomSharding

    stop_hb = threading.Event()

    def beat():
        while not stop_hb.wait(spec.heartbeat_s):
            hb[spec.rank] = time.time()
    hb[spec.rank] = time.time()
    threading.Thread(target=beat, daemon=True).start()
    try:
        dev = torch.device(spec.device)
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        kw = dict(backend=spec.backend, init_method=f"tcp://127.0.0.1:{spec.port}", rank=spec.rank,
                  world_size=spec.world, timeout=datetime.timedelta(seconds=3600))
        if spec.backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
        ctx = DistContext(spec.rank, spec.world, spec.rank, dev, spec.backend)
        gen = _resolve(spec.gen_factory)(spec.cfg, spec.device, spec)

        def done(rid: int) -> None:
            progress[spec.rank] = rid
        worker = RankWorker(ctx, gen, RoomSharding(spec.room_ids, spec.world), spec.negative, on_local_done=done)
        dist.barrier()                                   # every member is up
        if spec.rank != 0:
            worker.serve_forever()
        else:
            conn.send(("ready", os.getpid()))
            while True:
                msg = conn.recv()
                if msg[0] == "stop":
                    worker.run_round(STOP)  # type: ignore[arg-type]
                    break
                _, rid, jobs = msg
                res = worker.run_round(jobs, rid)
                conn.send(("result", rid, res, worker.last_gather_us))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001 - report and die; the front-end restarts the group
        msg = traceback.format_exc()
        log.error("[ERROR] worker %d failed: %s", spec.rank, msg)
        try:
            if conn is not None:
                conn.send(("error", -1, msg))
        except Exception:  # noqa: BLE001
            pass
        os._exit(5)
    finally:
        stop_hb.set()
    os._exit(0)


class _Group:
    """One epoch of the worker group (front-end side handle)."""

    def __init__(self, devices: List[str], epoch: int, sup: "GroupSupervisor") -> None:
        self.devices = list(devices)
        self.epoch = epoch
        ctx = pymp.get_context("spawn")
        W = len(devices)
        self.hb = ctx.Array("d", W, lock=False)
        self.progress = ctx.Array("i", W, lock=False)
        for r in range(W):
            self.progress[r] = -1
        self.conn, child = ctx.Pipe()
        port = free_port()
        self.procs = []
        for r, d in enumerate(devices):
            spec = WorkerSpec(r, W, port, sup.device_name(d), sup.backend, sup.room_ids, sup.negative,
                              sup.gen_factory, sup.cfg, epoch, d, sup.heartbeat_s, dict(sup.worker_env))
            p = ctx.Process(target=worker_main, args=(spec, child if r == 0 else None, self.hb, self.progress),
                            name=f"cassmantle-w{r}e{epoch}", daemon=True)
            p.start()
            self.procs.append(p)
        self.started = time.time()

    @property
    def world(self) -> int:
        return len(self.devices)

    def dead(self) -> List[int]:
        return [r for r, p in enumerate(self.procs) if p.exitcode is not None]

    def stale(self, stale_s: float) -> List[int]:
        now = time.time()
        return [r for r in range(self.world) if self.hb[r] > 0 and now - self.hb[r] > stale_s]

    def kill(self) -> None:
        for p in self.procs:
            if p.exitcode is None:
                try:
                    os.kill(p.pid, signal.SIGKILL)
                except (ProcessLookupError, TypeError):
                    pass
        for p in self.procs:
            p.join(timeout=30)
        try:
            self.conn.close()
        except Exception:  # noqa: BLE001
            pass

    def stop(self, timeout: float = 30.0) -> None:
        try:
            self.conn.send(("stop",))
        except Exception:  # noqa: BLE001
            pass
        t_end = time.time() + timeout
        for p in self.procs:
            p.join(timeout=max(0.1, t_end - time.time()))
        self.kill()


class GroupFailure(Exception):
    def __init__(self, reason: str, culprits: Sequence[int]) -> None:
        super().__init__(reason)
        self.culprits = list(culprits)


class GroupSupervisor:
    """Front-end owner of the worker group.  ``submit(room, prompts, seeds)`` -> Future of the
    room's images; rooms are sharded over the group's live workers (room ``i`` -> worker
    ``i mod W``, ``parallel.rooms.RoomSharding``)."""

    def __init__(self, cfg, devices: Sequence[str], room_ids: Sequence[str], backend: Optional[str] = None,
                 gen_factory: str = "cassmantle_amd.parallel.supervisor:default_generator",
                 window_s: float = 0.3, round_timeout_s: float = 600.0, stale_s: float = 30.0,
                 heartbeat_s: float = 0.5, start_timeout_s: float = 900.0, watch_period_s: float = 0.2,
                 max_restarts_without_culprit: int = 2, local: Optional[ImageGenerator] = None,
                 worker_env: Optional[Dict[str, str]] = None, resolution: Optional[int] = None,
                 reprobe_s: float = 120.0) -> None:
        self.cfg = cfg
        self.all_devices = list(devices)
        self.healthy = list(devices)
        self.retired: Dict[str, str] = {}
        self.room_ids = list(room_ids)
        self.backend = backend or ("nccl" if any(d.startswith("cuda") for d in devices) else "gloo")
        self.gen_factory = gen_factory
        self.negative = cfg.game.negative_prompt
        self.window = window_s
        self.round_timeout = round_timeout_s
        self.stale_s = stale_s
        self.heartbeat_s = heartbeat_s
        self.start_timeout = start_timeout_s
        self.watch_period = watch_period_s
        self.max_blind = max_restarts_without_culprit
        self.local = local
        self.worker_env = worker_env or {}
        self.resolution = resolution or cfg.model.resolution
        self.epoch = 0
        self.group: Optional[_Group] = None
        self.failures: List[Dict[str, Any]] = []
        self.rounds = 0
        self.gather_us: List[float] = []
        self._blind = 0
        self._round_id = 0
        self.reprobe_s = reprobe_s
        self._probe_backoff = reprobe_s
        self._next_probe = float("inf")
        self.probes: List[Dict[str, Any]] = []
        self._q: "queue.Queue" = queue.Queue()
        self._closed = False
        self._ready = threading.Event()
        self._thread = threading.Thread(target=self._loop, name="group-supervisor", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------------ devices / groups
    @staticmethod
    def device_name(d: str) -> str:
        return "cpu" if d.startswith("cpu") else d      # "cpu:1" labels a CPU worker slot (tests)

    def _start_group(self) -> None:
        if not self.healthy:
            self.group = None
            return
        self.epoch += 1
        g = _Group(self.healthy, self.epoch, self)
        self.group = g
        t_end = time.time() + self.start_timeout
        while True:
            if g.conn.poll(self.watch_period):
                msg = g.conn.recv()
                if msg[0] == "ready":
                    log.info("[INFO] worker group epoch %d up on %s", self.epoch, self.healthy)
                    return
                raise self._diagnose(g, 0, f"worker start failed: {msg[-1].strip().splitlines()[-1][:300]}")
            if g.dead():
                raise self._diagnose(g, 0, "worker exited during start")
            if time.time() > t_end:
                raise GroupFailure("worker group start timed out", [])

    def _retire(self, culprits: Sequence[int], reason: str) -> None:
        g = self.group
        devs = [g.devices[r] for r in culprits if g is not None and 0 <= r < g.world]
        for d in devs:
            if d in self.healthy:
                self.healthy.remove(d)
                self.retired[d] = reason
        self.failures.append({"epoch": self.epoch, "reason": reason, "retired": devs, "t": time.time()})
        if devs:
            self._blind = 0
        else:
            self._blind += 1
            if self._blind > self.max_blind:          # nobody to blame, keeps failing: stop using GPUs
                for d in list(self.healthy):
                    self.retired[d] = "repeated group failures"
                self.healthy.clear()
        if not self.healthy and self._next_probe == float("inf"):
            self._next_probe = time.time() + self._probe_backoff
        log.error("[ERROR] worker group epoch %d failed (%s); retired %s; healthy %s", self.epoch, reason, devs,
                  self.healthy)

    def _restart(self, culprits: Sequence[int], reason: str) -> None:
        self._retire(culprits, reason)
        if self.group is not None:
            self.group.kill()
        self.group = None
        while self.healthy and not self._closed:
            try:
                self._start_group()
                return
            except GroupFailure as e:
                self._retire(e.culprits, str(e))
                if self.group is not None:
                    self.group.kill()
                self.group = None

    def _maybe_reprobe(self) -> None:
        """With no live group: once the back-off has passed, put every retired device back and
        try a fresh group on them (a failed probe retires them again and doubles the back-off)."""
        if self.group is not None or not self.retired or self._closed or time.time() < self._next_probe:
            return
        back = [d for d in self.all_devices if d in self.retired]
        log.info("[INFO] re-probing retired devices %s", back)
        t0 = time.time()
        for d in back:
            self.retired.pop(d, None)
        self.healthy = [d for d in self.all_devices if d not in self.retired]
        self._blind = 0
        self._next_probe = float("inf")
        try:
            self._start_group()
        except GroupFailure as e:
            self._restart(e.culprits, str(e))
        ok = self.group is not None
        self.probes.append({"devices": back, "ok": ok, "s": round(time.time() - t0, 3)})
        if ok:
            self._probe_backoff = self.reprobe_s
        else:
            self._probe_backoff = min(2 * self._probe_backoff, 3600.0)
            self._next_probe = time.time() + self._probe_backoff

    # ------------------------------------------------------------------ requests
    def submit(self, room: str, prompts: Sequence[str], seeds: Sequence[int]) -> cf.Future:
        fut: cf.Future = cf.Future()
        if self._closed:
            fut.set_exception(ImageGenerationError("supervisor closed"))
            return fut
        self._q.put((room, list(prompts), list(seeds), fut))
        return fut

    def wait_ready(self, timeout: Optional[float] = None) -> bool:
        return self._ready.wait(timeout)

    def live_devices(self) -> List[str]:
        return list(self.group.devices) if self.group is not None else []

    # exit code of a worker that caught an exception (usually a collective broken by a dead
    # peer) and reported it: collateral, not a culprit
    REPORTED_EXIT = 5

    def _diagnose(self, g: "_Group", rid: int, reason: str, grace_s: float = 3.0) -> "GroupFailure":
        """Who broke the round.  A worker that died WITHOUT reporting (crash, OOM kill, signal)
        or stopped heart-beating is a culprit; peers whose collectives then failed exit with
        REPORTED_EXIT and are not.  With nobody dead, the workers that never finished their
        local generation of round ``rid`` are (a wedged GPU: RCCL would block the rest)."""
        t_end = time.time() + grace_s
        while True:
            crashed = [r for r in g.dead() if g.procs[r].exitcode not in (0, self.REPORTED_EXIT)]
            stale = g.stale(self.stale_s)
            if crashed or stale or time.time() > t_end:
                break
            time.sleep(0.05)
        culprits = sorted(set(crashed) | set(stale))
        if not culprits and rid > 0:
            culprits = [r for r in range(g.world) if g.progress[r] < rid and g.procs[r].exitcode is None]
            if len(culprits) == g.world:         # nobody finished: no evidence against anyone
                culprits = []
        codes = {r: g.procs[r].exitcode for r in range(g.world)}
        return GroupFailure(f"{reason}; exit codes {codes}", culprits)

    def _run_round(self, jobs) -> Dict[Tuple[str, int], np.ndarray]:
        g = self.group
        self._round_id += 1
        rid = self._round_id
        g.conn.send(("round", rid, jobs))
        t0 = time.monotonic()
        while True:
            if g.conn.poll(self.watch_period):
                msg = g.conn.recv()
                if msg[0] == "result" and msg[1] == rid:
                    if msg[3] is not None:
                        self.gather_us.append(float(msg[3]))
                    return msg[2]
                if msg[0] == "error":
                    raise self._diagnose(g, rid, f"leader failed: {msg[-1].strip().splitlines()[-1][:300]}")
                continue
            if g.dead():
                raise self._diagnose(g, rid, "worker exited")
            if g.stale(self.stale_s):
                raise self._diagnose(g, rid, "worker stopped heart-beating", grace_s=0.0)
            if self.round_timeout > 0 and time.monotonic() - t0 > self.round_timeout:
                raise self._diagnose(g, rid, f"round {rid} exceeded {self.round_timeout:.0f} s", grace_s=0.0)

    def _loop(self) -> None:
        from .rooms import GenJob
        try:
            self._start_group()
        except GroupFailure as e:
            self._restart(e.culprits, str(e))
        self._ready.set()
        while True:
            item = self._q.get()
            if item is None:
                break
            batch = [item]
            t_end = time.monotonic() + self.window
            every_room = set(self.room_ids)
            while True:
                # a room submits one request per round: once every room is in, the window closes
                if every_room and {b[0] for b in batch} >= every_room:
                    break
                rem = t_end - time.monotonic()
                if rem <= 0:
                    break
                try:
                    nxt = self._q.get(timeout=rem)
                except queue.Empty:
                    break
                if nxt is None:
                    self._q.put(None)
                    break
                batch.append(nxt)
            if self.group is None:
                self._maybe_reprobe()
            if self.group is None:
                self._serve_without_group(batch)
                continue
            jobs, spans = [], []
            for room, prompts, seeds, fut in batch:
                s = len(jobs)
                jobs.extend(GenJob(room, p, sd) for p, sd in zip(prompts, seeds))
                spans.append((s, len(jobs), room, fut))
            try:
                res = self._run_round(jobs)
                self.rounds += 1
                for s, e, room, fut in spans:
                    imgs = [res.get((room, i)) for i in range(s, e)]
                    if any(im is None for im in imgs):
                        fut.set_exception(ImageGenerationError(f"room {room}: generation failed"))
                    else:
                        fut.set_result(imgs)
            except (GroupFailure, EOFError, OSError, BrokenPipeError) as e:
                if not isinstance(e, GroupFailure):       # the leader's pipe broke
                    e = self._diagnose(self.group, self._round_id, f"leader pipe: {type(e).__name__}")
                culprits = e.culprits
                for *_, fut in spans:
                    if not fut.done():
                        fut.set_exception(ImageGenerationError(f"generation round failed: {e}"))
                self._restart(culprits, str(e))
            except Exception as e:  # noqa: BLE001 - unexpected (message shape, pickling): never kill this thread
                log.exception("[ERROR] supervisor round failed unexpectedly")
                for *_, fut in spans:
                    if not fut.done():
                        fut.set_exception(ImageGenerationError(f"generation round failed: {type(e).__name__}: {e}"))
                self._restart([], f"unexpected {type(e).__name__}: {e}")
        if self.group is not None:
            self.group.stop()
            self.group = None

    def _serve_without_group(self, batch) -> None:
        """No live group: a ``local`` generator serves the batch, otherwise each room's round
        repeats (its request fails fast; the room keeps its content, src/backend.py:211-215)."""
        for room, prompts, seeds, fut in batch:
            if self.local is None:
                fut.set_exception(ImageGenerationError("no healthy generation device left: the round repeats"))
                continue
            try:
                fut.set_result(self.local.generate(prompts, self.negative, seeds))
            except Exception as e:  # noqa: BLE001
                fut.set_exception(e)

    def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        self._q.put(None)
        self._thread.join(timeout=120)
        if self.group is not None:
            self.group.kill()
            self.group = None

    def status(self) -> Dict[str, Any]:
        return {"epoch": self.epoch, "live_devices": self.live_devices(), "retired": dict(self.retired),
                "rounds": self.rounds, "failures": list(self.failures), "probes": list(self.probes),
                "gather_us_p50": float(np.median(self.gather_us)) if self.gather_us else None}


class SupervisedImageGenerator(ImageGenerator):
    """Game-layer generator for one room, served by the supervised worker group."""

    def __init__(self, sup: GroupSupervisor, room: str, timeout_s: float = 1800.0) -> None:
        self.sup = sup
        self.room = room
        self.resolution = sup.resolution
        self.timeout = timeout_s

    def generate(self, prompts, negative_prompt, seeds):
        return self.sup.submit(self.room, prompts, seeds).result(timeout=self.timeout)
