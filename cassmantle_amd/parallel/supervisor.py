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
  ``reprobe_s`` (doubling per failed probe; reset only after the re-probed group served a round).
  The probe starts the group on a background thread: requests arriving meanwhile fail fast
  (their rooms repeat) instead of waiting for a group start.

Two dispatch modes:

* ``async`` (default): every worker has its own pipe; the front-end batches each worker's rooms
  and hands a worker its next batch as soon as THAT worker is idle.  A slow GPU (GPU 0 shares its
  device with the front-end's guess scorer) no longer holds the other GPUs' rooms at a round
  barrier: a fast worker's rooms complete, and start their next round, first.  Rooms are sharded
  by weight (``weights``: the scorer's device owns fewer rooms).  No collective runs after the
  start handshake, so a dead worker cannot hang a peer inside RCCL.
* ``lockstep``: the generation rounds of ``parallel.rooms.RankWorker`` -- C1 broadcast of the
  job list from the leader, local generation, C2 device-resident RCCL gather to the leader, C4
  barrier (the headline ``bench.py`` runs the same collectives).

Data plane of the async mode (``transport``): ``ipc`` leaves a worker's images in its HBM.
The worker copies each round's uint8 images into an outbox buffer in its own HBM, shared with
the front-end ONCE (a HIP IPC handle, torch's CUDA-tensor reduction over the pipe; re-shared only
when it grows), and the pipe carries just the round id and shape.  The front-end lands the round
with ONE copy of the mapped outbox: by DMA into pinned host memory (the JPEG encode needs host
pixels, ``land="host"``) or onto its own GPU (``land="device"``, default:
over xGMI when the worker sits on another GPU; ``DeviceImage`` handles whose pixels the blur
cache reads in HBM).  The
worker reuses its outbox only for its next round, which is dispatched after the front-end's copy
completed.  ``pipe`` pickles host arrays through the pipe instead.  On the CPU (tests) the
outbox is a shared-memory tensor: the same protocol.

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
    dispatch: str = "async"         # async | lockstep (module docstring)
    weights: Optional[List[float]] = None
    transport: str = "pipe"         # async data plane: ipc | pipe (module docstring)


class DeviceOutbox:
    """Worker end of the ``ipc`` data plane: one uint8 buffer in this worker's memory (HBM, or
    shared memory on the CPU) that every round's images are copied into.  ``put`` returns the
    buffer when it was (re)allocated -- the front-end must be sent the new mapping -- else None."""

    def __init__(self, device) -> None:
        import torch
        self.device = torch.device(device)
        self.buf = None
        # the worker thread's CURRENT stream, not a new one: every extra stream of a process that
        # shares its GPU was measured to cost the co-located work 14 % (profiles/r6_live_ipc_stream_ab.txt)
        self.stream = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None

    def put(self, images):
        import torch
        n = images.numel()
        fresh = None
        if self.buf is None or self.buf.numel() < n:
            cap = max(n, 2 * self.buf.numel()) if self.buf is not None else n
            self.buf = torch.empty(cap, dtype=torch.uint8, device=self.device)
            if self.device.type == "cpu":
                self.buf.share_memory_()
            fresh = self.buf
        if self.stream is not None:
            # the images are complete (their event was waited on); the copy is ordered on this
            # stream and finished before the front-end is told about it
            with torch.cuda.stream(self.stream):
                self.buf[:n].copy_(images.reshape(-1), non_blocking=True)
            self.stream.synchronize()
        else:
            self.buf[:n].copy_(images.reshape(-1))
        return fresh


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
    from .rooms import STOP, RankWorker, RoomSharding, generate_local, generate_local_device

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
        dist.barrier()                                   # every member is up
        if spec.dispatch == "async":
            # the front-end drives this worker alone: no collective after the handshake
            outbox = None
            if spec.transport == "ipc" and hasattr(gen, "generate_device"):
                import torch.multiprocessing  # noqa: F401 - tensor reductions (IPC / shm) for the pipe
                outbox = DeviceOutbox(dev)
            conn.send(("ready", os.getpid()))
            while True:
                msg = conn.recv()
                if msg[0] == "stop":
                    break
                _, rid, jobs = msg
                if outbox is None:
                    imgs = generate_local(gen, jobs, spec.negative)
                    done(rid)                            # device work finished (or failed)
                    conn.send(("result", rid, imgs, None))
                    continue
                dimg = generate_local_device(gen, jobs, spec.negative)
                if dimg is None:
                    done(rid)
                    conn.send(("result", rid, [None] * len(jobs), None))
                    continue
                fresh = outbox.put(dimg)
                done(rid)
                conn.send(("result_dev", rid, {"shape": tuple(dimg.shape), "buf": fresh}, None))
            dist.destroy_process_group()
            stop_hb.set()
            os._exit(0)
        worker = RankWorker(ctx, gen, RoomSharding(spec.room_ids, spec.world, spec.weights), spec.negative,
                            on_local_done=done)
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
    """One epoch of the worker group (front-end side handle).  ``conns[r]`` is the pipe to
    worker ``r`` (``async``: every worker; ``lockstep``: the leader only, ``conns[0]``)."""

    def __init__(self, devices: List[str], epoch: int, sup: "GroupSupervisor") -> None:
        self.devices = list(devices)
        self.epoch = epoch
        ctx = pymp.get_context("spawn")
        W = len(devices)
        self.hb = ctx.Array("d", W, lock=False)
        self.progress = ctx.Array("i", W, lock=False)
        for r in range(W):
            self.progress[r] = -1
        per_worker = sup.dispatch == "async"
        self.conns: List[Any] = []
        children: List[Any] = []
        for r in range(W if per_worker else 1):
            a, b = ctx.Pipe()
            self.conns.append(a)
            children.append(b)
        port = free_port()
        weights = sup.weights_for(devices)
        self.procs = []
        for r, d in enumerate(devices):
            spec = WorkerSpec(r, W, port, sup.device_name(d), sup.backend, sup.room_ids, sup.negative,
                              sup.gen_factory, sup.cfg, epoch, d, sup.heartbeat_s, dict(sup.worker_env),
                              sup.dispatch, weights, sup.transport if per_worker else "pipe")
            child = children[r] if per_worker else (children[0] if r == 0 else None)
            p = ctx.Process(target=worker_main, args=(spec, child, self.hb, self.progress),
                            name=f"cassmantle-w{r}e{epoch}", daemon=True)
            p.start()
            self.procs.append(p)
        for c in children:                   # the children hold their ends: EOF once they exit
            c.close()
        self.started = time.time()

    @property
    def conn(self):
        return self.conns[0]

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
        for c in self.conns:
            try:
                c.close()
            except Exception:  # noqa: BLE001
                pass

    def stop(self, timeout: float = 30.0) -> None:
        for c in self.conns:
            try:
                c.send(("stop",))
            except Exception:  # noqa: BLE001
                pass
        t_end = time.time() + timeout
        for p in self.procs:
            p.join(timeout=max(0.1, t_end - time.time()))
        self.kill()


class GroupFailure(Exception):
    def __init__(self, reason: str, culprits: Sequence[int], group: Optional[_Group] = None) -> None:
        super().__init__(reason)
        self.culprits = list(culprits)
        self.group = group


class GroupSupervisor:
    """Front-end owner of the worker group.  ``submit(room, prompts, seeds)`` -> Future of the
    room's images; rooms are sharded over the group's live workers by weight
    (``parallel.rooms.RoomSharding``; equal weights: room ``i`` -> worker ``i mod W``).

    ``weights`` maps a device label to its share (default 1.0); ``dispatch`` is ``async`` or
    ``lockstep`` (module docstring)."""

    def __init__(self, cfg, devices: Sequence[str], room_ids: Sequence[str], backend: Optional[str] = None,
                 gen_factory: str = "cassmantle_amd.parallel.supervisor:default_generator",
                 window_s: float = 0.3, round_timeout_s: float = 600.0, stale_s: float = 30.0,
                 heartbeat_s: float = 0.5, start_timeout_s: float = 900.0, watch_period_s: float = 0.2,
                 max_restarts_without_culprit: int = 2, local: Optional[ImageGenerator] = None,
                 worker_env: Optional[Dict[str, str]] = None, resolution: Optional[int] = None,
                 reprobe_s: float = 120.0, dispatch: str = "async",
                 weights: Optional[Dict[str, float]] = None, transport: str = "pipe",
                 frontend_device: Optional[str] = None, land: str = "device") -> None:
        if dispatch not in ("async", "lockstep"):
            raise ValueError(f"dispatch must be async or lockstep, not {dispatch!r}")
        if transport not in ("ipc", "pipe"):
            raise ValueError(f"transport must be ipc or pipe, not {transport!r}")
        if land not in ("host", "device"):
            raise ValueError(f"land must be host or device, not {land!r}")
        self.land = land
        # ``ipc``: images land on ``frontend_device`` (the front-end's GPU; None / cpu: host arrays)
        self.transport = transport
        self.frontend_device = frontend_device
        self._inbox: Dict[Tuple[int, int], Any] = {}   # (epoch, worker) -> its outbox, mapped here
        self._land_stream = None
        self.land_us: List[float] = []
        self.cfg = cfg
        self.all_devices = list(devices)
        if len(set(self.all_devices)) != len(self.all_devices):
            raise ValueError(f"duplicate device labels {self.all_devices} (use cuda:0#1 for a second slot)")
        self.healthy = list(devices)
        self.retired: Dict[str, str] = {}
        self.room_ids = list(room_ids)
        self.dispatch = dispatch
        self.weights = dict(weights or {})
        shared = len({self.device_name(d) for d in devices}) < len(devices)
        if backend is None:
            # RCCL refuses two ranks on one device: slots that share a GPU run gloo
            backend = "nccl" if any(d.startswith("cuda") for d in devices) and not shared else "gloo"
        elif backend == "nccl" and shared:
            raise ValueError("nccl (RCCL) cannot run two workers on one GPU; use gloo")
        self.backend = backend
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
        self.sharding = None
        self.failures: List[Dict[str, Any]] = []
        self.rounds = 0
        self.worker_rounds: Dict[str, int] = {}
        self.gather_us: List[float] = []
        self._blind = 0
        self._round_id = 0
        self.reprobe_s = reprobe_s
        self._probe_backoff = reprobe_s
        self._next_probe = float("inf")
        self._probe_thread: Optional[threading.Thread] = None
        self._probe_result: Optional[Tuple] = None
        self._probation = False
        self.probes: List[Dict[str, Any]] = []
        self._q: "queue.Queue" = queue.Queue()
        # async dispatch waits on the worker pipes AND this self-pipe; lockstep only on ``_q``,
        # so the self-pipe exists only in async mode.  Both ends are non-blocking and a write is
        # skipped while a wake-up is already pending: a writer can never block on a full pipe
        # (a blocking pipe that nobody drained hung every submit() after ~13k)
        self._wake_r: Optional[int] = None
        self._wake_w: Optional[int] = None
        if dispatch == "async":
            self._wake_r, self._wake_w = os.pipe()
            os.set_blocking(self._wake_r, False)
            os.set_blocking(self._wake_w, False)
        self._wake_pending = False
        self._wake_lock = threading.Lock()
        self._closed = False
        self._ready = threading.Event()
        self._thread = threading.Thread(target=self._loop, name="group-supervisor", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------------ devices / groups
    @staticmethod
    def device_name(d: str) -> str:
        """Device of a slot label: ``cpu:1`` labels a CPU worker slot (tests); ``cuda:0#1`` is a
        second worker slot on ``cuda:0`` (one-GPU rehearsal of a multi-worker group, gloo)."""
        return "cpu" if d.startswith("cpu") else d.split("#")[0]

    def weights_for(self, devices: Sequence[str]) -> List[float]:
        return [float(self.weights.get(d, self.weights.get(self.device_name(d), 1.0))) for d in devices]

    def _spawn(self, devices: List[str]) -> _Group:
        """Start a group on ``devices`` and wait for every pipe's ``ready``.  Raises GroupFailure
        (carrying the group, so the caller kills it)."""
        self.epoch += 1
        g = _Group(devices, self.epoch, self)
        t_end = time.time() + self.start_timeout
        waiting = set(range(len(g.conns)))
        while waiting:
            for r in list(waiting):
                c = g.conns[r]
                try:
                    if not c.poll(self.watch_period / max(1, len(waiting))):
                        continue
                    msg = c.recv()
                except (EOFError, OSError) as e:        # the worker died before it reported
                    f = self._diagnose(g, 0, f"worker pipe closed during start ({type(e).__name__})")
                    f.group = g
                    raise f
                if msg[0] == "ready":
                    waiting.discard(r)
                    continue
                f = self._diagnose(g, 0, f"worker start failed: {msg[-1].strip().splitlines()[-1][:300]}")
                f.group = g
                raise f
            if not waiting:
                break
            if g.dead():
                f = self._diagnose(g, 0, "worker exited during start")
                f.group = g
                raise f
            if time.time() > t_end:
                raise GroupFailure("worker group start timed out", [], g)
        log.info("[INFO] worker group epoch %d up on %s (%s dispatch)", g.epoch, devices, self.dispatch)
        return g

    def _adopt(self, g: Optional[_Group]) -> None:
        from .rooms import RoomSharding
        self.group = g
        self.sharding = RoomSharding(self.room_ids, g.world, self.weights_for(g.devices)) if g is not None else None

    def _start_group(self) -> None:
        if not self.healthy:
            self._adopt(None)
            return
        try:
            g = self._spawn(list(self.healthy))
        except GroupFailure as e:
            self.group = e.group                    # so _retire can name the culprits' devices
            raise
        self._adopt(g)

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
        if self._probation:                           # a re-probed group failed before serving
            self._probation = False
            self._probe_backoff = min(2 * self._probe_backoff, 3600.0)
        if not self.healthy and self._next_probe == float("inf"):
            self._next_probe = time.time() + self._probe_backoff
        log.error("[ERROR] worker group epoch %d failed (%s); retired %s; healthy %s", self.epoch, reason, devs,
                  self.healthy)

    def _drop_group(self) -> None:
        if self.group is not None:
            self.group.kill()
        self._adopt(None)

    def _restart(self, culprits: Sequence[int], reason: str) -> None:
        """Retire the culprits, kill the group, start a new one on the healthy devices.  Never
        raises: every start failure (a worker that dies without reporting, an unexpected
        message) retires what it can and tries the rest."""
        self._retire(culprits, reason)
        self._drop_group()
        while self.healthy and not self._closed:
            try:
                self._start_group()
                return
            except GroupFailure as e:
                self._retire(e.culprits, str(e))
            except Exception as e:  # noqa: BLE001 - never kill the supervisor thread
                log.exception("[ERROR] worker group start failed unexpectedly")
                self._retire([], f"start: {type(e).__name__}: {e}")
            self._drop_group()

    # ------------------------------------------------------------------ re-probing (background)
    def _probe_due(self) -> bool:
        return (self.group is None and bool(self.retired) and not self._closed and self._probe_thread is None
                and time.time() >= self._next_probe)

    def _start_probe(self, devices: Optional[Sequence[str]] = None) -> None:
        """With no live group and the back-off passed: start a fresh group on every retired
        device (or on ``devices``) on a background thread.  Requests keep failing fast meanwhile
        (a probe must not hold a batch for a whole group start)."""
        back = [d for d in self.all_devices if d in self.retired and (devices is None or d in devices)]
        log.info("[INFO] re-probing retired devices %s", back)
        self._next_probe = float("inf")
        t0 = time.time()

        def run():
            try:
                res = ("ok", self._spawn(back), back, t0)
            except GroupFailure as e:
                res = ("fail", e, back, t0)
            except Exception as e:  # noqa: BLE001
                res = ("fail", GroupFailure(f"probe: {type(e).__name__}: {e}", []), back, t0)
            self._probe_result = res
            self._wake()
        self._probe_thread = threading.Thread(target=run, name="group-probe", daemon=True)
        self._probe_thread.start()

    def _finish_probe(self) -> None:
        if self._probe_result is None:
            return
        self._probe_thread.join()
        kind, obj, back, t0 = self._probe_result
        self._probe_thread, self._probe_result = None, None
        self.probes.append({"devices": back, "ok": kind == "ok", "s": round(time.time() - t0, 3)})
        if kind == "ok":
            if self._closed:
                obj.kill()
                return
            for d in back:
                self.retired.pop(d, None)
            self.healthy = [d for d in self.all_devices if d not in self.retired]
            self._blind = 0
            self._probation = True                   # back-off resets after its first good round
            self._adopt(obj)
            return
        if obj.group is not None:
            obj.group.kill()
        bad = [obj.group.devices[r] for r in obj.culprits if obj.group is not None and 0 <= r < obj.group.world]
        self._probe_backoff = min(2 * self._probe_backoff, 3600.0)
        self._next_probe = time.time() + self._probe_backoff
        if bad and len(bad) < len(back) and not self._closed:
            # the innocent devices are tried again at once, on the same background path: their
            # group start (model load, graph capture) must not stall this loop, so
            # requests keep failing fast until the probe's group is adopted
            innocent = [d for d in back if d not in bad]
            for d in innocent:
                self.retired[d] = "re-probe pending (innocent in a failed probe)"
            self._start_probe(innocent)

    def _round_ok(self) -> None:
        self.rounds += 1
        if self._probation:
            self._probation = False
            self._probe_backoff = self.reprobe_s

    # ------------------------------------------------------------------ requests
    def _wake(self) -> None:
        if self._wake_w is None:                 # lockstep: the loop blocks on _q itself
            return
        with self._wake_lock:
            if self._wake_pending:
                return
            self._wake_pending = True
            try:
                os.write(self._wake_w, b"w")
            except (BlockingIOError, OSError):   # full or closed: a wake-up is already queued
                pass

    def _drain_wake(self) -> None:
        with self._wake_lock:
            self._wake_pending = False
            try:
                while os.read(self._wake_r, 4096):
                    pass
            except (BlockingIOError, OSError):
                pass

    def submit(self, room: str, prompts: Sequence[str], seeds: Sequence[int]) -> cf.Future:
        fut: cf.Future = cf.Future()
        if self._closed:
            fut.set_exception(ImageGenerationError("supervisor closed"))
            return fut
        self._q.put((room, list(prompts), list(seeds), fut, time.monotonic()))
        self._wake()
        return fut

    def wait_ready(self, timeout: Optional[float] = None) -> bool:
        return self._ready.wait(timeout)

    def live_devices(self) -> List[str]:
        return list(self.group.devices) if self.group is not None else []

    # exit code of a worker that caught an exception (usually a collective broken by a dead
    # peer) and reported it: collateral, not a culprit
    REPORTED_EXIT = 5

    def _diagnose(self, g: "_Group", rid: int, reason: str, grace_s: float = 3.0,
                  suspects: Optional[Sequence[int]] = None) -> "GroupFailure":
        """Who broke the round.  A worker that died WITHOUT reporting (crash, OOM kill, signal)
        or stopped heart-beating is a culprit; peers whose collectives then failed exit with
        REPORTED_EXIT and are not.  With nobody dead, the workers that never finished their
        local generation of round ``rid`` are (a wedged GPU: RCCL would block the rest);
        ``suspects`` (async dispatch) names the workers whose own round timed out."""
        t_end = time.time() + grace_s
        while True:
            crashed = [r for r in g.dead() if g.procs[r].exitcode not in (0, self.REPORTED_EXIT)]
            stale = g.stale(self.stale_s)
            if crashed or stale or time.time() > t_end:
                break
            time.sleep(0.05)
        if stale and not crashed:
            stale = self._confirm_stale(g, stale)
        culprits = sorted(set(crashed) | set(stale))
        if not culprits and suspects is not None:
            # async dispatch runs no collective after the start handshake, so a busy worker that
            # reported an error, exited (even with 0 / REPORTED_EXIT) or timed out is the culprit
            # itself, never collateral of a failed peer
            culprits = sorted(set(suspects))
        elif not culprits and rid > 0:
            culprits = [r for r in range(g.world) if g.progress[r] < rid and g.procs[r].exitcode is None]
            if len(culprits) == g.world:         # nobody finished: no evidence against anyone
                culprits = []
        codes = {r: g.procs[r].exitcode for r in range(g.world)}
        return GroupFailure(f"{reason}; exit codes {codes}", culprits)

    def _confirm_stale(self, g: "_Group", stale: Sequence[int]) -> List[int]:
        """Every live worker silent at once is more likely a host stall (CPU starvation, a
        paused container) than that many wedged GPUs: give the heartbeats a few periods to
        resume and keep only the workers that stay silent."""
        live = [r for r in range(g.world) if g.procs[r].exitcode is None]
        if len(live) < 2 or set(stale) < set(live):
            return list(stale)
        t_end = time.time() + max(2.0, 6 * self.heartbeat_s)
        while time.time() < t_end:
            time.sleep(0.1)
            still = g.stale(self.stale_s)
            if set(still) < set(stale):
                return still
        return g.stale(self.stale_s)

    # ------------------------------------------------------------------ lockstep rounds
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
            if g.stale(self.stale_s) and self._confirm_stale(g, g.stale(self.stale_s)):
                raise self._diagnose(g, rid, "worker stopped heart-beating", grace_s=0.0)
            if self.round_timeout > 0 and time.monotonic() - t0 > self.round_timeout:
                raise self._diagnose(g, rid, f"round {rid} exceeded {self.round_timeout:.0f} s", grace_s=0.0)

    def _next_batch(self) -> Optional[list]:
        """Lockstep: block for a request, then collect more until every room is in or the
        window closes.  None once closed."""
        while True:
            timeout = None
            if self.group is None and (self._probe_thread is not None or self.retired):
                timeout = self.watch_period
            try:
                item = self._q.get(timeout=timeout)
            except queue.Empty:
                self._tick_probe()
                continue
            break
        if item is None:
            return None
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
        return batch

    def _tick_probe(self) -> None:
        self._finish_probe()
        if self._probe_due():
            self._start_probe()

    def _loop_lockstep(self) -> None:
        from .rooms import GenJob
        while True:
            batch = self._next_batch()
            if batch is None:
                break
            self._tick_probe()
            if self.group is None:
                self._serve_without_group(batch)
                self._tick_probe()
                continue
            jobs, spans = [], []
            for room, prompts, seeds, fut, _ in batch:
                s = len(jobs)
                jobs.extend(GenJob(room, p, sd) for p, sd in zip(prompts, seeds))
                spans.append((s, len(jobs), room, fut))
            try:
                res = self._run_round(jobs)
                self._round_ok()
                for s, e, room, fut in spans:
                    imgs = [res.get((room, i)) for i in range(s, e)]
                    if any(im is None for im in imgs):
                        fut.set_exception(ImageGenerationError(f"room {room}: generation failed"))
                    else:
                        fut.set_result(imgs)
            except (GroupFailure, EOFError, OSError, BrokenPipeError) as e:
                if not isinstance(e, GroupFailure):       # the leader's pipe broke
                    e = self._diagnose(self.group, self._round_id, f"leader pipe: {type(e).__name__}")
                for *_, fut in spans:
                    if not fut.done():
                        fut.set_exception(ImageGenerationError(f"generation round failed: {e}"))
                self._restart(e.culprits, str(e))
            except Exception as e:  # noqa: BLE001 - unexpected (message shape, pickling): never kill this thread
                log.exception("[ERROR] supervisor round failed unexpectedly")
                for *_, fut in spans:
                    if not fut.done():
                        fut.set_exception(ImageGenerationError(f"generation round failed: {type(e).__name__}: {e}"))
                self._restart([], f"unexpected {type(e).__name__}: {e}")

    # ------------------------------------------------------------------ async (per-worker) rounds
    def _loop_async(self) -> None:
        """Each worker runs its own rounds: a worker is handed the pending requests of the rooms
        it owns as soon as it is idle and either every one of its rooms has asked or the oldest
        request waited ``window_s``.  Results resolve their rooms' futures as each worker
        finishes; nothing waits for the slowest GPU."""
        from multiprocessing.connection import wait as mp_wait
        from .rooms import GenJob
        pending: List[tuple] = []                 # (room, prompts, seeds, fut, t_submit)
        busy: Dict[int, tuple] = {}               # worker -> (rid, spans, t0, n_jobs)
        closing = False
        while True:
            # ---- collect requests
            while True:
                try:
                    item = self._q.get_nowait()
                except queue.Empty:
                    break
                if item is None:
                    closing = True
                    break
                pending.append(item)
            if closing:
                break
            self._tick_probe()
            g = self.group
            if g is None:
                if pending:
                    self._serve_without_group(pending)
                    pending = []
            else:
                # ---- dispatch to idle workers
                now = time.monotonic()
                by_w: Dict[int, List[tuple]] = {}
                for it in pending:
                    by_w.setdefault(self.sharding.owner(it[0]), []).append(it)
                for w, items in by_w.items():
                    if w in busy:
                        continue
                    mine = set(self.sharding.rooms_of(w))
                    if not ({it[0] for it in items} >= mine or now - min(it[4] for it in items) >= self.window):
                        continue
                    jobs, spans = [], []
                    for room, prompts, seeds, fut, _ in items:
                        s0 = len(jobs)
                        jobs.extend(GenJob(room, p, sd) for p, sd in zip(prompts, seeds))
                        spans.append((s0, len(jobs), room, fut))
                    self._round_id += 1
                    try:
                        g.conns[w].send(("round", self._round_id, jobs))
                    except (OSError, EOFError, BrokenPipeError):
                        pass                              # detected below as a dead worker
                    busy[w] = (self._round_id, spans, time.monotonic(), len(jobs))
                    taken = set(map(id, items))
                    pending = [it for it in pending if id(it) not in taken]
            # ---- wait for results / requests / timers
            timeout = self.watch_period if (busy or self._probe_thread is not None
                                            or (self.group is None and self.retired)) else None
            idle_waiting = [it[4] for it in pending if g is not None and self.sharding.owner(it[0]) not in busy]
            if idle_waiting:                      # an idle worker's batching window closes
                timeout = max(0.0, min(timeout if timeout is not None else 1e9,
                                       min(idle_waiting) + self.window - time.monotonic()))
            waitables = [self._wake_r] + [g.conns[w] for w in busy] if g is not None else [self._wake_r]
            ready = mp_wait(waitables, timeout)
            if self._wake_r in ready:
                self._drain_wake()
            if g is None or not busy:
                continue
            # ---- results and failures
            failure: Optional[GroupFailure] = None
            for w in list(busy):
                rid, spans, t0, n = busy[w]
                c = g.conns[w]
                if c in ready:
                    try:
                        msg = c.recv()
                    except (EOFError, OSError) as e:
                        failure = self._diagnose(g, rid, f"worker {w} pipe: {type(e).__name__}", suspects=[w])
                        break
                    if msg[0] in ("result", "result_dev") and msg[1] == rid:
                        del busy[w]
                        if msg[0] == "result":
                            imgs = msg[2]
                        else:
                            try:
                                imgs = self._land(g, w, msg[2])
                            except Exception as e:  # noqa: BLE001 - IPC mapping / copy failed
                                log.exception("[ERROR] landing worker %d's images failed; falling back to "
                                              "the pipe transport", w)
                                self.transport = "pipe"   # the restarted group sends host arrays
                                for s0, e0, room, fut in spans:
                                    if not fut.done():
                                        fut.set_exception(ImageGenerationError(f"image transport failed: {e}"))
                                failure = GroupFailure(f"ipc transport: {type(e).__name__}: {e}", [])
                                break
                        self._round_ok()
                        dev = g.devices[w]
                        self.worker_rounds[dev] = self.worker_rounds.get(dev, 0) + 1
                        for s0, e0, room, fut in spans:
                            got = imgs[s0:e0]
                            if fut.done():
                                continue
                            if len(got) != e0 - s0 or any(im is None for im in got):
                                fut.set_exception(ImageGenerationError(f"room {room}: generation failed"))
                            else:
                                fut.set_result(list(got))
                        continue
                    if msg[0] == "error":
                        failure = self._diagnose(g, rid, f"worker {w} failed: "
                                                 f"{msg[-1].strip().splitlines()[-1][:300]}", suspects=[w])
                        break
                if self.round_timeout > 0 and time.monotonic() - t0 > self.round_timeout:
                    failure = self._diagnose(g, rid, f"worker {w} round {rid} exceeded {self.round_timeout:.0f} s",
                                             grace_s=0.0, suspects=[w])
                    break
            if failure is None and busy:
                if g.dead():
                    failure = self._diagnose(g, max(b[0] for b in busy.values()), "worker exited",
                                             suspects=[w for w in busy if g.procs[w].exitcode is not None])
                elif g.stale(self.stale_s) and self._confirm_stale(g, g.stale(self.stale_s)):
                    failure = self._diagnose(g, 0, "worker stopped heart-beating", grace_s=0.0, suspects=[])
            if failure is not None:
                for _, spans, _, _ in busy.values():
                    for *_, fut in spans:
                        if not fut.done():
                            fut.set_exception(ImageGenerationError(f"generation round failed: {failure}"))
                busy.clear()
                self._restart(failure.culprits, str(failure))
        for it in pending:
            if not it[3].done():
                it[3].set_exception(ImageGenerationError("supervisor closed"))
        for _, spans, _, _ in busy.values():
            for *_, fut in spans:
                if not fut.done():
                    fut.set_exception(ImageGenerationError("supervisor closed"))

    def _stream_for(self, device):
        """The stream the landing copy runs on.  By default the thread's CURRENT stream (no new
        stream in the front-end: one more stream was measured to cost the co-located worker 14 %
        of its images/s -- the GPU's queue scheduler then time-slices more hardware queues,
        profiles/r6_live_ipc_stream_ab.txt); CASSMANTLE_IPC_STREAM=own: a dedicated stream."""
        import torch
        if os.environ.get("CASSMANTLE_IPC_STREAM", "current") == "own":
            if self._land_stream is None:
                self._land_stream = torch.cuda.Stream(device=device)
            return self._land_stream
        return torch.cuda.current_stream(device)

    def _land(self, g: "_Group", w: int, payload: Dict[str, Any]) -> List[Any]:
        """``ipc`` transport, front-end side: the worker's round is in its HBM outbox (mapped here
        once per outbox allocation, HIP IPC).  ``land="device"`` (default): one device-to-device
        copy onto ``frontend_device`` (xGMI when the worker's GPU differs) -> ``DeviceImage``
        handles the blur cache reads in HBM.  ``land="host"``: one DMA copy of the outbox into
        pinned host memory -> uint8 arrays.  Either copy runs on the thread's current stream: a
        landing stream of its own cost the co-located worker 14 % of its images/s and +1.2 ms
        score p50, both landings without it run at pipe speed (profiles/r6_live_ipc_stream_ab.txt)."""
        import torch
        from ..game.content import DeviceImage
        key = (g.epoch, w)
        if payload["buf"] is not None:
            self._inbox = {k: v for k, v in self._inbox.items() if k[0] == g.epoch and k != key}
            self._inbox[key] = payload["buf"]
        shape = tuple(payload["shape"])
        n = int(np.prod(shape))
        src = self._inbox[key][:n].view(shape)
        dev = torch.device(self.frontend_device) if self.frontend_device else None
        diag = os.environ.get("CASSMANTLE_IPC_DIAG", "")     # round-6 diagnosis of the live A/B
        if diag == "noland":
            return [np.zeros(shape[1:], np.uint8) for _ in range(shape[0])]
        t0 = time.perf_counter()
        if src.device.type != "cuda":                          # CPU workers: shared memory
            host = src.numpy()
            out = [host[i].copy() for i in range(shape[0])]
        elif self.land == "host" or dev is None or dev.type != "cuda":
            stream = self._stream_for(src.device)
            host = torch.empty(shape, dtype=torch.uint8, pin_memory=True)
            with torch.cuda.stream(stream):
                host.copy_(src, non_blocking=True)
            stream.synchronize()               # the worker may overwrite its outbox from its next round
            h = host.numpy()
            out = [h[i].copy() for i in range(shape[0])]
        else:
            stream = self._stream_for(dev)
            dst = torch.empty(shape, dtype=torch.uint8, device=dev)
            with torch.cuda.stream(stream):
                if src.device == dev and os.environ.get("CASSMANTLE_IPC_COPY", "kernel") == "kernel":
                    from .. import ops
                    ops.copy_(dst, src)            # in-tree 16-byte copy kernel (same device)
                else:
                    dst.copy_(src, non_blocking=True)
            stream.synchronize()
            out = [DeviceImage(dst[i]) for i in range(shape[0])]
        self.land_us.append((time.perf_counter() - t0) * 1e6)
        return out

    def _loop(self) -> None:
        try:
            self._start_group()
        except GroupFailure as e:
            self._restart(e.culprits, str(e))
        except Exception as e:  # noqa: BLE001
            log.exception("[ERROR] worker group start failed unexpectedly")
            self._restart([], f"start: {type(e).__name__}: {e}")
        self._ready.set()
        try:
            if self.dispatch == "async":
                self._loop_async()
            else:
                self._loop_lockstep()
        finally:
            if self.group is not None:
                self.group.stop()
                self._adopt(None)
            if self._probe_thread is not None:
                self._probe_thread.join(timeout=self.start_timeout)
                if self._probe_result is not None and self._probe_result[0] == "ok":
                    self._probe_result[1].kill()

    def _serve_without_group(self, batch) -> None:
        """No live group: a ``local`` generator serves the batch, otherwise each room's round
        repeats (its request fails fast; the room keeps its content, src/backend.py:211-215)."""
        for room, prompts, seeds, fut, *_ in batch:
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
        self._wake()
        self._thread.join(timeout=120)
        if self.group is not None:
            self.group.kill()
            self._adopt(None)
        if self._wake_w is not None and not self._thread.is_alive():
            with self._wake_lock:                # no writer can reach a recycled fd number
                w, r, self._wake_w = self._wake_w, self._wake_r, None
            os.close(w)
            os.close(r)

    def status(self) -> Dict[str, Any]:
        return {"epoch": self.epoch, "live_devices": self.live_devices(), "retired": dict(self.retired),
                "rounds": self.rounds, "failures": list(self.failures), "probes": list(self.probes),
                "dispatch": self.dispatch, "worker_rounds": dict(self.worker_rounds),
                "owners": ({r: self.group.devices[self.sharding.owner(r)] for r in self.room_ids}
                           if self.group is not None else {}),
                "gather_us_p50": float(np.median(self.gather_us)) if self.gather_us else None,
                "transport": self.transport if self.dispatch == "async" else "rccl-gather",
                "land_us_p50": float(np.median(self.land_us)) if self.land_us else None}


class SupervisedImageGenerator(ImageGenerator):
    """Game-layer generator for one room, served by the supervised worker group."""

    def __init__(self, sup: GroupSupervisor, room: str, timeout_s: float = 1800.0) -> None:
        self.sup = sup
        self.room = room
        self.resolution = sup.resolution
        self.timeout = timeout_s

    def generate(self, prompts, negative_prompt, seeds):
        return self.sup.submit(self.room, prompts, seeds).result(timeout=self.timeout)
