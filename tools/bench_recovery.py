"""How long rooms go without generation after a GPU worker dies (verdict r3 item 8).

The front-end's ``GroupSupervisor`` runs one worker per device.  This tool warms the group (graph
capture included), SIGKILLs a worker -- a crash / OOM kill / driver fault -- and then keeps
submitting a room's generation request until an image comes back.  On ONE device the dead
worker's device is retired, every device is then gone, and the supervisor's re-probe
(``reprobe_s``, 0 here) brings a fresh group up on the same device: the measured wall time is the
whole recovery path a one-GPU node takes (death detected, group torn down, worker process
spawned, process group + pipeline built, denoise graph captured, first image).  On N devices
the survivors' group restarts without the dead one.

    python tools/bench_recovery.py [--gpus 1] [--model sd15]

One JSON line: ``recovery_s`` (kill -> first image), the failed requests in between (the rooms'
rounds repeat meanwhile, as the reference's do, ``src/backend.py:211-215``), the group start time
of the respawn and the time of one steady-state generation for scale.
"""
import argparse
import json
import os
import signal
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--model", default="sd15")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--victim", type=int, default=0, help="worker rank to kill")
    a = ap.parse_args()
    import torch
    from cassmantle_amd.config import Config
    from cassmantle_amd.game.content import ImageGenerationError
    from cassmantle_amd.parallel.supervisor import GroupSupervisor
    from cassmantle_amd.pipeline import SPECS

    gpu = torch.cuda.device_count() > 0            # (no GPU initialisation in this process)
    devices = [f"cuda:{i}" if gpu else f"cpu:{i}" for i in range(a.gpus)]
    spec = SPECS[a.model]
    cfg = Config()
    cfg.model.image_model = a.model
    cfg.model.resolution = spec.resolution
    cfg.model.steps = spec.steps
    cfg.model.scheduler = spec.scheduler
    cfg.model.guidance_scale = spec.guidance
    cfg.model.device = "cuda" if gpu else "cpu"
    rooms = [""] + [str(i) for i in range(1, a.gpus)]
    t = time.perf_counter()
    sup = GroupSupervisor(cfg, devices, rooms, window_s=0.02, start_timeout_s=1200, reprobe_s=0.0,
                          watch_period_s=0.05)
    assert sup.wait_ready(1500) and sup.live_devices(), sup.status()
    start_s = time.perf_counter() - t
    prompts = [f"A painted style piece depicting the following: scene {j}." for j in range(a.batch)]

    def gen(room, seed):
        return sup.submit(room, prompts, [seed + j for j in range(a.batch)]).result(timeout=1800)

    gen("", 1)                                      # warm: graph capture
    t = time.perf_counter()
    gen("", 2)
    steady_s = time.perf_counter() - t
    victim = sup.group.procs[a.victim].pid
    t_kill = time.perf_counter()
    os.kill(victim, signal.SIGKILL)
    failed = 0
    while True:
        try:
            img = gen("", 3 + failed)
            break
        except ImageGenerationError:
            failed += 1
            if time.perf_counter() - t_kill > 1800:
                raise SystemExit("no recovery within 30 min")
    recovery_s = time.perf_counter() - t_kill
    st = sup.status()
    sup.close()
    print(json.dumps({
        "metric": "worker death -> first image from the respawned group (supervised worker groups)",
        "recovery_s": round(recovery_s, 2), "failed_requests_meanwhile": failed,
        "respawn_group_start_s": st["probes"][-1]["s"] if st["probes"] else None,
        "initial_group_start_s": round(start_s, 2), "steady_generation_s": round(steady_s, 3),
        "devices": devices, "victim": a.victim, "epoch": st["epoch"], "live_devices": st["live_devices"],
        "image_shape": list(img[0].shape), "config": {"model": a.model, "batch": a.batch}}), flush=True)


if __name__ == "__main__":
    main()
