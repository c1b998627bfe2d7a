"""Reproduce / rule out the round-1 stall: guess scoring on the LEGACY DEFAULT stream in one thread
while another thread replays the captured SD-1.5 denoise graph (tools/bench_live.py note).

Arms (``--arm``):
  legacy   the scorer's kernels + its D2H copy on the legacy NULL stream (round-1 stalling setup)
  stream   the scorer on its own non-blocking stream (what serving does)

Every ~1 s a progress line is printed.  A watchdog (faulthandler) dumps every thread's Python
stack and exits if the run makes no progress for ``--watchdog`` seconds, so a stall ends the
process with evidence of where each thread was blocked instead of hanging the box.

    python tools/repro_stall.py --arm legacy --seconds 40
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arm", default="legacy", choices=["legacy", "stream"])
    ap.add_argument("--seconds", type=float, default=40.0)
    ap.add_argument("--watchdog", type=float, default=45.0)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    from cassmantle_amd.game.scoring import score_pairs
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    from cassmantle_amd.scoring.encoder import EncoderBackend

    sd = StableDiffusion(SPECS["sd15"], device="cuda", seed=0)
    neg = "blurry"
    prompts = [f"a lantern tower {i}" for i in range(4)]
    sd.generate_tensor(prompts, neg, list(range(4)), steps=a.steps).cpu()      # capture the graph
    be = EncoderBackend(device="cuda", use_graphs=False)
    if a.arm == "legacy":
        be.stream = None        # scorer kernels + copies on the thread's legacy default stream
    words = ["lantern", "river", "tower", "ember", "shadow", "glowing", "crimson", "ancient"]
    score_pairs(be, [(w, "tower") for w in words], 0.01)
    torch.cuda.synchronize()

    stop = threading.Event()
    counts = {"images": 0, "scores": 0}

    def gen_loop():
        step = 0
        while not stop.is_set():
            sd.generate_tensor(prompts, neg, [step * 4 + j for j in range(4)], steps=a.steps).cpu()
            counts["images"] += 4
            step += 1

    th = threading.Thread(target=gen_loop, daemon=True)
    t0 = time.perf_counter()
    last_progress = time.perf_counter()
    faulthandler.dump_traceback_later(a.watchdog, exit=True)
    th.start()
    last = dict(counts)
    next_print = t0 + 1.0
    i = 0
    while time.perf_counter() - t0 < a.seconds:
        pairs = [(words[(i + j) % 8], "tower") for j in range(64)]
        score_pairs(be, pairs, 0.01)
        counts["scores"] += 1
        i += 1
        now = time.perf_counter()
        if now >= next_print:
            print(json.dumps({"t": round(now - t0, 1), **counts}), flush=True)
            if counts != last:
                faulthandler.cancel_dump_traceback_later()
                faulthandler.dump_traceback_later(a.watchdog, exit=True)
                last = dict(counts)
            next_print = now + 1.0
    stop.set()
    th.join(timeout=120)
    faulthandler.cancel_dump_traceback_later()
    print(json.dumps({"arm": a.arm, "result": "no stall", "seconds": round(time.perf_counter() - t0, 1), **counts}),
          flush=True)


if __name__ == "__main__":
    main()
