"""Where does a latency-bound UNet GEMM spend its time?  The level-3 projections (M = 2048,
N = 1280, K = 1280: 27 calls per SD-1.5 UNet eval at 17-24 us, ~400 TF/s) timed at K = 64 ..
2560 for the candidate tiles, each as 20 back-to-back launches replayed from a captured graph
(no host launch cost), so the intercept (per-launch floor: dispatch, prologue, epilogue, drain)
and the slope (per 64-deep k-tile) separate.  Also the floor of an empty in-tree kernel.

    python tools/probe_small_gemm.py [--m 2048 --n 1280]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402
from cassmantle_amd.ops._ext import ext  # noqa: E402


def graph_time(fn, reps=20, replays=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(replays):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * replays) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=2048)
    ap.add_argument("--n", type=int, default=1280)
    ap.add_argument("--ks", default="64,128,256,640,1280,2560")
    ap.add_argument("--cfgs", default="3,0,13,16,21,22,23,8")
    ap.add_argument("--rotate", type=int, default=1,
                    help="cycle through this many weight AND activation copies per replay (>= 40 at "
                         "M 2048 x N 1280: every launch reads both from HBM, as a UNet eval does for weights)")
    ap.add_argument("--splits", default="1,2,4")
    a = ap.parse_args()
    ops.set_mode("hip")
    ops.load_gemm_tuning()
    z = torch.zeros(256, device="cuda", dtype=torch.float32)
    print(json.dumps({"case": "empty zero_ kernel", "us": round(graph_time(lambda: ops.zero_(z)), 2)}), flush=True)
    for K in [int(k) for k in a.ks.split(",")]:
        xs = [(torch.randn(a.m, K, device="cuda") * 0.5).to(torch.bfloat16) for _ in range(a.rotate)]
        ws = [(torch.randn(a.n, K, device="cuda") / K ** 0.5).to(torch.bfloat16) for _ in range(a.rotate)]
        b = torch.zeros(a.n, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(a.m, a.n, device="cuda", dtype=torch.bfloat16)
        it = [0]

        def call():
            i = it[0] % a.rotate
            it[0] += 1
            ops.linear(xs[i], ws[i], b, out=out)
        x, w = xs[0], ws[0]
        row = {"M": a.m, "N": a.n, "K": K}
        for c in [int(c) for c in a.cfgs.split(",")]:
            for sp in [int(v) for v in a.splits.split(",")]:
                if sp > 1 and K // 64 // sp < 4:
                    continue
                ext().gemm_set_override(c, sp)
                ops.linear(x, w, b, out=out)
                got = tuple(ext().gemm_last_plan())
                if got != (c, sp):
                    continue
                row[f"{c}/{sp}"] = round(graph_time(call, reps=max(20, a.rotate)), 2)
        ext().gemm_set_override(-1, 0)
        row["auto"] = round(graph_time(call, reps=max(20, a.rotate)), 2)
        row["auto_plan"] = list(ext().gemm_last_plan())
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
