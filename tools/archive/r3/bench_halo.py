"""Halo-staged 3x3 conv (tile configs 24 / 25, gemm_halo.h) vs the CONV-2 ping-pong tiles on the
SD-1.5 UNet / VAE 3x3 conv shapes, with the UNet epilogue (bias, per-image time bias, GroupNorm
statistics; residual on the second conv of a ResNet block).  Each arm: 10 back-to-back launches
replayed from a captured graph, arms interleaved over rounds in one process; median us.

    python tools/bench_halo.py [--rounds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402
from cassmantle_amd.ops._ext import ext  # noqa: E402

SHAPES = [  # B, H, W, Cin, Cout, residual
    (8, 64, 64, 320, 320, False), (8, 64, 64, 320, 320, True), (8, 64, 64, 640, 320, False),
    (8, 64, 64, 960, 320, False), (8, 32, 32, 320, 640, False), (8, 32, 32, 640, 640, True),
    (8, 32, 32, 1280, 640, False), (8, 32, 32, 1920, 640, False), (8, 16, 16, 640, 1280, False),
    (8, 16, 16, 1280, 1280, True), (8, 16, 16, 2560, 1280, False),
    (4, 64, 64, 512, 512, False),            # VAE decoder, 64^2 level
]
ARMS = [(8, 1), (8, 2), (20, 1), (20, 2), (7, 1), (24, 1), (24, 2), (24, 3), (24, 4), (25, 1), (25, 2)]


def graph_time(fn, reps=10):
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
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * reps) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    ops.set_mode("hip")
    ops.load_gemm_tuning()
    for (B, H, W, Cin, Cout, resid) in SHAPES:
        x = (torch.randn(B, H, W, Cin, device="cuda") * 0.5).to(torch.bfloat16)
        w = (torch.randn(Cout, 3, 3, Cin, device="cuda") * (9 * Cin) ** -0.5).to(torch.bfloat16)
        b = (torch.randn(Cout, device="cuda") * 0.1).to(torch.bfloat16)
        cb = (torch.randn(B, Cout, device="cuda") * 0.1).to(torch.bfloat16)
        res = (torch.randn(B, H, W, Cout, device="cuda") * 0.5).to(torch.bfloat16) if resid else None
        st = ops.new_stats(B, Cout, "cuda")
        flop = 2.0 * B * H * W * Cout * 9 * Cin

        def call():
            ops.zero_(st)
            ops.conv2d(x, w, b, residual=res, chan_bias=cb, stats=st)

        ext().gemm_set_override(-1, 0)
        call()
        auto = tuple(ext().gemm_last_plan())
        ref = ops.conv2d(x, w, b, residual=res, chan_bias=cb)
        arms = {"auto": (-1, 0)}
        for c, sp in ARMS:
            ext().gemm_set_override(c, sp)
            call()
            if tuple(ext().gemm_last_plan()) == (c, sp):
                out = ops.conv2d(x, w, b, residual=res, chan_bias=cb)
                err = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
                assert err < 1e-2, (c, sp, err)
                arms[f"{c}/{sp}"] = (c, sp)
        times = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, (c, sp) in arms.items():
                ext().gemm_set_override(c, sp)
                times[k].append(graph_time(call))
        ext().gemm_set_override(-1, 0)
        med = {k: round(statistics.median(v), 2) for k, v in times.items()}
        best = min(med, key=med.get)
        print(json.dumps({"shape": [B, H, W, Cin, Cout], "residual": resid, "auto_plan": list(auto),
                          "best": best, "best_us": med[best], "best_tflops": round(flop / med[best] / 1e6, 1),
                          "us": med}), flush=True)


if __name__ == "__main__":
    main()
