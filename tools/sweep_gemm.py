"""Tile-config x split-K sweep of the GEMM/conv planner at the UNet shapes that are too small to
fill 256 CUs with one tile per block (the 32x32 / 16x16 / 8x8 levels, batch 8).  Prints one JSON
line per shape: the cost model's pick, the measured best and the full table (us, including the
split-K reduce pass).

    python tools/sweep_gemm.py [--iters 20]
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

CFGS = {0: "128x128", 1: "128x160", 2: "256x64", 3: "128x64", 5: "256x160/8w", 6: "256x128/8w"}
SPLITS = [1, 2, 3, 4, 6, 8, 12, 16]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def rnd(*s, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).to(torch.bfloat16)


def cases():
    # (name, callable factory) at batch 8 (4 images x CFG)
    for B, H, Cin, Cout, st in [(8, 32, 640, 640, 1), (8, 32, 1280, 640, 1), (8, 16, 1280, 1280, 1),
                                (8, 16, 2560, 1280, 1), (8, 8, 1280, 1280, 1), (8, 8, 2560, 1280, 1),
                                (8, 64, 320, 320, 2), (8, 32, 640, 640, 2), (8, 16, 1280, 1280, 2)]:
        x = rnd(B, H, H, Cin)
        w = rnd(Cout, 3, 3, Cin, scale=(9 * Cin) ** -0.5)
        b = rnd(Cout, scale=0.1)
        Ho = H // st
        yield (f"conv{H}x{H}_{Cin}->{Cout}_s{st}", 2.0 * B * Ho * Ho * Cout * 9 * Cin,
               lambda x=x, w=w, b=b, st=st: ops.conv2d(x, w, b, stride=st, padding=1))
    for M, N, K in [(8192, 640, 640), (8192, 1920, 640), (8192, 640, 2560), (2048, 1280, 1280),
                    (2048, 3840, 1280), (2048, 1280, 5120), (512, 1280, 1280), (512, 3840, 1280),
                    (512, 1280, 5120)]:
        x, w, b = rnd(M, K), rnd(N, K, scale=K ** -0.5), rnd(N, scale=0.1)
        yield f"gemm_{M}x{N}x{K}", 2.0 * M * N * K, lambda x=x, w=w, b=b: ops.linear(x, w, b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    ops.set_mode("hip")
    with torch.no_grad():
        for name, fl, fn in cases():
            ext().gemm_set_override(-1, 0)
            auto = timeit(fn, a.iters)
            table = {}
            for c in CFGS:
                for sp in SPLITS:
                    ext().gemm_set_override(c, sp)
                    table[f"{c}/{sp}"] = round(timeit(fn, a.iters), 1)
            ext().gemm_set_override(-1, 0)
            best = min(table, key=table.get)
            print(json.dumps({"shape": name, "auto_us": round(auto, 1), "best": best, "best_us": table[best],
                              "auto_tflops": round(fl / auto / 1e6, 1), "best_tflops": round(fl / table[best] / 1e6, 1),
                              "table": table}), flush=True)


if __name__ == "__main__":
    main()
