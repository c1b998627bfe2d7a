"""A/B of the A-in-registers short-K GEMM (ops/csrc/gemm_areg.hip, cfg 15) against the planner's
pick (tuning table off) and stock torch (hipBLASLt) at the SD-1.5 batch-8 (CFG x 4 images) level-1/2
transformer shapes.  Interleaved rounds, median per arm, one JSON line per shape.

    python tools/bench_areg.py [--rounds 5] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("CASSMANTLE_GEMM_TUNE", "0")
from cassmantle_amd import ops  # noqa: E402
from cassmantle_amd.ops._ext import ext  # noqa: E402

# (name, M, N, K, act, residual)
SHAPES = [
    ("l1_qkv", 32768, 960, 320, "none", False),
    ("l1_proj", 32768, 320, 320, "none", True),
    ("l1_q", 32768, 320, 320, "none", False),
    ("l1_geglu", 32768, 1280, 320, "geglu", False),
    ("l2_qkv", 8192, 1920, 640, "none", False),
    ("l2_proj", 8192, 640, 640, "none", True),
    ("l2_geglu", 8192, 2560, 640, "geglu", False),
]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    ops.set_mode("hip")
    ext().gemm_tune_clear()
    for name, M, N, K, act, res in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        nw = 2 * N if act == "geglu" else N
        w = (torch.randn(nw, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
        b = (torch.randn(nw, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
        r = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16) if res else None
        arms = {}

        def mk(cfg):
            def f():
                ext().gemm_set_override(cfg, 0)
                ops.linear(x, w, b, residual=r, act=act)
            return f
        arms["auto"] = mk(-1)
        arms["areg"] = mk(15)
        arms["torch"] = lambda: torch.nn.functional.linear(x, w, b)
        res_t = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, f in arms.items():
                res_t[k].append(timeit(f, a.iters))
        ext().gemm_set_override(-1, 0)
        med = {k: round(statistics.median(v), 2) for k, v in res_t.items()}
        flops = 2.0 * M * nw * K
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "act": act, "us": med,
                          "areg_tflops": round(flops / med["areg"] / 1e6, 1),
                          "areg_vs_auto": round(med["auto"] / med["areg"], 3)}), flush=True)


if __name__ == "__main__":
    main()
