"""fp8 attention block shapes (ops.FP8_ATTN_VARIANTS: NQ query groups x NS key splits) at the
SDXL shapes, K/V pre-packed (the kernel alone) and with the per-call pack, vs the bf16 kernel.
Interleaved rounds, median per arm; one JSON line per shape.

    python tools/bench_attn_fp8.py [--rounds 5] [--iters 30]
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

SHAPES = [(2, 1024, 1024, 20), (2, 4096, 4096, 10), (2, 1024, 77, 20), (2, 4096, 77, 10)]


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
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    for B, Nq, Nk, H in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(0)
        q = torch.randn(B, Nq, H, 64, device="cuda", generator=g).to(torch.bfloat16)
        k = torch.randn(B, Nk, H, 64, device="cuda", generator=g).to(torch.bfloat16)
        v = torch.randn(B, Nk, H, 64, device="cuda", generator=g).to(torch.bfloat16)
        kv8 = ops.pack_kv_fp8(k, v)

        def arm(var, pre):
            def f():
                ops.set_fp8_attention_variant(var)
                if pre:
                    ops.attention(q, k, v, fp8=True, kv8=kv8)
                else:
                    ops.attention(q, k, v, fp8="force")
            return f
        arms = {"bf16": lambda: ops.attention(q, k, v), "pack": lambda: ops.pack_kv_fp8(k, v, out=kv8)}
        arms["rule"] = arm(None, True)
        for var in ops.FP8_ATTN_VARIANTS:
            arms[var] = arm(var, True)
        res = {n: [] for n in arms}
        for _ in range(a.rounds):
            for n, fn in arms.items():
                res[n].append(timeit(fn, a.iters))
        ops.set_fp8_attention_variant(None)
        med = {n: round(statistics.median(v), 2) for n, v in res.items()}
        best = min(ops.FP8_ATTN_VARIANTS, key=lambda n: med[n])
        print(json.dumps({"shape": [B, Nq, Nk, H, 64], "us": med, "best": best,
                          "rule_vs_bf16": round(med["bf16"] / med["rule"], 3),
                          "rule_plus_pack_vs_bf16": round(med["bf16"] / (med["rule"] + med["pack"]), 3)}), flush=True)


if __name__ == "__main__":
    main()
