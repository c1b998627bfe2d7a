"""Flash-attention microbenchmark at the SD-1.5 / SDXL / text-encoder shapes, bf16 and (head dim
64) OCP-fp8, vs stock torch SDPA.  Interleaved rounds, median per arm, one JSON line per shape.

    python tools/bench_attn.py [--rounds 5] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402

SHAPES = [  # B, Nq, Nk, H, d
    (8, 4096, 4096, 8, 40),     # SD-1.5 level-1 self-attention (batch 4 x CFG)
    (8, 4096, 77, 8, 40),       # SD-1.5 level-1 cross-attention
    (8, 1024, 1024, 8, 80),     # SD-1.5 level-2
    (8, 256, 256, 8, 160),      # SD-1.5 level-3
    (2, 4096, 4096, 10, 64),    # SDXL level-2 self (batch 1 x CFG)
    (2, 1024, 1024, 20, 64),    # SDXL level-3 self
    (2, 4096, 77, 10, 64),      # SDXL level-2 cross
    (2, 1024, 77, 20, 64),      # SDXL level-3 cross
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
    ap.add_argument("--only-d", type=int, default=None)
    a = ap.parse_args()
    ops.set_mode("hip")
    for B, Nq, Nk, H, d in SHAPES:
        if a.only_d is not None and d != a.only_d:
            continue
        g = torch.Generator(device="cuda").manual_seed(0)
        q = torch.randn(B, Nq, H, d, device="cuda", generator=g).to(torch.bfloat16)
        k = torch.randn(B, Nk, H, d, device="cuda", generator=g).to(torch.bfloat16)
        v = torch.randn(B, Nk, H, d, device="cuda", generator=g).to(torch.bfloat16)
        arms = {"bf16": lambda: ops.attention(q, k, v),
                "sdpa": lambda: F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2))}
        if d == 40:                        # the 32x32x16 kernel the 16x16 one replaced (A/B)
            def old_kernel():
                ops.set_attention_d40_variant("32x32")
                ops.attention(q, k, v)
                ops.set_attention_d40_variant(None)
            arms["bf16_32x32"] = old_kernel
        if d == 64:
            arms["fp8"] = lambda: ops.attention(q, k, v, fp8="force")
            kv8 = ops.pack_kv_fp8(k, v)          # cross-attention: packed once per text context
            arms["fp8_prepacked"] = lambda: ops.attention(q, k, v, fp8=True, kv8=kv8)
        res = {kk: [] for kk in arms}
        for _ in range(a.rounds):
            for kk, f in arms.items():
                res[kk].append(timeit(f, a.iters))
        med = {kk: round(statistics.median(x), 2) for kk, x in res.items()}
        flops = 4.0 * B * H * Nq * Nk * d
        line = {"shape": [B, Nq, Nk, H, d], "us": med, "bf16_tflops": round(flops / med["bf16"] / 1e6, 1),
                "bf16_vs_sdpa": round(med["sdpa"] / med["bf16"], 3)}
        if "bf16_32x32" in med:
            line["d40_16x16_vs_32x32"] = round(med["bf16_32x32"] / med["bf16"], 3)
        if "fp8" in med:
            line["fp8_vs_bf16"] = round(med["bf16"] / med["fp8"], 3)
            line["fp8_prepacked_vs_bf16"] = round(med["bf16"] / med["fp8_prepacked"], 3)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
