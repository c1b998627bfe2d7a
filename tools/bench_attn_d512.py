"""A/B of the head-dim-512 attention (VAE mid-block): the flash kernel (ops/csrc/attention_d512.hip)
vs the round-1 GEMM -> row-softmax -> GEMM path (ops._attention_gemm, materialises S) vs stock
torch SDPA, at the SD-1.5 VAE shape (4 images x 4096 tokens) and the SDXL one (1 x 16384).
Interleaved rounds, median per arm, one JSON line per shape.

    python tools/bench_attn_d512.py [--rounds 5] [--iters 10]
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
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    ops.set_mode("hip")
    for B, N in [(4, 4096), (1, 16384), (2, 16384)]:
        qkv = torch.randn(B, N, 3, 1, 512, device="cuda").to(torch.bfloat16)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        arms = {
            "flash": lambda: ops.attention(q, k, v),
            "sdpa": lambda: F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)),
        }
        if N <= 4096:      # the materialised-S path: [B, N, N] fp32 (1 GiB per image at 16384)
            arms["gemm_path"] = lambda: ops._attention_gemm(q, k, v, 512 ** -0.5, False, None)
        res = {kk: [] for kk in arms}
        for _ in range(a.rounds):
            for kk, f in arms.items():
                res[kk].append(timeit(f, a.iters))
        med = {kk: round(statistics.median(v), 1) for kk, v in res.items()}
        flops = 4.0 * B * N * N * 512
        err = (ops.attention(q, k, v).float() - F.scaled_dot_product_attention(
            q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)).transpose(1, 2).float()).abs().max().item()
        print(json.dumps({"B": B, "N": N, "us": med, "flash_tflops": round(flops / med["flash"] / 1e6, 1),
                          "flash_vs_sdpa": round(med["sdpa"] / med["flash"], 3), "max_abs_diff_vs_sdpa": err}),
              flush=True)
        del qkv, q, k, v
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
