"""Per-op microbenchmark at the SD-1.5 / VAE shapes: HIP kernels vs stock PyTorch-ROCm ops
(hipBLASLt GEMM, MIOpen conv, aotriton SDPA, ATen norms).  Prints one JSON line per case.

    python tools/bench_ops.py [--only gemm,conv,attn,norm] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def rnd(*s, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).to(torch.bfloat16)


def emit(kind, shape, flops, t_ours, t_ref, extra=None):
    d = {"op": kind, "shape": shape, "ours_us": round(t_ours, 1), "torch_us": round(t_ref, 1),
         "speedup": round(t_ref / t_ours, 3)}
    if flops:
        d["ours_tflops"] = round(flops / t_ours / 1e6, 1)
        d["torch_tflops"] = round(flops / t_ref / 1e6, 1)
    if extra:
        d.update(extra)
    print(json.dumps(d), flush=True)


def bench_gemm(it):
    for M, N, K, act in [(32768, 320, 320, None), (32768, 960, 320, None), (32768, 2560, 320, "geglu"),
                         (32768, 320, 1280, None), (8192, 640, 640, None), (8192, 2560, 2560, "geglu"),
                         (8192, 640, 2560, None), (2048, 1280, 1280, None), (616, 768, 768, None),
                         (4096, 4096, 4096, None)]:
        x = rnd(M, K)
        w = rnd(2 * N if act == "geglu" else N, K, scale=K ** -0.5)
        b = rnd(w.shape[0], scale=0.1)
        ops.set_mode("hip")
        t1 = timeit(lambda: ops.linear(x, w, b, act=act), it)
        ops.set_mode("torch")
        t2 = timeit(lambda: ops.linear(x, w, b, act=act), it)
        ops.set_mode("hip")
        fl = 2.0 * M * w.shape[0] * K
        emit("gemm" + ("_geglu" if act else ""), [M, N, K], fl, t1, t2)


def bench_conv(it):
    for B, H, Cin, Cout, st, up in [(8, 64, 320, 320, 1, False), (8, 64, 640, 320, 1, False),
                                   (8, 32, 640, 640, 1, False), (8, 16, 1280, 1280, 1, False),
                                   (8, 8, 1280, 1280, 1, False), (8, 64, 320, 320, 2, False),
                                   (8, 32, 1280, 1280, 1, True),
                                   (4, 64, 512, 512, 1, False), (4, 128, 512, 512, 1, False),
                                   (4, 256, 512, 256, 1, False), (4, 256, 256, 256, 1, False),
                                   (4, 512, 256, 128, 1, False), (4, 512, 128, 128, 1, False),
                                   (8, 64, 4, 320, 1, False), (8, 64, 320, 4, 1, False), (4, 512, 128, 3, 1, False)]:
        x = rnd(B, H, H, Cin)
        w = rnd(Cout, 3, 3, Cin, scale=(9 * Cin) ** -0.5)
        b = rnd(Cout, scale=0.1)
        ops.set_mode("hip")
        t1 = timeit(lambda: ops.conv2d(x, w, b, stride=st, padding=1, upsample=up), it)
        ops.set_mode("torch")
        t2 = timeit(lambda: ops.conv2d(x, w, b, stride=st, padding=1, upsample=up), it)
        ops.set_mode("hip")
        Ho = (2 * H if up else H) // st
        fl = 2.0 * B * Ho * Ho * Cout * 9 * Cin
        emit("conv3x3", [B, H, H, Cin, Cout, st, int(up)], fl, t1, t2)


def bench_attn(it):
    for B, Nq, Nk, Hh, d in [(8, 4096, 4096, 8, 40), (8, 4096, 77, 8, 40), (8, 1024, 1024, 8, 80),
                             (8, 1024, 77, 8, 80), (8, 256, 256, 8, 160), (8, 64, 64, 8, 160),
                             (4, 4096, 4096, 1, 512), (8, 77, 77, 12, 64)]:
        q, k, v = rnd(B, Nq, Hh, d), rnd(B, Nk, Hh, d), rnd(B, Nk, Hh, d)
        ops.set_mode("hip")
        t1 = timeit(lambda: ops.attention(q, k, v), it)
        ops.set_mode("torch")
        t2 = timeit(lambda: ops.attention(q, k, v), it)
        ops.set_mode("hip")
        fl = 4.0 * B * Hh * Nq * Nk * d
        emit("attention", [B, Nq, Nk, Hh, d], fl, t1, t2)
    # SDXL shapes (head dim 64): bf16 kernel vs the fp8 (OCP e4m3) kernel (BASELINE config 4)
    for B, Nq, Nk, Hh in [(2, 4096, 4096, 10), (2, 1024, 1024, 20), (2, 4096, 77, 10), (2, 1024, 77, 20)]:
        q, k, v = rnd(B, Nq, Hh, 64), rnd(B, Nk, Hh, 64), rnd(B, Nk, Hh, 64)
        t8 = timeit(lambda: ops.attention(q, k, v, fp8="force"), it)
        t16 = timeit(lambda: ops.attention(q, k, v), it)
        emit("attention_fp8_vs_bf16", [B, Nq, Nk, Hh, 64], 4.0 * B * Hh * Nq * Nk * 64, t8, t16)


def bench_norm(it):
    for shape, G in [((8, 64, 64, 320), 32), ((8, 64, 64, 640), 32), ((8, 16, 16, 2560), 32),
                     ((4, 512, 512, 128), 32), ((4, 256, 256, 256), 32), ((4, 128, 128, 512), 32)]:
        x = rnd(*shape)
        g, b = rnd(shape[-1]), rnd(shape[-1])
        ops.set_mode("hip")
        t1 = timeit(lambda: ops.group_norm(x, G, g, b, 1e-5, True), it)
        ops.set_mode("torch")
        t2 = timeit(lambda: ops.group_norm(x, G, g, b, 1e-5, True), it)
        ops.set_mode("hip")
        gb = 2 * x.numel() * 2 / 1e9
        emit("group_norm_silu", list(shape), 0, t1, t2, {"ours_GBps": round(gb / (t1 * 1e-6), 1)})
    for rows, D in [(32768, 320), (8192, 640), (2048, 1280), (924, 768)]:
        x = rnd(rows, D)
        g, b = rnd(D), rnd(D)
        ops.set_mode("hip")
        t1 = timeit(lambda: ops.layer_norm(x, g, b, 1e-5), it)
        ops.set_mode("torch")
        t2 = timeit(lambda: ops.layer_norm(x, g, b, 1e-5), it)
        ops.set_mode("hip")
        gb = 2 * x.numel() * 2 / 1e9
        emit("layer_norm", [rows, D], 0, t1, t2, {"ours_GBps": round(gb / (t1 * 1e-6), 1)})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="gemm,conv,attn,norm")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    torch.manual_seed(0)
    sel = a.only.split(",")
    with torch.no_grad():
        if "gemm" in sel:
            bench_gemm(a.iters)
        if "conv" in sel:
            bench_conv(a.iters)
        if "attn" in sel:
            bench_attn(a.iters)
        if "norm" in sel:
            bench_norm(a.iters)


if __name__ == "__main__":
    main()
