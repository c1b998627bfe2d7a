"""Microbenchmark of the decode-path kernels (GEMV, decode attention) on Mistral-7B shapes.

    python tools/bench_decode.py       -> one JSON line per case (us, achieved GB/s)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cassmantle_amd import ops  # noqa: E402


def timeit(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters // 20):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (iters // 20 * 20)


def main():
    dev = "cuda"
    for (N, K, act) in [(6144, 4096, None), (4096, 4096, None), (14336, 4096, "swiglu"), (4096, 14336, None),
                        (32000, 4096, None)]:
        x = torch.randn(1, K, device=dev).bfloat16()
        w = (torch.randn((2 * N if act else N), K, device=dev) * 0.02).bfloat16()
        gam = torch.ones(K, device=dev).bfloat16()
        us = timeit(lambda: ops.linear(x, w, act=act))
        us_rms = timeit(lambda: ops.rms_linear(x, gam, 1e-5, w, act=act))
        gbs = w.numel() * 2 / us / 1e3
        print(json.dumps({"op": "gemv", "N": N, "K": K, "act": act, "us": round(us, 2), "GBps": round(gbs, 1),
                          "us_rms_fused": round(us_rms, 2)}))
    for (L, ln) in [(512, 96), (512, 500), (4096, 300), (4096, 4000)]:
        q = torch.randn(1, 32, 128, device=dev).bfloat16()
        kc = torch.randn(1, L, 8, 128, device=dev).bfloat16()
        vc = torch.randn(1, L, 8, 128, device=dev).bfloat16()
        lens = torch.tensor([ln], device=dev, dtype=torch.int32)
        us = timeit(lambda: ops.decode_attention(q, kc, vc, lens))
        print(json.dumps({"op": "decode_attention", "L": L, "len": ln, "us": round(us, 2),
                          "GBps": round(2 * ln * 8 * 128 * 2 / us / 1e3, 1)}))


if __name__ == "__main__":
    main()
