"""Per-kernel fixed cost inside a replayed hipGraph: N back-to-back tiny kernels (the in-tree
advance_step kernel: one thread, one int) vs N=0, and a few real norm kernels for scale."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd.ops._ext import ext  # noqa: E402


def graph_time(fn, reps=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    e = ext()
    step = torch.zeros(1, dtype=torch.int32, device="cuda")
    for n in (1, 100, 500, 1000):
        t = graph_time(lambda: [e.advance_step(step) for _ in range(n)])
        print(f"graph of {n:5d} tiny kernels: {t:9.1f} us total, {t / n:6.2f} us/kernel", flush=True)


if __name__ == "__main__":
    main()
