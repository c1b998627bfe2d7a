"""Can the next layer's weights be warmed while the current layer runs?  (the
small-grid UNet GEMMs lose 0.81 ms per SD-1.5 eval to cold weights, r5_diag_cold_warm_sd15.txt.)

120 GEMMs of M 2048 x N 1280 x K 1280 (the level-3 projections) on 120 DIFFERENT weights
(400 MB: more than the 256 MB MALL, so every weight is cold when its GEMM runs, as in a UNet
eval), activations warm, captured in one graph and replayed.  Variants:
  cold     : the GEMMs alone
  warm     : 120 GEMMs on ONE weight (the warm ceiling)
  serial   : prefetch(W_i) then GEMM_i on the same stream (prefetch cost + a MALL-warm GEMM)
  pf_only  : the 120 prefetches alone
  branch1  : prefetch(W_{i+1}) on a side stream forked at GEMM_i (graph branch)
  branch2  : same, two GEMMs ahead
  branchm  : branch1 with the side stream CU-masked to 8 CUs (one per XCD)
Prints one JSON line per variant: us per GEMM (graph time / 120).

    python tools/probe_weight_prefetch.py [--blocks 64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402


def timed(g, replays=5):
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(replays):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / replays * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-w", type=int, default=120)
    ap.add_argument("--m", type=int, default=2048)
    ap.add_argument("--n", type=int, default=1280)
    ap.add_argument("--k", type=int, default=1280)
    ap.add_argument("--blocks", default="16,64")
    a = ap.parse_args()
    ops.set_mode("hip")
    ops.load_gemm_tuning()
    dev = torch.device("cuda")
    x = (torch.randn(a.m, a.k, device=dev) * 0.5).to(torch.bfloat16)
    ws = [(torch.randn(a.n, a.k, device=dev) * a.k ** -0.5).to(torch.bfloat16) for _ in range(a.n_w)]
    bias = torch.zeros(a.n, device=dev, dtype=torch.bfloat16)
    outs = [torch.empty(a.m, a.n, device=dev, dtype=torch.bfloat16) for _ in range(2)]
    side = torch.cuda.Stream()
    masked = None
    try:
        from cassmantle_amd.runtime.cumask import masked_stream
        masked = masked_stream(dev, list(range(8)))
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"cumask": f"unavailable: {e}"}), flush=True)

    def gemm(i, w):
        ops.linear(x, w, bias, out=outs[i & 1])

    def capture(body):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body()
        return g

    res = {}

    def run(name, body):
        us = timed(capture(body)) / a.n_w
        res[name] = us
        print(json.dumps({"variant": name, "us_per_gemm": round(us, 2)}), flush=True)

    run("cold", lambda: [gemm(i, ws[i]) for i in range(a.n_w)])
    run("warm", lambda: [gemm(i, ws[0]) for i in range(a.n_w)])
    for blocks in [int(b) for b in a.blocks.split(",")]:
        def serial():
            for i in range(a.n_w):
                ops.prefetch(ws[i], blocks)
                gemm(i, ws[i])
        run(f"serial_b{blocks}", serial)
        run(f"pf_only_b{blocks}", lambda: [ops.prefetch(ws[i], blocks) for i in range(a.n_w)])
        for ahead, stream, tag in ((1, side, "branch1"), (2, side, "branch2"), (1, masked, "branchm")):
            if stream is None:
                continue

            def branch(ahead=ahead, stream=stream):
                cur = torch.cuda.current_stream()
                for i in range(a.n_w):
                    if i + ahead < a.n_w:
                        stream.wait_stream(cur)
                        with torch.cuda.stream(stream):
                            ops.prefetch(ws[i + ahead], blocks)
                    gemm(i, ws[i])
                cur.wait_stream(stream)
            run(f"{tag}_b{blocks}", branch)
    print(json.dumps({"summary": {k: round(v, 2) for k, v in res.items()},
                      "shape": [a.m, a.n, a.k], "weights": a.n_w}), flush=True)


if __name__ == "__main__":
    main()
