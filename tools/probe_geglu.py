"""Where does the level-3 GEGLU projection lose its time?  SDXL's feed-forward input GEMM
(M 2048 x N 2 x 5120 x K 1280, h * gelu(g)) runs at ~72 us = 740 TF/s on the gated 256x160 tile
(8 waves stacked on M) while the same tile family reaches 1.0-1.25 PF/s on plain large-M GEMMs.
This times, as graph-replayed back-to-back launches, the gated call next to the plain GEMM of
the same total width (N 10240, no activation / exact GELU epilogue) and the half-width plain
GEMM (N 5120), for each candidate tile, so the gating cost and the tile's own mainloop separate.

    python tools/probe_geglu.py [--m 2048 --k 1280 --n 5120]
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
from tools.probe_small_gemm import graph_time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=2048)
    ap.add_argument("--k", type=int, default=1280)
    ap.add_argument("--n", type=int, default=5120, help="gated output width (weight rows = 2n)")
    ap.add_argument("--cfgs", default="8,9,12,33,-1")
    ap.add_argument("--rotate", type=int, default=8)
    a = ap.parse_args()
    ops.set_mode("hip")
    ops.load_gemm_tuning()
    ext().gemm_record_keys(True)
    M, K, N = a.m, a.k, a.n
    xs = [(torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16) for _ in range(a.rotate)]
    ws = [(torch.randn(2 * N, K, device="cuda") * K ** -0.5).to(torch.bfloat16) for _ in range(a.rotate)]
    b = torch.randn(2 * N, device="cuda").to(torch.bfloat16) * 0.1
    out_g = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    out_p = torch.empty(M, 2 * N, device="cuda", dtype=torch.bfloat16)
    out_h = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    flop_full = 2.0 * M * 2 * N * K
    cases = {
        "gated": (lambda i: ops.linear(xs[i], ws[i], b, act="geglu", out=out_g), flop_full),
        "plain_2n": (lambda i: ops.linear(xs[i], ws[i], b, out=out_p), flop_full),
        "gelu_2n": (lambda i: ops.linear(xs[i], ws[i], b, act="gelu", out=out_p), flop_full),
        "plain_n": (lambda i: ops.linear(xs[i], ws[i][:N], b[:N], out=out_h), flop_full / 2),
    }
    # reference check of the gated output once (tuned plan)
    ext().gemm_set_override(-1, 0)
    y = ops.linear(xs[0], ws[0], b, act="geglu")
    hg = xs[0].float() @ ws[0].float().t() + b.float()
    ref = hg[:, :N] * torch.nn.functional.gelu(hg[:, N:])
    print(json.dumps({"check": "gated vs fp32", "max_abs": float((y.float() - ref).abs().max()),
                      "ref_max": float(ref.abs().max())}), flush=True)
    for cfg in [int(c) for c in a.cfgs.split(",")]:
        for name, (fn, flop) in cases.items():
            ext().gemm_set_override(cfg, 1 if cfg >= 0 else 0)
            cnt = [0]

            def call():
                fn(cnt[0] % a.rotate)
                cnt[0] += 1
            try:
                us = graph_time(call, reps=2 * a.rotate, replays=5)
                ops.linear(xs[0], ws[0], b, act="geglu" if name == "gated" else None)
                key = ext().gemm_last_key()
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"cfg": cfg, "case": name, "error": str(e)[:200]}), flush=True)
                continue
            print(json.dumps({"cfg": cfg, "case": name, "us": round(us, 2),
                              "tflops": round(flop / us * 1e-6, 1), "key": key}), flush=True)
    ext().gemm_set_override(-1, 0)


if __name__ == "__main__":
    main()
