"""Fixed vs per-tile cost of the attention kernels on the short SDXL / SD-1.5 grids: the same
(B, Nq, H, d) timed at growing key counts, graph-replayed back to back, so the intercept (launch,
prologue, epilogue) and the slope (per 64-key tile) separate.

    python tools/probe_attn_overhead.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402
from tools.probe_small_gemm import graph_time  # noqa: E402

CASES = [  # name, B, Nq, H, d, fp8
    ("sdxl_l3_fp8", 2, 1024, 20, 64, True),
    ("sdxl_l3_bf16", 2, 1024, 20, 64, False),
    ("sd15_l3_b8", 8, 256, 8, 160, False),
    ("sd15_l2_b8", 8, 1024, 8, 80, False),
    ("sd15_l1_b2", 2, 4096, 8, 40, False),
    ("sd15_l3_b2", 2, 256, 8, 160, False),
    ("sd15_l2_b2", 2, 1024, 8, 80, False),
]


def main():
    ops.set_mode("hip")
    for name, B, Nq, H, d, fp8 in CASES:
        for Nk in (64, 256, 1024, 4096):
            if Nk > 4 * Nq and Nk > 256:
                continue
            g = torch.Generator(device="cuda").manual_seed(0)
            q = torch.randn(B, Nq, H, d, device="cuda", generator=g).to(torch.bfloat16)
            k = torch.randn(B, Nk, H, d, device="cuda", generator=g).to(torch.bfloat16)
            v = torch.randn(B, Nk, H, d, device="cuda", generator=g).to(torch.bfloat16)
            out = torch.empty_like(q)
            if fp8:
                kv8 = ops.pack_kv_fp8(k, v)
                fn = lambda: ops.attention(q, k, v, fp8=True, kv8=kv8)  # noqa: E731
            else:
                fn = lambda: ops.attention(q, k, v)  # noqa: E731
            us = graph_time(fn, reps=20, replays=5)
            print(json.dumps({"case": name, "B": B, "Nq": Nq, "H": H, "d": d, "Nk": Nk, "us": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
