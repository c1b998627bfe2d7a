"""Weight-streaming GEMMs with cold weights: time a linear layer whose weight comes from HBM on
every call (as in a UNet evaluation, which reads each of its ~1.7 GB (SD-1.5) / ~5 GB (SDXL) of
weights once) against the same layer re-run on one L2 / MALL-resident weight (what the in-situ
autotuner measures).  Each cold call uses the next of R weight copies, R x |W| >= 512 MiB (twice
the 256 MiB Infinity Cache); the activations stay the same tensor (warm), as in the pipeline.

    python tools/cold_weight_probe.py [--arms 26:1,31:1,34:1] [--shapes 2048x1280x1280,...]

Prints one JSON line per (shape, arm): warm_us, cold_us.
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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="2048x1280x1280,2048x1280x5120,8192x640x640,2048x640x1280,8192x640x2560")
    ap.add_argument("--arms", default="3:1,26:1,27:1,31:1,32:1,34:1,35:1,31:2,14:1,33:1,20:1")
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--mib", type=int, default=512)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for sh in a.shapes.split(","):
        M, N, K = (int(v) for v in sh.split("x"))
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        r = (torch.randn(M, N, device=dev) * 0.5).to(torch.bfloat16)
        wbytes = N * K * 2
        R = max(2, min(1024, (a.mib << 20) // wbytes + 1))
        ws = [(torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16) for _ in range(R)]
        b = torch.zeros(N, device=dev, dtype=torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for arm in a.arms.split(","):
            cfg, split = (int(v) for v in arm.split(":"))
            ext().gemm_set_override(cfg, split)
            try:
                res = {}
                for mode in ("warm", "cold"):
                    for i in range(min(R, 8)):                    # plan / first-launch warm-up
                        ops.linear(x, ws[i], b, residual=r, out=out)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for i in range(a.iters):
                        ops.linear(x, ws[(i % R) if mode == "cold" else 0], b, residual=r, out=out)
                    e1.record()
                    torch.cuda.synchronize()
                    res[mode] = e0.elapsed_time(e1) * 1e3 / a.iters
                plan = list(ext().gemm_last_plan())
            finally:
                ext().gemm_set_override(-1, 0)
            print(json.dumps({"shape": [M, N, K], "arm": [cfg, split], "plan": plan, "copies": R,
                              "warm_us": round(res["warm"], 2), "cold_us": round(res["cold"], 2)}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
