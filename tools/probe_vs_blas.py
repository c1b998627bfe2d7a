"""Speed-of-light check of the in-tree GEMM against the vendor library on the UNet's GEMM shapes:
y = x @ w^T (bf16 in, bf16 out, fp32 accumulate) as graph-replayed back-to-back launches, the
in-tree kernel on its tuned plan (``ops.linear``) next to ``torch.matmul`` (hipBLASLt), both on
rotating weight / activation copies.  Measurement only: the vendor GEMM is never on a serving path.

    python tools/probe_vs_blas.py [--shapes 2048x1280x1280,...]
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

SHAPES = ("2048x1280x1280,2048x1280x5120,2048x10240x1280,2048x3840x1280,8192x640x640,8192x5120x640,"
          "32768x320x320,32768x2560x320,32768x960x320,8192x1280x640,4096x4096x4096,16384x8192x4096")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=SHAPES, help="MxNxK list")
    ap.add_argument("--rotate", type=int, default=4)
    ap.add_argument("--cfgs", default="", help="also time the in-tree kernel forced to these cfg[:split] plans")
    a = ap.parse_args()
    ops.set_mode("hip")
    ops.load_gemm_tuning()
    for s in a.shapes.split(","):
        M, N, K = (int(v) for v in s.split("x"))
        rot = a.rotate if M * K + N * K < (1 << 27) else 1
        xs = [(torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16) for _ in range(rot)]
        ws = [(torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16) for _ in range(rot)]
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        cnt = [0]

        def ours():
            i = cnt[0] % rot
            cnt[0] += 1
            ops.linear(xs[i], ws[i], out=out)

        def blas():
            i = cnt[0] % rot
            cnt[0] += 1
            torch.matmul(xs[i], ws[i].t(), out=out)
        flop = 2.0 * M * N * K
        reps = max(2, min(40, int(2e11 / flop)))
        t_ours = graph_time(ours, reps=reps, replays=5)
        t_blas = graph_time(blas, reps=reps, replays=5)
        y0 = ops.linear(xs[0], ws[0])
        y1 = torch.matmul(xs[0], ws[0].t())
        err = float((y0.float() - y1.float()).abs().max())
        for cs in [c for c in a.cfgs.split(",") if c]:
            cfg, _, sp = cs.partition(":")
            ext().gemm_set_override(int(cfg), int(sp or 1))
            try:
                t_c = graph_time(ours, reps=reps, replays=5)
                print(json.dumps({"shape": s, "cfg": cs, "us": round(t_c, 2), "tf": round(flop / t_c * 1e-6, 1)}), flush=True)
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"shape": s, "cfg": cs, "error": str(e)[:160]}), flush=True)
            ext().gemm_set_override(-1, 0)
        print(json.dumps({"shape": s, "ours_us": round(t_ours, 2), "blas_us": round(t_blas, 2),
                          "ours_tf": round(flop / t_ours * 1e-6, 1), "blas_tf": round(flop / t_blas * 1e-6, 1),
                          "ratio": round(t_ours / t_blas, 3), "max_abs_diff": err}), flush=True)


if __name__ == "__main__":
    main()
