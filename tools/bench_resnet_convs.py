"""The SD-1.5 ResNet 3x3 convolutions at every UNet level, as the UNet calls them (bias, per-image
time-embedding bias, GroupNorm statistics of the output), through the tuned plan; one JSON line per
shape (us per call, median of rounds; the plan).  Used for same-box A/Bs of kernel variants
(tools/gpu/so_ab.sh), e.g. the GroupNorm+SiLU prologue cost probe.

    python tools/bench_resnet_convs.py [--rounds 5] [--iters 20] [--linear]

``--linear``: the transformer projections with a residual epilogue instead (attention / cross
output projections and proj_out at every level, the FF down projection).
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402
from cassmantle_amd.ops._ext import ext  # noqa: E402

LINEAR = [(32768, 320, 320), (32768, 320, 1280), (8192, 640, 640), (8192, 640, 2560), (2048, 1280, 1280),
          (2048, 1280, 5120), (512, 1280, 1280)]
SHAPES = [(8, 64, 320, 320), (8, 64, 640, 320), (8, 32, 640, 640), (8, 32, 1280, 640), (8, 16, 1280, 1280),
          (8, 16, 2560, 1280), (8, 8, 1280, 1280), (8, 8, 2560, 1280)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--linear", action="store_true")
    a = ap.parse_args()
    ops.set_mode("hip")
    g = torch.Generator(device="cuda").manual_seed(0)
    for shape in (LINEAR if a.linear else SHAPES):
        if a.linear:
            M, N, K = shape
            x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
            w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
            b = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
            r = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)

            def f():
                ops.linear(x, w, b, residual=r)
        else:
            B, H, Cin, Cout = shape
            x = torch.randn(B, H, H, Cin, device="cuda", generator=g).to(torch.bfloat16)
            w = (torch.randn(Cout, 3, 3, Cin, device="cuda", generator=g) * (9 * Cin) ** -0.5).to(torch.bfloat16)
            b = torch.randn(Cout, device="cuda", generator=g).to(torch.bfloat16)
            cb = torch.randn(B, Cout, device="cuda", generator=g).to(torch.bfloat16)
            st = ops.new_stats(B, Cout, "cuda")

            def f():
                ops.conv2d(x, w, b, padding=1, chan_bias=cb, stats=st)
        f()
        plan = [int(v) for v in ext().gemm_last_plan()]
        ts = []
        for _ in range(a.rounds):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                f()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / a.iters * 1e3)
        print(json.dumps({"shape": list(shape), "us": round(statistics.median(ts), 2), "plan": plan}), flush=True)


if __name__ == "__main__":
    main()
