"""Register-staged GEMM tiles (cfg 17/18/19) vs the table / planner pick on the SD-1.5 shapes:
error vs the fp32 reference and median us per arm (forced plans through gemm_set_override).

    python tools/bench_regstage.py
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402
from cassmantle_amd.ops import reference as ref  # noqa: E402
from cassmantle_amd.ops._ext import ext  # noqa: E402

ops.load_gemm_tuning()
g = torch.Generator().manual_seed(0)


def rnd(*s, scale=1.0):
    return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).cuda()


def timeit(f, iters=30):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters * 1e3)
    return statistics.median(ts)


cases = []
for M, N, K, res in [(2048, 1280, 1280, True), (2048, 1280, 1280, False), (512, 1280, 1280, True), (8192, 640, 640, True),
                     (32768, 320, 320, True), (2048, 1280, 5120, True), (8192, 640, 2560, True), (32768, 320, 1280, True)]:
    x, w, b = rnd(M, K), rnd(N, K, scale=K ** -0.5), rnd(N, scale=0.1)
    r = rnd(M, N) if res else None
    cases.append((f"linear m{M} n{N} k{K} r{int(res)}", (lambda x=x, w=w, b=b, r=r: ops.linear(x, w, b, residual=r)),
                  ref.linear(x, w, b, residual=r)))
for B, H, Cin, Cout in [(8, 64, 320, 320), (8, 32, 640, 640), (8, 16, 1280, 1280), (8, 8, 1280, 1280)]:
    x = rnd(B, H, H, Cin)
    w = rnd(Cout, 3, 3, Cin, scale=(9 * Cin) ** -0.5)
    b = rnd(Cout, scale=0.1)
    cases.append((f"conv b{B} h{H} ci{Cin} co{Cout}", (lambda x=x, w=w, b=b: ops.conv2d(x, w, b, 1, 1)),
                  ref.conv2d(x, w, b, 1, 1)))
for name, f, exp in cases:
    out = {"case": name}
    for arm, cfg, sp in (("auto", -1, 0), ("r17", 17, 1), ("r18", 18, 1), ("r19", 19, 1), ("r17s2", 17, 2), ("r18s2", 18, 2)):
        ext().gemm_set_override(cfg, sp)
        y = f()
        torch.cuda.synchronize()
        out[arm] = [round(timeit(f), 2), list(ext().gemm_last_plan()),
                    round(((y.float() - exp.float()).norm() / exp.float().norm()).item(), 4)]
        ext().gemm_set_override(-1, 0)
    print(json.dumps(out), flush=True)
