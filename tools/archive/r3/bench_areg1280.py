"""K = 1280 A-in-registers GEMM (CASSMANTLE_AREG_K1280=1, forced cfg 15) vs the planner / table
pick on the level-3 / level-4 projection shapes: error vs the fp32 reference and median us.

    CASSMANTLE_AREG_K1280=1 python tools/bench_areg1280.py
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


for M, N, K, res, ln in [(2048, 1280, 1280, True, False), (2048, 1280, 1280, False, False), (2048, 3840, 1280, False, True),
                         (512, 1280, 1280, True, False), (512, 3840, 1280, False, True)]:
    x = rnd(M, K)
    w = rnd(N, K, scale=K ** -0.5)
    b = rnd(N, scale=0.1)
    r = rnd(M, N) if res else None
    if ln:
        gm = (torch.rand(K, generator=g) + 0.5).to(torch.bfloat16).cuda()
        bt = rnd(K, scale=0.1)
        fold = ops.ln_fold(gm, bt, w, b)
        f = lambda: ops.ln_linear(x, gm, bt, 1e-5, w, fold=fold)
        exp = ref.linear(torch.nn.functional.layer_norm(x.float(), (K,), gm.float(), bt.float(), 1e-5).to(torch.bfloat16), w, b)
    else:
        f = lambda: ops.linear(x, w, b, residual=r)
        exp = ref.linear(x, w, b, residual=r)
    out = {"M": M, "N": N, "K": K, "res": res, "ln": ln}
    for arm, cfg in (("auto", -1), ("areg", 15)):
        ext().gemm_set_override(cfg, 1 if cfg >= 0 else 0)
        y = f()
        torch.cuda.synchronize()
        out[arm + "_plan"] = list(ext().gemm_last_plan())
        out[arm + "_err"] = round(((y.float() - exp.float()).norm() / exp.float().norm()).item(), 5)
        out[arm + "_us"] = round(timeit(f), 2)
        ext().gemm_set_override(-1, 0)
    print(json.dumps(out), flush=True)
