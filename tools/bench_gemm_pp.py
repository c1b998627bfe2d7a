"""A/B of the ping-pong 8-wave GEMM (ops/csrc/gemm_pp.h, configs 7-10) against the 4-wave
kernel's planner pick and stock PyTorch (hipBLASLt / MIOpen) at the SD-1.5 batch-8 shapes.
Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24); one JSON line per
shape with the median over rounds of every arm.

    python tools/bench_gemm_pp.py [--rounds 3] [--iters 20] [--only conv,gemm]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402
from cassmantle_amd.ops import reference as ref  # noqa: E402
from cassmantle_amd.ops._ext import ext  # noqa: E402


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def rnd(*s, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).to(torch.bfloat16)


def cases(only):
    if "conv" in only:
        for B, H, Cin, Cout, st in [(8, 64, 320, 320, 1), (8, 64, 640, 320, 1), (8, 32, 640, 640, 1),
                                    (8, 32, 1280, 640, 1), (8, 16, 1280, 1280, 1), (8, 64, 320, 320, 2)]:
            x = rnd(B, H, H, Cin)
            w = rnd(Cout, 3, 3, Cin, scale=(9 * Cin) ** -0.5)
            b = rnd(Cout, scale=0.1)
            Ho = H // st
            fl = 2.0 * B * Ho * Ho * Cout * 9 * Cin
            wt = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            xt = x.permute(0, 3, 1, 2)

            def tfn(xt=xt, wt=wt, b=b, st=st):
                return F.conv2d(xt, wt, b, stride=st, padding=1)
            yield (f"conv{H}_{Cin}->{Cout}_s{st}", fl, lambda x=x, w=w, b=b, st=st: ops.conv2d(x, w, b, stride=st, padding=1),
                   tfn, lambda x=x, w=w, b=b, st=st: ref.conv2d(x[:1], w, b, st, 1))
        for B, H, C in [(8, 32, 640), (8, 16, 1280)]:
            x = rnd(B, H, H, C)
            w = rnd(C, 3, 3, C, scale=(9 * C) ** -0.5)
            w4 = ops.fold_upsample_weights(w)
            fl = 2.0 * B * 4 * H * H * C * 4 * C
            yield (f"up2conv{H}_{C}", fl, lambda x=x, w=w, w4=w4: ops.conv2d_up2(x, w, w4), None,
                   lambda x=x, w=w: ref.conv2d(x[:1], w, None, 1, 1, None, True))
    if "epi" in only:
        # the in-situ epilogues: GroupNorm statistics + per-image bias (+ residual)
        B, H, C = 8, 64, 320
        x = rnd(B, H, H, C)
        w = rnd(C, 3, 3, C, scale=(9 * C) ** -0.5)
        b, cb, res = rnd(C, scale=0.1), rnd(B, C, scale=0.1), rnd(B, H, H, C)
        st = ops.new_stats(B, C, "cuda")
        fl = 2.0 * B * H * H * C * 9 * C
        yield ("conv64_320_stats_cb", fl, lambda: ops.conv2d(x, w, b, chan_bias=cb, stats=st.zero_()), None,
               lambda: ref.conv2d(x[:1], w, b, 1, 1, None, False, cb[:1]))
        yield ("conv64_320_stats_cb_res", fl, lambda: ops.conv2d(x, w, b, residual=res, chan_bias=cb, stats=st.zero_()),
               None, lambda: ref.conv2d(x[:1], w, b, 1, 1, res[:1], False, cb[:1]))
        x2 = rnd(8, 1024, 640)
        w2 = rnd(640, 640, scale=640 ** -0.5)
        b2, r2 = rnd(640, scale=0.1), rnd(8, 1024, 640)
        st2 = ops.new_stats(8, 640, "cuda")
        yield ("gemm8192x640x640_stats_res", 2.0 * 8192 * 640 * 640,
               lambda: ops.linear(x2, w2, b2, residual=r2, stats=st2.zero_()), None,
               lambda: ref.linear(x2[:1], w2, b2, residual=r2[:1]))
    if "gemm" in only:
        for M, N, K, act in [(32768, 320, 320, None), (32768, 960, 320, None), (32768, 320, 1280, None),
                             (32768, 1280, 320, "geglu"), (8192, 640, 640, None), (8192, 1920, 640, None),
                             (8192, 640, 2560, None), (8192, 2560, 640, "geglu"), (2048, 1280, 1280, None),
                             (4096, 4096, 4096, None), (8192, 8192, 8192, None)]:
            x = rnd(M, K)
            w = rnd(2 * N if act else N, K, scale=K ** -0.5)
            b = rnd(w.shape[0], scale=0.1)

            def tfn(x=x, w=w, b=b, act=act):
                y = F.linear(x, w, b)
                if act:
                    h, g = y.chunk(2, -1)
                    y = h * F.gelu(g)
                return y
            yield (f"gemm{M}x{N}x{K}{'_' + act if act else ''}", 2.0 * M * w.shape[0] * K,
                   lambda x=x, w=w, b=b, act=act: ops.linear(x, w, b, act=act), tfn,
                   lambda x=x, w=w, b=b, act=act: ref.linear(x[:512], w, b, act=act))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="conv,gemm")
    ap.add_argument("--splits", default="1,2,4")
    a = ap.parse_args()
    ops.set_mode("hip")
    splits = [int(s) for s in a.splits.split(",")]
    arms = [("auto", -1, 0)] + [(f"pp{c}/{s}", c, s) for c in (7, 8, 9, 10) for s in splits]
    with torch.no_grad():
        for name, fl, fn, tfn, reffn in cases(a.only.split(",")):
            # numerics of every arm on the leading rows vs the fp32 reference
            errs = {}
            exp = reffn().float()
            for arm, c, s in arms:
                ext().gemm_set_override(c, s)
                y = fn().float()
                y = y.reshape(-1, y.shape[-1])[: exp.reshape(-1, exp.shape[-1]).shape[0]]
                e = exp.reshape(-1, exp.shape[-1])
                errs[arm] = round(((y - e).norm() / e.norm()).item(), 5)
            res = {k: [] for k, _, _ in arms}
            res["torch"] = []
            for _ in range(a.rounds):
                for arm, c, s in arms:
                    ext().gemm_set_override(c, s)
                    res[arm].append(timeit(fn, a.iters))
                ext().gemm_set_override(-1, 0)
                if tfn is not None:
                    res["torch"].append(timeit(tfn, a.iters))
            ext().gemm_set_override(-1, 0)
            med = {k: round(statistics.median(v), 1) for k, v in res.items() if v}
            best = min((k for k in med if k.startswith("pp")), key=med.get)
            out = {"shape": name, "auto_us": med["auto"], "best_pp": best, "best_pp_us": med[best],
                   "torch_us": med.get("torch"), "speedup_vs_auto": round(med["auto"] / med[best], 3),
                   "best_pp_tflops": round(fl / med[best] / 1e6, 1), "auto_tflops": round(fl / med["auto"] / 1e6, 1),
                   "max_err": max(errs.values()), "table": med, "errs": errs}
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
