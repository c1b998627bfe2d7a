"""Achieved HBM bandwidth of the memory-bound UNet passes (verdict r2 item 8):

* gn_apply_cs_kernel -- GroupNorm(+SiLU) apply from producer statistics (read x, write y);
  timed with events here;
* splitk_reduce_stats_kernel -- the split-K second pass of the 16^2 / 8^2 convolutions (read
  split fp32 slabs, write bf16, per-channel statistics); its time comes from a rocprofv3 kernel
  trace of this script: run it under ``rocprofv3 --kernel-trace`` and pass the trace to
  ``--trace`` afterwards (matched by the reduce kernel's grid).

    rocprofv3 --kernel-trace -d gpurun_out/membound -o run --output-format csv -- python tools/bench_membound.py
    python tools/bench_membound.py --trace gpurun_out/membound/.../run_kernel_trace.csv
"""
import argparse
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GN_SHAPES = [(8, 64, 64, 320), (8, 64, 64, 640), (8, 64, 64, 960), (8, 32, 32, 640), (8, 32, 32, 1280),
             (8, 16, 16, 1280), (8, 16, 16, 2560), (8, 8, 8, 2560)]
# SD-1.5 convolutions that split K (batch 4 x CFG): NHWC input, Cin -> Cout, 3x3
CONV_SHAPES = [(8, 16, 16, 1280, 1280), (8, 16, 16, 2560, 1280), (8, 8, 8, 1280, 1280), (8, 8, 8, 2560, 1280)]
# SDXL (batch 1 x CFG) GroupNorm applies: 128^2 / 64^2 / 32^2 levels incl. the up-block concat widths
SDXL_GN_SHAPES = [(2, 128, 128, 320), (2, 128, 128, 640), (2, 128, 128, 960), (2, 64, 64, 640),
                  (2, 64, 64, 1280), (2, 64, 64, 1920), (2, 32, 32, 1280), (2, 32, 32, 2560)]
# SD VAE decoder GroupNorm applies at the bench's batch 4 (512^2 output: 64^2 .. 512^2 levels)
VAE_GN_SHAPES = [(4, 64, 64, 512), (4, 128, 128, 512), (4, 256, 256, 512), (4, 256, 256, 256),
                 (4, 512, 512, 256), (4, 512, 512, 128)]
ITERS = 30


def run(gn_only: bool = False, shapes=GN_SHAPES):
    import torch
    from cassmantle_amd import ops
    from cassmantle_amd.ops._ext import ext
    for shape in shapes:
        x = (torch.randn(*shape, device="cuda") + 0.3).to(torch.bfloat16)
        C = shape[-1]
        st = ops.new_stats(shape[0], C, "cuda")
        ops.channel_stats(x, st)
        g = torch.ones(C, device="cuda", dtype=torch.bfloat16)
        b = torch.zeros(C, device="cuda", dtype=torch.bfloat16)

        def f():
            return ops.group_norm(x, 32, g, b, 1e-5, True, stats=st)
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(ITERS):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / ITERS * 1e3
        nbytes = 2 * x.numel() * 2
        print(json.dumps({"kernel": "gn_apply_cs", "shape": list(shape), "us": round(us, 2), "bytes": nbytes,
                          "TBps": round(nbytes / us / 1e6, 2)}), flush=True)
    for B, H, W, Cin, Cout in ([] if gn_only else CONV_SHAPES):
        x = (torch.randn(B, H, W, Cin, device="cuda") * 0.5).to(torch.bfloat16)
        w = (torch.randn(Cout, 3, 3, Cin, device="cuda") * (9 * Cin) ** -0.5).to(torch.bfloat16)
        st = ops.new_stats(B, Cout, "cuda")
        ops.conv2d(x, w, None, padding=1, stats=st)
        cfg, split = (int(v) for v in ext().gemm_last_plan())
        for _ in range(ITERS):
            ops.zero_(st)
            ops.conv2d(x, w, None, padding=1, stats=st)
        torch.cuda.synchronize()
        M, N = B * H * W, Cout
        grid_x = ((N // 4 + 15) // 16) * 256
        nbytes = split * M * N * 4 + M * N * 2
        print(json.dumps({"kernel": "splitk_reduce_stats", "conv": [B, H, W, Cin, Cout], "M": M, "N": N,
                          "split": split, "cfg": cfg, "grid": [grid_x, (M + 63) // 64], "bytes": nbytes}), flush=True)


def from_trace(path, lines):
    rows = list(csv.DictReader(open(path)))
    dur = collections.defaultdict(list)
    for r in rows:
        if "splitk_reduce_stats_kernel" in r["Kernel_Name"]:
            dur[(int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]))].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for ln in lines:
        if ln.get("kernel") != "splitk_reduce_stats" or ln["split"] <= 1:
            continue
        d = sorted(dur.get(tuple(ln["grid"]), []))
        if not d:
            continue
        med = d[len(d) // 2]
        ln["us"] = round(med, 2)
        ln["TBps"] = round(ln["bytes"] / med / 1e6, 2)
        print(json.dumps(ln))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", default=None, help="rocprofv3 kernel trace of a previous run")
    ap.add_argument("--lines", default=None, help="that run's JSON output (for --trace)")
    ap.add_argument("--gn-only", action="store_true", help="only the GroupNorm applies")
    ap.add_argument("--sdxl", action="store_true", help="the SDXL GroupNorm shapes (implies --gn-only)")
    ap.add_argument("--vae", action="store_true", help="the SD VAE decoder GroupNorm shapes (implies --gn-only)")
    a = ap.parse_args()
    if a.trace:
        from_trace(a.trace, [json.loads(x) for x in open(a.lines) if x.startswith("{")])
    else:
        run(a.gn_only or a.sdxl or a.vae, SDXL_GN_SHAPES if a.sdxl else (VAE_GN_SHAPES if a.vae else GN_SHAPES))
