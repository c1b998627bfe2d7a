"""LayerNorm-folded GEMM (ops.ln_linear, A-in-registers kernel) under concurrency: the same call
repeated on one stream while a second stream runs background kernels of one family, outputs
compared bit-for-bit with a quiet reference; reports differing runs, max |diff| and rows differing.

    python tools/dbg_lnk_conc.py [modes...]     modes: pp c0 deep conv gn attn areg none
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402
from cassmantle_amd.ops import ext  # noqa: E402

torch.manual_seed(0)
dev = "cuda"
s_bg = torch.cuda.Stream()
bgA = torch.randn(8192, 2048, device=dev).to(torch.bfloat16)
bgW = (torch.randn(2048, 2048, device=dev) * 0.02).to(torch.bfloat16)
bgX = torch.randn(4, 128, 128, 256, device=dev).to(torch.bfloat16)
bgC = (torch.randn(256, 3, 3, 256, device=dev) * 0.02).to(torch.bfloat16)
gnw = torch.ones(256, device=dev, dtype=torch.bfloat16)
gnb = torch.zeros(256, device=dev, dtype=torch.bfloat16)
q = torch.randn(8, 4096, 8, 40, device=dev).to(torch.bfloat16)
lx = (torch.randn(8192, 320, device=dev)).to(torch.bfloat16)
lg = torch.ones(320, device=dev, dtype=torch.bfloat16)
lb = torch.zeros(320, device=dev, dtype=torch.bfloat16)
lw = (torch.randn(960, 320, device=dev) * 0.05).to(torch.bfloat16)
lfold = ops.ln_fold(lg, lb, lw, None)


def background(mode, n):
    cfg = {"pp": 7, "c0": 0, "deep": 13}.get(mode)
    with torch.cuda.stream(s_bg):
        for _ in range(n):
            if cfg is not None:
                ext().gemm_set_override(cfg, 1)
                ops.linear(bgA, bgW)
                ext().gemm_set_override(-1, 0)
            elif mode == "conv":
                ops.conv2d(bgX, bgC, None, 1, 1)
            elif mode == "gn":
                ops.group_norm(bgX, 32, gnw, gnb, 1e-5, silu=True)
            elif mode == "attn":
                ops.attention(q, q, q)
            elif mode == "areg":
                ops.ln_linear(lx, lg, lb, 1e-5, lw, fold=lfold)


modes = sys.argv[1:] or ["none", "pp", "c0", "deep", "conv", "gn", "attn", "areg"]
print("knobs", {k: v for k, v in os.environ.items() if k.startswith("CASSMANTLE_")}, flush=True)
for M, K, N, act in [(8192, 320, 960, None), (8192, 320, 1280, "geglu")]:
    x = (torch.randn(M, K, device=dev) * 2 + 0.5).to(torch.bfloat16)
    g = (torch.rand(K, device=dev) + 0.5).to(torch.bfloat16)
    b = (torch.randn(K, device=dev) * 0.1).to(torch.bfloat16)
    nw = 2 * N if act else N
    w = (torch.randn(nw, K, device=dev) * K ** -0.5).to(torch.bfloat16)
    wb = (torch.randn(nw, device=dev) * 0.1).to(torch.bfloat16)
    fold = ops.ln_fold(g, b, w, wb)
    ref = ops.ln_linear(x, g, b, 1e-5, w, act=act, fold=fold).clone()
    torch.cuda.synchronize()
    for mode in modes:
        outs = []
        background(mode, 30)
        for _ in range(40):
            outs.append(ops.ln_linear(x, g, b, 1e-5, w, act=act, fold=fold))
        torch.cuda.synchronize()
        bad, mx, rows = 0, 0.0, 0
        for y in outs:
            if not torch.equal(y, ref):
                bad += 1
                d = (y.float() - ref.float()).abs()
                mx = max(mx, d.max().item())
                rows = max(rows, int((d.amax(1) > 0).sum()))
        print(f"M {M} K {K} N {N} act {act} bg {mode:5s}: diff {bad}/40, max|d| {mx:.4g}, rows {rows}", flush=True)
