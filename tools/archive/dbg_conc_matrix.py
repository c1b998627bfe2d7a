"""Which kernel corrupts which under two-stream concurrency: victim GEMM families (LN-folded
A-in-registers, plain A-in-registers, 4-wave, ping-pong) repeated on the main stream while an
aggressor family runs on a second stream; outputs compared bit-for-bit with a quiet reference."""
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

M, K, N = 8192, 320, 960
x = (torch.randn(M, K, device=dev) * 2 + 0.5).to(torch.bfloat16)
g = (torch.rand(K, device=dev) + 0.5).to(torch.bfloat16)
b = (torch.randn(K, device=dev) * 0.1).to(torch.bfloat16)
w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
wb = (torch.randn(N, device=dev) * 0.1).to(torch.bfloat16)
fold = ops.ln_fold(g, b, w, wb)
x640 = (torch.randn(M, 640, device=dev)).to(torch.bfloat16)
w640 = (torch.randn(640, 640, device=dev) * 640 ** -0.5).to(torch.bfloat16)


def victim(kind):
    if kind == "ln_areg":
        return ops.ln_linear(x, g, b, 1e-5, w, fold=fold)
    if kind == "areg320":
        ext().gemm_set_override(15, 1)
        try:
            return ops.linear(x, w, wb)
        finally:
            ext().gemm_set_override(-1, 0)
    cfg = {"areg": 15, "c0": 0, "pp": 8, "deep": 14}[kind]
    ext().gemm_set_override(cfg, 1)
    try:
        return ops.linear(x640 if kind == "areg" else x, w640 if kind == "areg" else w, wb[:640] if kind == "areg" else wb)
    finally:
        ext().gemm_set_override(-1, 0)


def aggressor(kind, n):
    if kind == "none":
        return
    cfg = {"c0": 0, "pp": 7, "c3": 3}[kind]
    with torch.cuda.stream(s_bg):
        for _ in range(n):
            ext().gemm_set_override(cfg, 1)
            ops.linear(bgA, bgW)
            ext().gemm_set_override(-1, 0)


for vk in (sys.argv[1:] or ["ln_areg", "areg320", "areg", "c0", "pp", "deep"]):
    ref = victim(vk).clone()
    torch.cuda.synchronize()
    for ak in ["none", "c0"]:
        aggressor(ak, 30)
        outs = [victim(vk) for _ in range(40)]
        torch.cuda.synchronize()
        bad, mx = 0, 0.0
        for y in outs:
            if not torch.equal(y, ref):
                bad += 1
                mx = max(mx, (y.float() - ref.float()).abs().max().item())
        print(f"{os.environ.get('CASSMANTLE_AREG_V', '-')} victim {vk:8s} aggressor {ak:5s}: diff {bad}/40 max|d| {mx:.3g}", flush=True)
