"""Run-to-run determinism of the LayerNorm-folded GEMM (ops.ln_linear) on synthetic rows,
K = 320 and 640, plain and GEGLU (the A-in-registers kernel's in-kernel LayerNorm).

    python tools/dbg_det_lnk.py
"""
import sys

import torch

sys.path.insert(0, ".")
from cassmantle_amd import ops  # noqa: E402

torch.manual_seed(0)
for M, K, N, act in [(2048, 640, 1920, None), (8192, 320, 960, None), (8192, 640, 640, None),
                     (2048, 640, 2560, "geglu"), (8192, 320, 1280, "geglu")]:
    x = (torch.randn(M, K, device="cuda") * 2 + 0.5).to(torch.bfloat16)
    g = (torch.rand(K, device="cuda") + 0.5).to(torch.bfloat16)
    b = (torch.randn(K, device="cuda") * 0.1).to(torch.bfloat16)
    nw = 2 * N if act else N
    w = (torch.randn(nw, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    wb = (torch.randn(nw, device="cuda") * 0.1).to(torch.bfloat16)
    fold = ops.ln_fold(g, b, w, wb)
    ref = ops.ln_linear(x, g, b, 1e-5, w, act=act, fold=fold).clone()
    bad = 0
    for _ in range(30):
        y = ops.ln_linear(x, g, b, 1e-5, w, act=act, fold=fold)
        bad += int(not torch.equal(y, ref))
    torch.cuda.synchronize()
    print(f"M {M} K {K} N {N} act {act}: differing runs {bad}/30", flush=True)
