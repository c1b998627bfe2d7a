"""Characterise the rows the LN-folded GEMM gets wrong under two-stream concurrency: for every
differing row fit y - b' = a * (x @ Wf^T) + c * wsum by least squares.  A pure LayerNorm-statistics
error leaves a tiny residual (a = rstd', c = -rstd' * mean'); anything else (wrong A values,
wrong W tile) does not."""
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
wf, wsum, bf = fold
ref = ops.ln_linear(x, g, b, 1e-5, w, fold=fold).clone()
xf = x.float()
mu = xf.mean(1)
rstd = torch.rsqrt(xf.var(1, unbiased=False) + 1e-5)
P = xf @ wf.float().t()                      # [M, N]
shown = 0
for it in range(int(os.environ.get("ITERS", "12"))):
    with torch.cuda.stream(s_bg):
        for _ in range(30):
            ext().gemm_set_override(0, 1)
            ops.linear(bgA, bgW)
            ext().gemm_set_override(-1, 0)
    outs = [ops.ln_linear(x, g, b, 1e-5, w, fold=fold) for _ in range(40)]
    torch.cuda.synchronize()
    for y in outs:
        if torch.equal(y, ref):
            continue
        d = (y.float() - ref.float()).abs().amax(1)
        rows = torch.nonzero(d > 0).flatten().tolist()
        groups = sorted({r // 16 for r in rows})
        print(f"iter {it}: {len(rows)} rows differ, 16-row groups {groups[:8]} (block {[q // 8 for q in groups[:8]]}, "
              f"wave {[(q % 8) // 2 for q in groups[:8]]}, j {[q % 2 for q in groups[:8]]})", flush=True)
        for r in rows[:4]:
            yb = y[r].float() - bf.float()
            A = torch.stack([P[r], wsum.float()], 1)
            sol = torch.linalg.lstsq(A.cpu(), yb.cpu().unsqueeze(1)).solution.flatten()
            res = (A.cpu() @ sol - yb.cpu()).norm() / yb.norm().cpu()
            a, c = sol.tolist()
            print(f"   row {r}: rstd' {a:.5f} (true {rstd[r].item():.5f}) mean' {-c / a:.5f} "
                  f"(true {mu[r].item():.5f}) rel.residual {res.item():.2e} maxdiff {d[r].item():.3g}", flush=True)
        shown += 1
        if shown >= 6:
            sys.exit(0)
print("done")
