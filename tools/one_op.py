"""Run one op shape repeatedly (for rocprofv3 counter collection)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cassmantle_amd import ops
kind = sys.argv[1]
iters = int(os.environ.get("ITERS", "20"))
torch.manual_seed(0)
def rnd(*s, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).to(torch.bfloat16)
with torch.no_grad():
    if kind == "conv":
        B, H, Cin, Cout = [int(v) for v in sys.argv[2:6]]
        x = rnd(B, H, H, Cin); w = rnd(Cout, 3, 3, Cin, scale=(9 * Cin) ** -0.5); b = rnd(Cout)
        f = lambda: ops.conv2d(x, w, b)
    elif kind == "gemm":
        M, N, K = [int(v) for v in sys.argv[2:5]]
        x = rnd(M, K); w = rnd(N, K, scale=K ** -0.5); b = rnd(N)
        f = lambda: ops.linear(x, w, b)
    elif kind == "attn":
        B, N, H, d = [int(v) for v in sys.argv[2:6]]
        q, k, v = rnd(B, N, H, d), rnd(B, N, H, d), rnd(B, N, H, d)
        f = lambda: ops.attention(q, k, v)
    elif kind == "attn8":
        B, N, H, d = [int(v) for v in sys.argv[2:6]]
        q, k, v = rnd(B, N, H, d), rnd(B, N, H, d), rnd(B, N, H, d)
        f = lambda: ops.attention(q, k, v, fp8="force")
    elif kind == "lngeglu":   # LayerNorm-folded GEGLU projection (A-in-registers kernel)
        M, N, K = [int(v) for v in sys.argv[2:5]]
        x = rnd(M, K); g = (torch.rand(K, device="cuda") + 0.5).to(torch.bfloat16); bt = rnd(K, scale=0.1)
        w = rnd(2 * N, K, scale=K ** -0.5); b = rnd(2 * N, scale=0.1)
        fold = ops.ln_fold(g, bt, w, b)
        f = lambda: ops.ln_linear(x, g, bt, 1e-5, w, act="geglu", fold=fold)
    for _ in range(iters):
        f()
    torch.cuda.synchronize()
print("ok")
