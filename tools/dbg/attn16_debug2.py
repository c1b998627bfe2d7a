import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from cassmantle_amd import ops
from cassmantle_amd.ops import reference as ref

def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()

ops.set_attention_d40_variant("16x16")
for Nk in (16, 32, 48, 64):
    for dims in [(0, 8), (8, 16), (16, 24), (24, 32), (0, 32), (32, 40)]:
        torch.manual_seed(1)
        q = torch.zeros(1, 32, 1, 40, device="cuda")
        k = torch.zeros(1, Nk, 1, 40, device="cuda")
        q[..., dims[0]:dims[1]] = torch.randn(1, 32, 1, dims[1] - dims[0], device="cuda") * 2
        k[..., dims[0]:dims[1]] = torch.randn(1, Nk, 1, dims[1] - dims[0], device="cuda") * 2
        v = torch.randn(1, Nk, 1, 40, device="cuda")
        q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
        out = ops.attention(q, k, v)
        exp = ref.attention(q, k, v)
        print("Nk", Nk, "dims", dims, "rel", round(rel(out, exp), 4), "q-rows bad:",
              [i for i in range(32) if rel(out[0, i], exp[0, i]) > 0.05][:12])
