"""Debug the 16x16-block d=40 attention: zero out parts of Q/K/V and compare with the reference."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from cassmantle_amd import ops
from cassmantle_amd.ops import reference as ref

def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()

torch.manual_seed(0)
B, N, H, d = 1, 64, 1, 40
for name, qm, km, vm in [("full", None, None, None), ("qk_d<32", slice(32, 40), slice(32, 40), None),
                         ("qk_d>=32only", slice(0, 32), slice(0, 32), None), ("q=0", "zero", None, None),
                         ("v_d<16", None, None, slice(16, 40))]:
    q = torch.randn(B, N, H, d, device="cuda").to(torch.bfloat16)
    k = torch.randn(B, N, H, d, device="cuda").to(torch.bfloat16)
    v = torch.randn(B, N, H, d, device="cuda").to(torch.bfloat16)
    if qm == "zero":
        q.zero_()
    elif qm is not None:
        q[..., qm] = 0
    if km is not None:
        k[..., km] = 0
    if vm is not None:
        v[..., vm] = 0
    for var in ("16x16", "32x32"):
        ops.set_attention_d40_variant(var)
        out = ops.attention(q, k, v)
        exp = ref.attention(q, k, v)
        print(name, var, "rel", round(rel(out, exp), 4), "per-d err", [round(x, 3) for x in ((out.float() - exp.float()).abs().mean((0, 1, 2))).tolist()[:40:4]])
    ops.set_attention_d40_variant(None)
# P check: V = one-hot keys -> output = P itself (N keys = 40 -> keys map to dims)
N = 40
q = torch.randn(1, 16, 1, 40, device="cuda").to(torch.bfloat16)
k = torch.randn(1, N, 1, 40, device="cuda").to(torch.bfloat16)
v = torch.eye(40, device="cuda").to(torch.bfloat16).view(1, N, 1, 40)
ops.set_attention_d40_variant("16x16")
out = ops.attention(q, k, v)
exp = ref.attention(q, k, v)
print("P as output: rel", rel(out, exp))
print("row0 out", [round(x, 3) for x in out[0, 0, 0].float().tolist()])
print("row0 exp", [round(x, 3) for x in exp[0, 0, 0].float().tolist()])
