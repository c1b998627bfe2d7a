"""Run-to-run determinism of one SD-1.5 UNet evaluation (batch 8) with the fused GroupNorm
statistics (fp32 atomics: order-dependent rounding) vs the two-pass GroupNorm.

    python tools/dbg_determinism.py
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from cassmantle_amd.models import layers  # noqa: E402
from cassmantle_amd.models.unet import SD15_UNET, UNet  # noqa: E402


def cos(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return (a @ b / (a.norm() * b.norm())).item()


m = UNet(SD15_UNET, seed=0).cuda()
g = torch.Generator().manual_seed(0)
x = torch.randn(8, 64, 64, 4, generator=g).to(torch.bfloat16).cuda()
t = torch.full((8,), 500.0, device="cuda")
ctx = torch.randn(8, 77, 768, generator=g).to(torch.bfloat16).cuda()
out = {}
with torch.no_grad():
    for fuse in (False, True):
        layers._GN_FUSE = fuse
        ys = [m(x, t, ctx).clone() for _ in range(4)]
        out[f"fuse{int(fuse)}"] = {"max_abs_diff_runs": max((ys[0].float() - y.float()).abs().max().item() for y in ys[1:]),
                                   "min_cos_runs": min(cos(ys[0], y) for y in ys[1:]),
                                   "absmax": ys[0].float().abs().max().item()}
        out[f"y{int(fuse)}"] = ys[0]
print(json.dumps({"fuse0": out["fuse0"], "fuse1": out["fuse1"], "cos_fused_vs_twopass": cos(out["y0"], out["y1"])}))
