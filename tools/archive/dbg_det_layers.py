"""Find the first UNet module whose output differs between two identical evaluations
(run-to-run determinism bisect; the inputs of tests/test_models_gpu.py's determinism test).

    python tools/dbg_det_layers.py
"""
import sys

import torch

sys.path.insert(0, ".")
from cassmantle_amd.models.unet import SD15_UNET, UNet  # noqa: E402

m = UNet(SD15_UNET, seed=1).cuda()
g = torch.Generator().manual_seed(2)
x = torch.randn(8, 32, 32, 4, generator=g).to(torch.bfloat16).cuda()
t = torch.full((8,), 700.0, device="cuda")
ctx = torch.randn(8, 77, 768, generator=g).to(torch.bfloat16).cuda()
rec = [[], []]
cur = {"i": 0}


def hook(name):
    def f(mod, inp, out):
        o = out[0] if isinstance(out, tuple) else out
        if torch.is_tensor(o):
            torch.cuda.synchronize()
            rec[cur["i"]].append((name, o.detach().clone()))
    return f


for n, mod in m.named_modules():
    if n:
        mod.register_forward_hook(hook(n))
with torch.no_grad():
    for i in range(2):
        cur["i"] = i
        y = m(x, t, ctx)
        torch.cuda.synchronize()
shown = 0
for (n0, a), (n1, b) in zip(rec[0], rec[1]):
    same = a.shape == b.shape and torch.equal(a, b)
    if not same:
        d = (a.float() - b.float()).abs()
        print(f"DIFF {n0:60s} {tuple(a.shape)} maxdiff {d.max().item():.3e} n_diff {(d > 0).sum().item()}")
        shown += 1
        if shown >= 12:
            break
print("modules recorded", len(rec[0]), len(rec[1]), "first-diff shown", shown)
