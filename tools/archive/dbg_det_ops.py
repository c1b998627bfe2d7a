"""Op-level run-to-run determinism at one transformer block (the block where
tools/dbg_det_layers.py saw the first difference): LayerNorm-folded QKV GEMM, attention and the
output projection, each repeated on identical inputs.

    python tools/dbg_det_ops.py [block-name]
"""
import sys

import torch

sys.path.insert(0, ".")
from cassmantle_amd import ops  # noqa: E402
from cassmantle_amd.models.unet import SD15_UNET, UNet  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "up.2.attentions.1.transformer_blocks.0"
m = UNet(SD15_UNET, seed=1).cuda()
g = torch.Generator().manual_seed(2)
x = torch.randn(8, 32, 32, 4, generator=g).to(torch.bfloat16).cuda()
t = torch.full((8,), 700.0, device="cuda")
ctx = torch.randn(8, 77, 768, generator=g).to(torch.bfloat16).cuda()
blk = dict(m.named_modules())[name]
cap = {}


def pre(mod, args):
    cap.setdefault("x", args[0].detach().clone())


blk.register_forward_pre_hook(pre)
with torch.no_grad():
    m(x, t, ctx)
    xb = cap["x"]
    f = blk.folds()
    n1 = blk.norm1
    print("block input", tuple(xb.shape))

    def rep(label, fn, n=30):
        ref = fn().clone()
        bad = 0
        for _ in range(n):
            y = fn()
            if not torch.equal(y, ref):
                bad += 1
        torch.cuda.synchronize()
        print(f"{label:40s} shape {tuple(ref.shape)} runs {n} differing {bad}", flush=True)
        return ref

    qkv = rep("ln_linear qkv (LN folded)", lambda: ops.ln_linear(xb, n1.weight, n1.bias, n1.eps, blk.attn1.to_qkv.weight, fold=f[0]))
    rep("linear qkv of layer_norm (unfolded)", lambda: blk.attn1.to_qkv(blk.norm1(xb)))
    rep("layer_norm", lambda: blk.norm1(xb))
    B, N = qkv.shape[0], qkv.shape[1]
    a1 = blk.attn1
    q5 = qkv.view(B, N, 3, a1.heads, a1.head_dim)
    o = rep("attention", lambda: ops.attention(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2]))
    o2 = o.reshape(B, N, a1.dim)
    rep("to_out(+residual)", lambda: a1.to_out(o2, residual=xb))
    rep("to_out(no residual)", lambda: a1.to_out(o2))

    # where do the runs differ?  per 16-column chunk and per 128-row block, vs the unfolded result
    ref = blk.attn1.to_qkv(blk.norm1(xb)).float().reshape(-1, qkv.shape[-1])
    ys = [ops.ln_linear(xb, n1.weight, n1.bias, n1.eps, blk.attn1.to_qkv.weight, fold=f[0]).float().reshape(-1, qkv.shape[-1])
          for _ in range(4)]
    for k, y in enumerate(ys):
        d = (y - ref).abs()
        bad = d > 0.05 * ref.abs().clamp_min(0.5)
        rows_bad = bad.any(1).nonzero().flatten()
        cols_bad = bad.any(0).nonzero().flatten()
        print(f"run {k}: max |y-ref| {d.max().item():.3e}  elements off {bad.sum().item()}  rows {rows_bad.numel()} "
              f"(first {rows_bad[:8].tolist()})  cols {cols_bad.numel()} (first {cols_bad[:8].tolist()})", flush=True)
        if k:
            dd = (y - ys[0]).abs() > 0
            r = dd.any(1).nonzero().flatten()
            c = dd.any(0).nonzero().flatten()
            print(f"   vs run 0: differing elements {dd.sum().item()} rows {r.numel()} first {r[:8].tolist()} "
                  f"cols {c.numel()} first {c[:8].tolist()} col-chunks {sorted(set((c // 16).tolist()))[:12]}", flush=True)
