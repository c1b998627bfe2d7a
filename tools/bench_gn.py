"""GroupNorm(+SiLU) apply-from-producer-statistics microbenchmark at the UNet / VAE shapes
(statistics from ops.channel_stats, timed apply only).  Prints GB/s per shape.

    python tools/bench_gn.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402

for shape in [(8, 64, 64, 320), (8, 64, 64, 640), (8, 32, 32, 640), (8, 32, 32, 1280), (8, 16, 16, 1280),
              (8, 16, 16, 2560), (8, 8, 8, 2560), (4, 128, 128, 512), (4, 512, 512, 128)]:
    x = (torch.randn(*shape, device="cuda") + 0.3).to(torch.bfloat16)
    C = shape[-1]
    st = ops.new_stats(shape[0], C, "cuda")
    ops.channel_stats(x, st)
    g = torch.ones(C, device="cuda", dtype=torch.bfloat16)
    b = torch.zeros(C, device="cuda", dtype=torch.bfloat16)
    f = lambda: ops.group_norm(x, 32, g, b, 1e-5, True, stats=st)
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    print(json.dumps({"shape": list(shape), "us": round(us, 2), "GBps": round(2 * x.numel() * 2 / us / 1e3, 1)}))
