"""Which CUs does a CU-mask bit name?  Times a full-chip GEMM on streams masked OFF 8 / 16 / 32
CUs chosen two ways -- contiguous bit ids (round-robin over the XCDs if the driver deals bits
out per XCD) and bit ids at stride 32 (all on one XCD under that mapping) -- against the
unmasked stream.  One JSON line per case.

    python tools/cumask_probe.py [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402
from cassmantle_amd.ops._ext import ext  # noqa: E402
from cassmantle_amd.runtime.cumask import masked_stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    total = int(ext().cu_count(0))
    g = torch.Generator(device="cpu").manual_seed(0)
    x = (torch.randn(8192, 4096, generator=g) * 0.1).to(dev, torch.bfloat16)
    w = (torch.randn(4096, 4096, generator=g) * 0.02).to(dev, torch.bfloat16)
    cases = [("all", [])]
    for n in (8, 16, 32):
        cases.append((f"contig{n}", list(range(n))))
        cases.append((f"stride{n}", [(i * (total // n)) % total for i in range(n)]))
    for name, off in cases:
        keep = [c for c in range(total) if c not in set(off)]
        s = masked_stream(dev, keep) if off else torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            for _ in range(5):
                ops.linear(x, w)
            s.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.iters):
                ops.linear(x, w)
            e1.record(s)
            s.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        print(json.dumps({"case": name, "cus_off": len(off), "us": round(us, 1),
                          "tflops": round(2 * 8192 * 4096 * 4096 / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
