"""Decode throughput of the local prompt LM (random-init weights, batch 1, hipGraph decode loop).

    python tools/bench_lm.py --model mistral-7b --new 96 --prompt-len 64

Prints one JSON line: ms/token, tokens/s and the HBM-bandwidth bound (weights bytes / 8 TB/s).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cassmantle_amd.models.lm import LM_CONFIGS, LMTextGenerator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--new", type=int, default=96)
    ap.add_argument("--prompt-len", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-graphs", action="store_true")
    a = ap.parse_args()
    cfg = LM_CONFIGS[a.model]
    t0 = time.time()
    g = LMTextGenerator(cfg, device="cuda", use_graphs=not a.no_graphs, max_new_cap=max(a.new, 8))
    torch.cuda.synchronize()
    init_s = time.time() - t0
    params = sum(p.numel() for p in g.model.parameters())
    prompt = [256] + [65 + (i % 26) for i in range(a.prompt_len - 1)]
    g.generate_ids(prompt, a.new, a.new)          # warmup + graph capture
    torch.cuda.synchronize()
    # prefill alone
    t0 = time.time()
    for _ in range(a.reps):
        g.generate_ids(prompt, 1, 1)
    torch.cuda.synchronize()
    t_one = (time.time() - t0) / a.reps
    t0 = time.time()
    for _ in range(a.reps):
        g.generate_ids(prompt, a.new, a.new)
    torch.cuda.synchronize()
    t_all = (time.time() - t0) / a.reps
    ms_tok = (t_all - t_one) / max(1, a.new - 1) * 1e3
    bound_ms = params * 2 / 8.0e12 * 1e3
    print(json.dumps({"model": cfg.name, "params": params, "init_s": round(init_s, 2),
                      "prompt_len": a.prompt_len, "new_tokens": a.new,
                      "prefill_plus_1_ms": round(t_one * 1e3, 2), "decode_ms_per_token": round(ms_tok, 3),
                      "decode_tokens_per_s": round(1e3 / ms_tok, 1), "hbm_bound_ms_per_token": round(bound_ms, 3),
                      "graphs": not a.no_graphs}))


if __name__ == "__main__":
    main()
