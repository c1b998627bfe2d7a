"""Measure every GEMM / conv launch of a real pipeline pass under every eligible kernel plan and
write the fastest per shape to ``cassmantle_amd/ops/gemm_tuning.json`` (the table the C++ planner
consults before its cost model; ops.load_gemm_tuning).

The pass is the benchmark's own work: CLIP encode of a 4-image room (CFG batch 8), one UNet
evaluation at batch 8 and the VAE decode of 4 latents, SD-1.5 512^2 (and optionally SDXL).  Each
recorded launch is re-run with identical tensors and epilogue flags (bias / residual / per-image
bias / GroupNorm statistics), so the timing is the in-situ kernel, not a stand-in.  Arms are
interleaved over rounds in one process (cdna_hip_programming.md §5.4 rule 24); the default
planner's pick is always an arm, so an entry is only written when a plan beats it.

    python tools/autotune_gemm.py [--models sd15] [--rounds 3] [--iters 10] [--out PATH]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import ops  # noqa: E402
from cassmantle_amd.ops._ext import ext  # noqa: E402

# the live tile configs (gemm.hip is_live_cfg): 0-10 4/8-wave and ping-pong tiles, 12-14 deep ring,
# 15 = A-in-registers short-K kernel, 16 = 128x80 deep ring, 20-22 = pp 128x160 / 128x128 / 128x64,
# 26/27 = 8-wave 128x80 / 128x64 deep ring, 31-33 = producer-wave 128x80 / 128x64 / 128x160 deep rings
CFGS = [*range(0, 11), 12, 13, 14, 15, 16, 20, 21, 22, 26, 27, 31, 32, 33]
SPLITS = [1, 2, 3, 4, 6, 8, 12, 16]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def weight_rotation(key: str, call, mib: int):
    """-> a closure that re-launches ``call`` with the next of R copies of its weight each time
    (R x |W| >= ``mib`` MiB: every call reads its weight from HBM, as a UNet eval does), or None
    when the weight argument cannot be identified.  The weight is the bf16 tensor argument with
    Nw x K elements (key fields w / k) that is not the first tensor argument (the activations)."""
    f = dict(t[:1] and (t[0], t[1:]) for t in key.split() if t[:1] in "wk" and t[1:].lstrip("-").isdigit())
    if "w" not in f or "k" not in f or not hasattr(call, "args"):
        return None
    numel = int(f["w"]) * int(f["k"])
    tens = [i for i, v in enumerate(call.args) if torch.is_tensor(v)]
    cand = [i for i in tens[1:] if call.args[i].dtype == torch.bfloat16 and call.args[i].numel() == numel]
    if len(cand) != 1:
        return None
    wi = cand[0]
    w = call.args[wi]
    reps = max(2, min(512, (mib << 20) // max(1, w.numel() * 2) + 1))
    copies = [w.clone() for _ in range(reps)]
    state = {"i": 0}

    def run():
        args = list(call.args)
        args[wi] = copies[state["i"] % reps]
        state["i"] += 1
        call.fn(*args, **call.kw)
    run.copies = copies
    return run


def record_pass(model: str, batch: int):
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    from cassmantle_amd.models.schedulers import make_plan
    spec = SPECS[model]
    sd = StableDiffusion(spec, device="cuda", use_graphs=False)
    prompts = [f"A painted style piece depicting the following: scene {i}." for i in range(batch)]
    plan = make_plan(spec.scheduler, 2, spec.guidance)
    with torch.no_grad():
        ops.record_gemms(True)
        ctx, added = sd.encode_prompt(prompts, "blurry, distorted, fake, abstract, negative")
        x0 = sd.init_latents(list(range(batch)), plan)
        st = sd._state(batch, ctx, plan, added)
        sd.unet.set_context(ctx)
        st.load_time(*sd.unet.time_table(st.tsteps, st.unet_in.shape[0], added))
        st.load(x0, ctx, added)
        sd._unet_step(st)
        sd.vae.decode_uint8(st.x.to(sd.dtype))
        torch.cuda.synchronize()
        rec = ops.record_gemms(False)
    return sd, rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="sd15")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(ops.__file__), "gemm_tuning.json"))
    ap.add_argument("--merge", action="store_true", help="keep existing entries of other shapes")
    ap.add_argument("--cfgs", default=None,
                    help="comma list of tile configs to time (default: all); with --merge the shape's "
                         "existing table plan is always an arm, so a partial sweep only adds new winners")
    ap.add_argument("--cold", type=int, default=0, metavar="MIB",
                    help="time every arm with its weight read from HBM on each call (rotating over "
                         "copies totalling MIB MiB, e.g. 512 = twice the Infinity Cache), as in a "
                         "UNet eval; 0 = warm (the same weight tensor re-run)")
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",")] if a.cfgs else CFGS
    os.environ["CASSMANTLE_GEMM_TUNE"] = "0"
    ops.set_mode("hip")
    ext().gemm_tune_clear()
    entries = {}
    if a.merge and os.path.exists(a.out):
        for e in json.load(open(a.out)).get("entries", []):
            entries[e["key"]] = e
    t_start = time.time()
    for model in a.models.split(","):
        keep, rec = record_pass(model, a.batch)
        calls = {}
        counts = {}
        for key, fn in rec:
            counts[key] = counts.get(key, 0) + 1
            calls.setdefault(key, fn)
        print(f"[autotune] {model}: {len(rec)} launches, {len(calls)} shapes", flush=True)
        ext().gemm_record_keys(True)
        for i, (key, fn) in enumerate(calls.items()):
            # the distinct plans this shape can actually run (forced configs fall back when ineligible)
            arms = {}
            ext().gemm_set_override(-1, 0)
            fn()
            arms[tuple(ext().gemm_last_plan())] = "auto"
            if key in entries:                      # the existing table plan (merge)
                ext().gemm_set_override(entries[key]["cfg"], entries[key]["split"])
                fn()
                arms.setdefault(tuple(ext().gemm_last_plan()), "table")
            for c in cfgs:
                for sp in SPLITS:
                    ext().gemm_set_override(c, sp)
                    fn()
                    pl = tuple(ext().gemm_last_plan())
                    arms.setdefault(pl, f"{c}/{sp}")
            ext().gemm_set_override(-1, 0)
            auto_plan = next(k for k, v in arms.items() if v == "auto")
            run = weight_rotation(key, fn, a.cold) if a.cold else None
            res = {pl: [] for pl in arms}
            for _ in range(a.rounds):
                for pl in arms:
                    ext().gemm_set_override(pl[0], pl[1])
                    res[pl].append(timeit(run or fn, a.iters))
            ext().gemm_set_override(-1, 0)
            del run
            med = {pl: statistics.median(v) for pl, v in res.items()}
            best = min(med, key=med.get)
            gain = med[auto_plan] / med[best]
            line = {"key": key, "cold": bool(a.cold), "calls_per_pass": counts[key], "auto": list(auto_plan),
                    "auto_us": round(med[auto_plan], 2), "best": list(best), "best_us": round(med[best], 2),
                    "gain": round(gain, 3), "arms": len(arms)}
            print(json.dumps(line), flush=True)
            if best != auto_plan and gain > 1.02 and (key not in entries or arms[best] != "table"):
                entries[key] = {"key": key, "cfg": best[0], "split": best[1], "us": round(med[best], 2),
                                "auto_us": round(med[auto_plan], 2), "model": model}
        ext().gemm_record_keys(False)
        del keep
        torch.cuda.empty_cache()
    out = {"device": torch.cuda.get_device_name(0), "generated_s": round(time.time() - t_start, 1),
           "entries": sorted(entries.values(), key=lambda e: e["key"])}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(f"[autotune] wrote {len(entries)} entries to {a.out}", flush=True)


if __name__ == "__main__":
    main()
