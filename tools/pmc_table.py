"""Per-kernel PMC table of a model's benchmark step (verdict r3 item 4: "tiling choices shown with
rocprof counters"): for the top-N (kernel, grid) rows by time, the MFMA-busy fraction, VALU and
SALU instructions per MFMA, LDS bank-conflict rate, L2 hit rate, HBM bytes (FETCH_SIZE +
WRITE_SIZE), achieved TF/s and TB/s, and the roofline bound.

Input: one directory per counter pass (``pmc_p1`` .. ``pmc_p4``, rocprofv3 ``--pmc`` CSV output) and
a kernel-trace directory (``trace``) of the same command, all under ROOT (tools/gpu/pmc_table.sh
writes that layout).

    python tools/pmc_table.py ROOT [--top 12] [--title "..."]

Rows are keyed by (kernel name, total grid size); counters are averaged per dispatch.  FLOPs come
from the MFMA instruction count and the MFMA shape each kernel family issues (16x16x32 bf16 for
the GEMM / conv kernels, 32x32x16 bf16 for attention, 32x32x64 e4m3 for the fp8 attention).
Ridge point: 2.5 PF/s bf16 dense / 8 TB/s HBM = 312 FLOP/byte (MI355X; fp8 rows use 5 PF/s).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re

PEAK_BF16 = 2.5e15
PEAK_FP8 = 5.0e15
HBM = 8.0e12


def short(name: str) -> str:
    n = name.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*$", "", n)


def mfma_flops(name: str) -> float:
    """FLOPs of one MFMA instruction of this kernel family."""
    if "attn_fp8" in name:
        return 2 * 32 * 32 * 64
    if name.startswith(("attn_fwd", "attn_d512")):
        return 2 * 32 * 32 * 16
    if name.startswith("attn_mx"):          # per 64-key tile: 6 x 32x32x16 + 12 x 16x16x32
        return (6 * 2 * 32 * 32 * 16 + 12 * 2 * 16 * 16 * 32) / 18
    return 2 * 16 * 16 * 32


def grid_total(row: dict) -> int:
    if "Grid_Size" in row and row["Grid_Size"]:
        return int(float(row["Grid_Size"]))
    return int(row.get("Grid_Size_X", 1)) * int(row.get("Grid_Size_Y", 1)) * int(row.get("Grid_Size_Z", 1))


def load_trace(root: str):
    rows = []
    for f in glob.glob(os.path.join(root, "trace", "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        k = (short(r["Kernel_Name"]), grid_total(r))
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return agg


def load_counters(root: str):
    """-> {(kernel, grid): {counter: mean per dispatch}}"""
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in sorted(glob.glob(os.path.join(root, "pmc_*"))):
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = (short(r["Kernel_Name"]), grid_total(r))
                c = r["Counter_Name"]
                sums[k][c] += float(r["Counter_Value"])
                disp[k][c].add((d, r.get("Dispatch_Id") or r.get("Correlation_Id") or len(disp[k][c])))
    out = {}
    for k, cs in sums.items():
        out[k] = {c: v / max(1, len(disp[k][c])) for c, v in cs.items()}
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    trace = load_trace(a.root)
    ctr = load_counters(a.root)
    tot = sum(v[1] for v in trace.values())
    if a.title:
        print(f"# {a.title}")
    print(f"# traced kernel time {tot / 1e3:.2f} ms; top {a.top} (kernel, grid) rows by total time; counters are "
          "means per dispatch")
    print("# MFMA%: SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x SQ_BUSY_CU_CYCLES); VALU/M, SALU/M: instructions per MFMA "
          "instruction; LDSc%: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; L2hit%: TCC_HIT / (TCC_HIT + TCC_MISS); "
          "HBM MB: FETCH_SIZE + WRITE_SIZE; bound: FLOP/byte vs the ridge (312 bf16, 625 fp8) -> compute|memory, "
          "%bound = achieved / that roof")
    hdr = (f"{'kernel':58s} {'grid':>9s} {'n':>4s} {'us':>8s} {'%time':>6s} {'MFMA%':>6s} {'VALU/M':>7s} {'SALU/M':>7s} "
           f"{'LDSc%':>6s} {'L2hit%':>7s} {'HBM MB':>8s} {'TF/s':>7s} {'TB/s':>6s} {'bound':>8s} {'%bound':>7s}")
    print(hdr)
    for k, (n, t) in sorted(trace.items(), key=lambda kv: -kv[1][1])[:a.top]:
        us = t / n
        c = ctr.get(k, {})

        def g(name, default=float("nan")):
            return c.get(name, default)
        mfma_pct = 100 * g("SQ_VALU_MFMA_BUSY_CYCLES") / (4 * g("SQ_BUSY_CU_CYCLES")) if g("SQ_BUSY_CU_CYCLES", 0) else float("nan")
        vm = g("SQ_INSTS_VALU") / g("SQ_INSTS_MFMA") if g("SQ_INSTS_MFMA", 0) else float("nan")
        sm = g("SQ_INSTS_SALU") / g("SQ_INSTS_MFMA") if g("SQ_INSTS_MFMA", 0) else float("nan")
        ldsc = 100 * g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE") if g("SQ_LDS_IDX_ACTIVE", 0) else float("nan")
        hit, miss = g("TCC_HIT_sum"), g("TCC_MISS_sum")
        l2 = 100 * hit / (hit + miss) if (hit + miss) == (hit + miss) and (hit + miss) > 0 else float("nan")
        hbm = (g("FETCH_SIZE", 0) + g("WRITE_SIZE", 0)) * 1024          # rocprof reports KB
        flops = g("SQ_INSTS_MFMA", 0) * mfma_flops(k[0])
        tfs = flops / (us * 1e-6) / 1e12 if us > 0 else 0
        tbs = hbm / (us * 1e-6) / 1e12 if us > 0 and hbm > 0 else float("nan")
        peak = PEAK_FP8 if "fp8" in k[0] else PEAK_BF16
        ridge = peak / HBM
        if flops > 0 and hbm > 0:
            ai = flops / hbm
            bound = "compute" if ai >= ridge else "memory"
            roof = peak if ai >= ridge else ai * HBM
            pct = 100 * (flops / (us * 1e-6)) / roof
        elif hbm > 0:
            bound, pct = "memory", 100 * (hbm / (us * 1e-6)) / HBM
        else:
            bound, pct = "-", float("nan")
        name = k[0] if len(k[0]) <= 58 else k[0][:57] + "~"
        print(f"{name:58s} {k[1]:9d} {n:4d} {us:8.1f} {100 * t / tot:6.1f} {mfma_pct:6.1f} {vm:7.2f} {sm:7.2f} {ldsc:6.1f} "
              f"{l2:7.1f} {hbm / 1e6:8.2f} {tfs:7.0f} {tbs:6.2f} {bound:>8s} {pct:7.1f}")
    missing = [k for k, _ in sorted(trace.items(), key=lambda kv: -kv[1][1])[:a.top] if k not in ctr]
    if missing:
        print(f"# {len(missing)} rows without counters (grid keys differ between the trace and the PMC runs): "
              + "; ".join(f"{k[0][:40]}@{k[1]}" for k in missing))


if __name__ == "__main__":
    main()
