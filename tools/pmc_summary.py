"""Summarise rocprofv3 --pmc CSVs (pass a / pass b per tag) for the dispatches of one kernel
family: mean counter value per dispatch plus derived ratios.

    python tools/pmc_summary.py gpurun_out pmc_attn_8_4096_8_40 attn_ > summary.txt
"""
from __future__ import annotations

import collections
import csv
import glob
import os
import sys


def load(path, kernel_prefix):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_prefix not in row["Kernel_Name"]:
                    continue
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    root, tag, prefix = sys.argv[1], sys.argv[2], sys.argv[3]
    c = {}
    for part in ("a", "b"):
        v, _ = load(os.path.join(root, f"{tag}_{part}"), prefix)
        c.update(v)
    print(tag, f"(kernels starting '{prefix}', mean per dispatch)")
    for k in sorted(c):
        print(f"  {k:28s} {c[k]:.4g}")

    def r(a, b):
        return c[a] / c[b] if c.get(a) is not None and c.get(b) else float("nan")
    print(f"  -> s_waitcnt waits / wave cycles   {100 * r('SQ_WAIT_INST_ANY', 'SQ_WAVE_CYCLES'):.1f}%")
    print(f"  -> any waits / wave cycles         {100 * r('SQ_WAIT_ANY', 'SQ_WAVE_CYCLES'):.1f}%")
    print(f"  -> MFMA busy / (busy cycles x CUs) {100 * c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(1.0, c.get('SQ_BUSY_CU_CYCLES', 0) * 4):.1f}% (per SIMD)")
    print(f"  -> VALU / MFMA instructions        {r('SQ_INSTS_VALU', 'SQ_INSTS_MFMA'):.2f}")
    print(f"  -> SALU / MFMA instructions        {r('SQ_INSTS_SALU', 'SQ_INSTS_MFMA'):.2f}")
    print(f"  -> LDS bank-conflict / LDS active  {100 * r('SQ_LDS_BANK_CONFLICT', 'SQ_LDS_IDX_ACTIVE'):.1f}%")


if __name__ == "__main__":
    main()
