"""Summarise a rocprofv3 kernel trace: time per (kernel, grid) and per kernel family.

    python tools/prof_summary.py gpurun_out/prof_q/run_kernel_trace.csv [--top 40] [--per N]
--per N divides totals by N (e.g. the number of UNet evaluations in the traced run).
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--skip-before", default=None,
                    help="ignore kernels before the first one whose name contains this string")
    ap.add_argument("--last-gen", action="store_true",
                    help="steady state only: summarise the LAST generation (after the previous image's "
                         "to_uint8 up to the last one), per UNet eval = per latent_step_kernel launch")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if a.last_gen:
        ends = [i for i, r in enumerate(rows) if "to_uint8_kernel" in r["Kernel_Name"]]
        if len(ends) >= 2:
            rows = rows[ends[-2] + 1:ends[-1] + 1]
        evals = sum("latent_step_kernel" in r["Kernel_Name"] for r in rows)
        if evals:
            a.per = float(evals)
        span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e6
        print(f"steady state: last generation only, {len(rows)} launches, {evals} UNet evals, "
              f"wall {span:.2f} ms first start -> last end")
    if a.skip_before:
        first = next((i for i, r in enumerate(rows) if a.skip_before in r["Kernel_Name"]), 0)
        rows = rows[first:]
    by_grid = collections.defaultdict(lambda: [0, 0.0])
    fam = collections.defaultdict(float)
    for r in rows:
        n = r["Kernel_Name"].replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        key = (n[:70], r["Grid_Size_X"], r["Grid_Size_Y"])
        by_grid[key][0] += 1
        by_grid[key][1] += d
        fam[re.split(r"[<(]", n)[0]] += d
    tot = sum(v[1] for v in by_grid.values())
    print(f"total {tot / 1e3:.2f} ms  (per unit: {tot / 1e3 / a.per:.3f} ms)")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:20]:
        print(f"  {v / 1e3 / a.per:8.3f} ms {100 * v / tot:5.1f}%  {k}")
    for k, v in sorted(by_grid.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{v[1] / 1e3 / a.per:8.3f}ms {100 * v[1] / tot:5.1f}% n={v[0]:5d} avg={v[1] / v[0]:8.1f}us {k}")
    # kernels that are not this repository's (in-tree kernels live in an anonymous namespace of
    # cassmantle_amd/ops/csrc): ATen, hipBLASLt (Cijk_*), rocBLAS, HIP runtime blits
    ours = [r for r in rows if "anonymous namespace" in r["Kernel_Name"] or r["Kernel_Name"].startswith(("attn_", "gemm_"))]
    other = collections.Counter(r["Kernel_Name"][:90] for r in rows if r not in ours)
    print(f"non-in-tree kernels: {sum(other.values())} launches of {len(other)} kinds")
    for k, n in other.most_common(30):
        print(f"  {n:6d}  {k}")
    # the same census restricted to the LAST generation (everything after the previous image's
    # to_uint8 up to the last one: encode, denoise, decode) -- model load / weight upload /
    # capture-time copies fall outside it
    ends = [i for i, r in enumerate(rows) if "to_uint8_kernel" in r["Kernel_Name"]]
    if ends:
        lo = ends[-2] + 1 if len(ends) > 1 else 0
        win = rows[lo:ends[-1] + 1]
        gen = collections.Counter(r["Kernel_Name"][:90] for r in win
                                  if not ("anonymous namespace" in r["Kernel_Name"]
                                          or r["Kernel_Name"].startswith(("attn_", "gemm_"))))
        print(f"last generation: {len(win)} launches, non-in-tree: {sum(gen.values())} of {len(gen)} kinds")
        for k, n in gen.most_common(30):
            print(f"  {n:6d}  {k}")


if __name__ == "__main__":
    main()
