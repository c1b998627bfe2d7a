"""Cold vs warm cost of every GEMM / conv in the steady-state generation of a kernel trace taken
with CASSMANTLE_DIAG_TWICE=1 (each launch issued twice back to back, ops/__init__.py): the first
of a pair sees the operands as the pipeline leaves them (weights from HBM, activations wherever
the producer left them), the second the same bytes warm in MALL / L2.  Grouped by (kernel, grid).

    python tools/diag_twice.py gpurun_out/prof_x/run_kernel_trace.csv [--top 30]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "to_uint8_kernel" in r["Kernel_Name"]]
    if len(ends) >= 2:
        rows = rows[ends[-2] + 1:ends[-1] + 1]
    evals = max(1, sum("latent_step_kernel" in r["Kernel_Name"] for r in rows))
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    i = 0
    while i + 1 < len(rows):
        r0, r1 = rows[i], rows[i + 1]
        n0 = r0["Kernel_Name"]
        if "gemm" in n0 and n0 == r1["Kernel_Name"] and r0["Grid_Size_X"] == r1["Grid_Size_X"]:
            d0 = (int(r0["End_Timestamp"]) - int(r0["Start_Timestamp"])) / 1e3
            d1 = (int(r1["End_Timestamp"]) - int(r1["Start_Timestamp"])) / 1e3
            k = (n0.replace("void (anonymous namespace)::", "")[:60], r0["Grid_Size_X"], r0["Grid_Size_Y"])
            agg[k][0] += 1
            agg[k][1] += d0
            agg[k][2] += d1
            i += 2
            continue
        i += 1
    tc = sum(v[1] for v in agg.values())
    tw = sum(v[2] for v in agg.values())
    print(f"{evals} evals; GEMM/conv pairs {sum(v[0] for v in agg.values())}: cold {tc / 1e3 / evals:.3f} ms/eval, "
          f"warm {tw / 1e3 / evals:.3f} ms/eval, cold - warm {(tc - tw) / 1e3 / evals:.3f} ms/eval")
    for k, v in sorted(agg.items(), key=lambda kv: -(kv[1][1] - kv[1][2]))[:a.top]:
        n, c, w = v
        print(f"{(c - w) / 1e3 / evals:7.3f} ms/eval  n={n:5d} cold {c / n:7.1f} warm {w / n:7.1f} us  {k}")


if __name__ == "__main__":
    main()
