"""Table of an interleaved A/B (tools/gpu/so_ab.sh): one row per KEY value, one column per arm,
the FIELD values of every repetition (a/b) and the arm's ratio to the first arm.

    python tools/ab_table.py KEY FIELD PREFIX arm1 arm2 ...
KEY / FIELD are JSON paths with dots (e.g. ``shape``, ``us.bf16``)."""
import glob
import json
import sys


def get(d, path):
    for p in path.split("."):
        d = d[p]
    return d


def main():
    key, field, prefix, arms = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4:]
    rows = {}
    for arm in arms:
        for f in sorted(glob.glob(f"{prefix}_{arm}_*.jsonl")):
            for line in open(f):
                if not line.startswith("{"):
                    continue
                d = json.loads(line)
                try:
                    rows.setdefault(str(get(d, key)), {}).setdefault(arm, []).append(float(get(d, field)))
                except KeyError:
                    continue
    print(f"{key:28s} " + " ".join(f"{a:>22s}" for a in arms))
    for k, d in rows.items():
        base = sum(d.get(arms[0], [float('nan')])) / max(1, len(d.get(arms[0], [])))
        cells = []
        for a in arms:
            v = d.get(a, [])
            m = sum(v) / len(v) if v else float("nan")
            cells.append(f"{'/'.join(f'{x:.2f}' for x in v)} ({m / base:.3f})" if v else "-")
        print(f"{k:28s} " + " ".join(f"{c:>22s}" for c in cells))


if __name__ == "__main__":
    main()
