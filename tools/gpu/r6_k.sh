#!/bin/bash
# round 6: GroupNorm apply variants on the UNet / SDXL / VAE shapes (us per call, TB/s):
# tree (4 rows per thread in flight), U8 (8 rows), NT (non-temporal output stores), U8NT; x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6k
mkdir -p $O
for rep in 1 2; do
  for v in tree gnU8 gnNT gnU8NT; do
    so=""; [ $v != tree ] && so=variants/$v.so
    for set in "" "--sdxl" "--vae"; do
      CASSMANTLE_EXT_SO=$so timeout -k 10 200 python tools/bench_membound.py --gn-only $set >> $O/gn_${v}_$rep.jsonl 2> $O/gn_${v}_$rep.err || { tail -5 $O/gn_${v}_$rep.err; exit 1; }
    done
  done
done
python - <<'PY'
import json, glob, collections
res = collections.defaultdict(dict)
for f in sorted(glob.glob("gpurun_out/r6k/gn_*.jsonl")):
    v = f.split("gn_")[1].rsplit("_", 1)[0]; rep = f.rsplit("_", 1)[1].split(".")[0]
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); res[tuple(d["shape"])][f"{v}/{rep}"] = (d["us"], d["TBps"])
vs = ["tree", "gnU8", "gnNT", "gnU8NT"]
print("shape".ljust(24) + "".join(v.rjust(22) for v in vs))
for sh, r in res.items():
    row = str(list(sh)).ljust(24)
    for v in vs:
        a, b = r.get(f"{v}/1"), r.get(f"{v}/2")
        row += (f"{a[0]:.1f}/{b[0]:.1f} ({max(a[1], b[1]):.2f})" if a and b else "-").rjust(22)
    print(row)
PY
