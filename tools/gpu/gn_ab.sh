#!/bin/bash
# Same-box A/B of the GroupNorm apply kernel: the in-tree extension vs variants/norm_old.so (the
# previous norm.hip, tools/build_variant.py), interleaved x2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in new old; do
    so=""; [ $v = old ] && so=variants/norm_old.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 200 python tools/bench_membound.py --gn-only > gpurun_out/gn_ab_${v}_$rep.jsonl 2> gpurun_out/gn_ab_${v}_$rep.err || { tail -5 gpurun_out/gn_ab_${v}_$rep.err; exit 1; }
  done
done
python - <<'PY'
import json
rows={}
for v in ("new","old"):
    for rep in (1,2):
        for l in open(f"gpurun_out/gn_ab_{v}_{rep}.jsonl"):
            if l.startswith("{"):
                d=json.loads(l); rows.setdefault(tuple(d["shape"]),{}).setdefault(v,[]).append(d["us"])
print(f"{'shape':22s} {'old us':>14s} {'new us':>14s}")
for k,d in rows.items():
    print(f"{str(list(k)):22s} {'/'.join(f'{x:.2f}' for x in d['old']):>14s} {'/'.join(f'{x:.2f}' for x in d['new']):>14s}")
PY
