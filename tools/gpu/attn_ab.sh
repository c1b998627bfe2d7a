#!/bin/bash
# Same-box A/B of the bf16 attention kernel: in-tree extension vs variants/attn_old.so, x2 interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in new old; do
    so=""; [ $v = old ] && so=variants/attn_old.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python tools/bench_attn.py --rounds 3 --iters 10 > gpurun_out/attn_ab_${v}_$rep.jsonl 2> gpurun_out/attn_ab_${v}_$rep.err || { tail -5 gpurun_out/attn_ab_${v}_$rep.err; exit 1; }
  done
done
python - <<'PY'
import json
rows={}
for v in ("new","old"):
    for rep in (1,2):
        for l in open(f"gpurun_out/attn_ab_{v}_{rep}.jsonl"):
            if l.startswith("{"):
                d=json.loads(l); rows.setdefault(tuple(d["shape"]),{}).setdefault(v,[]).append(d["us"]["bf16"])
print(f"{'shape':26s} {'old bf16 us':>16s} {'new bf16 us':>16s}")
for k,d in rows.items():
    print(f"{str(list(k)):26s} {'/'.join(f'{x:.1f}' for x in d['old']):>16s} {'/'.join(f'{x:.1f}' for x in d['new']):>16s}")
PY
