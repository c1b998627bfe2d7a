#!/bin/bash
# round 6: d40 attention staging through per-tile buffer resources (A16_BUFLD) and the tile loop
# unrolled by two (A16_UNROLL2): numerics of the variant, kernel A/B at d = 40, bench A/B x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6q
mkdir -p $O
CASSMANTLE_EXT_SO=variants/a16_11.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "attention or attn" -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_11.txt 2>&1 || { tail -30 $O/tests_11.txt; exit 1; }
tail -1 $O/tests_11.txt
for rep in 1 2; do
  for v in tree 10 11; do
    so=""; [ $v != tree ] && so=variants/a16_$v.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 200 python tools/bench_attn.py --rounds 3 --iters 20 --only-d 40 > $O/attn_${v}_$rep.jsonl 2> $O/attn_${v}_$rep.err || { tail -5 $O/attn_${v}_$rep.err; exit 1; }
  done
done
python - <<'PY'
import json
rows={}
for v in ("tree","10","11"):
    for rep in (1,2):
        for l in open(f"gpurun_out/r6q/attn_{v}_{rep}.jsonl"):
            if l.startswith("{"):
                d=json.loads(l); rows.setdefault(tuple(d["shape"]),{}).setdefault(v,[]).append(d["us"]["bf16"])
for k,d in rows.items():
    print(list(k), {v: "/".join(f"{x:.1f}" for x in xs) for v, xs in d.items()})
PY
for rep in 1 2; do
  for v in tree 11; do
    so=""; [ $v != tree ] && so=variants/a16_$v.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-score --no-batch1 --no-live --no-sdxl > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -20 $O/bench_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', $rep, d['ms_per_step'], d['stage_mean_ms'])"
  done
done
