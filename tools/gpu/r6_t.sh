#!/bin/bash
# round 6: fp8 attention hot-loop VALU (fp8 P packs without the zero-fill v_mov: f8x4 as one asm pair)
# in-tree vs the previous attention source (variants/attn_old.so):
# numerics, kernel A/B at head dim 64, SDXL fp8 step A/B x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "attention or attn or fp8" -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  for v in new old; do
    so=""; [ $v = old ] && so=variants/attn_old.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 200 python tools/bench_attn.py --rounds 3 --iters 20 --only-d 64 > $O/attn_${v}_$rep.jsonl 2> $O/attn_${v}_$rep.err || { tail -5 $O/attn_${v}_$rep.err; exit 1; }
  done
done
python - <<'PY'
import json
rows={}
for v in ("new","old"):
    for rep in (1,2):
        for l in open(f"gpurun_out/r6t/attn_{v}_{rep}.jsonl"):
            if l.startswith("{"):
                d=json.loads(l); rows.setdefault(tuple(d["shape"]),{}).setdefault(v,[]).append(d["us"])
for k,d in rows.items():
    print(list(k), {v: xs for v, xs in d.items()})
PY
for rep in 1 2; do
  for v in new old; do
    so=""; [ $v = old ] && so=variants/attn_old.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 400 python bench.py --model sdxl --fp8-attention --batch 1 --steps 3 --warmup 1 --no-score --no-batch1 --no-live --no-sdxl > $O/sdxl_${v}_$rep.json 2> $O/sdxl_${v}_$rep.err || { tail -20 $O/sdxl_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/sdxl_${v}_$rep.json'));print('$v', $rep, d['ms_per_step'], d['stage_mean_ms'])"
  done
done
