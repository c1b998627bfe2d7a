#!/bin/bash
# round 6: d40 attention deferred-max threshold 16 (variants/thr16.so) vs 8 (tree): numerics,
# kernel A/B, bench x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6x
mkdir -p $O
CASSMANTLE_EXT_SO=variants/thr16.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "attention or attn" -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  for v in tree thr16; do
    so=""; [ $v != tree ] && so=variants/$v.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 200 python tools/bench_attn.py --rounds 3 --iters 20 --only-d 40 > $O/attn_${v}_$rep.jsonl 2> $O/attn_${v}_$rep.err || { tail -5 $O/attn_${v}_$rep.err; exit 1; }
    echo "$v $rep $(grep -h '"shape"' $O/attn_${v}_$rep.jsonl | head -1)"
  done
done
for rep in 1 2; do
  for v in tree thr16; do
    so=""; [ $v != tree ] && so=variants/$v.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-score --no-batch1 --no-live --no-sdxl > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -20 $O/bench_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', $rep, d['ms_per_step'], d['stage_mean_ms'])"
  done
done
