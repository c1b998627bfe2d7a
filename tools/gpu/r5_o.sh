#!/bin/bash
# round 5: conflict-free K rows for the d=40 kernels: numerics, kernel A/B (x2) vs the K-stride-48
# build, PMC rows, then the bench step A/B (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out/r5o; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "d40 or test_attention" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2; do
  timeout -k 10 300 python -u tools/bench_attn.py --only-d 40 --rounds 7 --iters 20 > $O/attn_new_$rep.jsonl 2>&1 || { tail -20 $O/attn_new_$rep.jsonl; exit 1; }
  grep shape $O/attn_new_$rep.jsonl
  CASSMANTLE_EXT_SO=variants/a16_kstr48.so timeout -k 10 300 python -u tools/bench_attn.py --only-d 40 --rounds 7 --iters 20 > $O/attn_k48_$rep.jsonl 2>&1 || { tail -20 $O/attn_k48_$rep.jsonl; exit 1; }
  grep shape $O/attn_k48_$rep.jsonl
done
CMD="python tools/bench_attn.py --only-d 40 --rounds 1 --iters 3" TOP=5 bash tools/gpu/pmc_table.sh attn_d40b || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-batch1 > $O/bench_new_$rep.json 2> $O/bench_new_$rep.err || { tail -5 $O/bench_new_$rep.err; exit 1; }
  CASSMANTLE_EXT_SO=variants/a16_kstr48.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-batch1 > $O/bench_k48_$rep.json 2> $O/bench_k48_$rep.err || { tail -5 $O/bench_k48_$rep.err; exit 1; }
  python -c "import json;a=json.load(open('$O/bench_new_$rep.json'));b=json.load(open('$O/bench_k48_$rep.json'));print('rep $rep new', a['ms_per_step'], 'k48', b['ms_per_step'])"
done
