#!/bin/bash
# round 5: fragment prefetch across the two k-steps of a deep-ring / 2-stage GEMM k-tile
# (GEMM_FRAG_PREFETCH=1, variants/fp1.so) vs the tree: small-GEMM probe, GEMM numerics, bench x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5i
mkdir -p $O
CASSMANTLE_EXT_SO=variants/fp1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or conv or linear or split" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for v in tree fp1; do
  so=""; [ "$v" != tree ] && so=variants/$v.so
  CASSMANTLE_EXT_SO=$so timeout -k 10 300 python tools/probe_small_gemm.py --m 2048 --n 1280 --ks 640,1280,2560 --cfgs 31,26,16,3,14,33 --splits 1,2 --rotate 40 > $O/probe_$v.jsonl 2> $O/probe_$v.err || { tail -20 $O/probe_$v.err; exit 1; }
  echo $v; grep '"M"' $O/probe_$v.jsonl
done
for rep in 1 2; do
  for v in tree fp1; do
    so=""; [ "$v" != tree ] && so=variants/$v.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-score > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -20 $O/bench_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', $rep, d['ms_per_step'], d['batch1_s_per_image'], d['stage_mean_ms'])"
  done
done
