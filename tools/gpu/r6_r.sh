#!/bin/bash
# round 6: gated A-in-registers GEMM tiles without residual registers (in-tree) vs the previous source (variants/areg_old.so): numerics, bench x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6r
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -k "areg or layer_norm or gn_linear or geglu or unet" -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  for v in new old; do
    so=""; [ $v = old ] && so=variants/areg_old.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-score --no-batch1 --no-live --no-sdxl > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -20 $O/bench_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', $rep, d['ms_per_step'], d['stage_mean_ms'])"
  done
done
