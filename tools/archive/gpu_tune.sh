#!/bin/bash
# kernel numerics for every forced tile config, then the in-situ autotune pass + bench A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "pp or gemm or conv" --timeout 120 --timeout-method thread \
  > gpurun_out/tune_tests.log 2>&1
rc=$?; tail -5 gpurun_out/tune_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/autotune_gemm.py ${TUNE_ARGS} > gpurun_out/autotune.jsonl 2> gpurun_out/autotune.err
rc=$?; echo "autotune rc=$rc"; tail -3 gpurun_out/autotune.err; tail -2 gpurun_out/autotune.jsonl
[ $rc -ne 0 ] && exit $rc
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/gemm_tuning.json
for t in 0 1 0 1; do
  CASSMANTLE_GEMM_TUNE=$t timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-score > gpurun_out/bench_tune$t.log 2>&1 || { tail gpurun_out/bench_tune$t.log; exit 1; }
  echo "tune=$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_tune$t.log)"
done
echo TUNEDONE
