#!/bin/bash
# in-situ autotune of the current kernels, then bench A/B previous table vs new table (same box)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/autotune_gemm.py ${TUNE_ARGS} > gpurun_out/autotune.jsonl 2> gpurun_out/autotune.err
rc=$?; echo "autotune rc=$rc"; tail -3 gpurun_out/autotune.err; tail -2 gpurun_out/autotune.jsonl
[ $rc -ne 0 ] && exit $rc
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/gemm_tuning.json
for t in prev new prev new prev new; do
  if [ $t = prev ]; then tp=tools/gemm_tuning_prev.json; else tp=; fi
  CASSMANTLE_GEMM_TUNE_PATH=$tp timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-score --no-batch1 > gpurun_out/bench_tune.log 2>&1 || { tail gpurun_out/bench_tune.log; exit 1; }
  echo "table=$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_tune.log)"
done
