#!/bin/bash
# a new tile config ($CFG): numerics of every forced tile, in-situ autotune of the SD-1.5 pass,
# merge only the shapes it wins, then same-box bench committed vs merged table
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "pp_linear or pp_geglu" --timeout 120 --timeout-method thread > gpurun_out/cfgnew_tests.log 2>&1
rc=$?; tail -1 gpurun_out/cfgnew_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/autotune_gemm.py --out gpurun_out/tune_sd15.json > gpurun_out/autotune_sd15.jsonl 2> gpurun_out/autotune_sd15.err
rc=$?; echo "autotune rc=$rc"; [ $rc -ne 0 ] && exit $rc
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/table_cnew.json
for c in ${CFG:-16}; do
  python tools/merge_tuning.py gpurun_out/tune_sd15.json --table gpurun_out/table_cnew.json --only-cfg $c || exit 1
  grep "\"best\": \[$c," gpurun_out/autotune_sd15.jsonl | cut -c1-220
done
for arm in base new base new base new; do
  if [ $arm = new ]; then tp=gpurun_out/table_cnew.json; else tp=; fi
  CASSMANTLE_GEMM_TUNE_PATH=$tp timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-score --no-batch1 > gpurun_out/bench_cnew.log 2>&1 || { tail gpurun_out/bench_cnew.log; exit 1; }
  echo "table=$arm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_cnew.log)"
done
