#!/bin/bash
# round-2 GPU check: all numerics, smoke, bench, then the legacy-stream stall reproduction
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/$name.log"
  echo "rc=$rc"
  return $rc
}
run kernels 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread && \
run models 900 python -u -m pytest tests/test_models_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread && \
run smoke 300 python -u __graft_entry__.py smoke && \
run bench 600 python -u bench.py --steps 3 --warmup 1 && \
run stall_stream 150 python -u tools/repro_stall.py --arm stream --seconds 40 && \
run stall_legacy 150 python -u tools/repro_stall.py --arm legacy --seconds 40
echo "ALLDONE rc=$?"
