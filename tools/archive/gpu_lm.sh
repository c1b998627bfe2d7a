#!/bin/bash
# LM decode path on the GPU: numerics + graph decode + 7B decode throughput, then the SD bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
: > gpurun_out/steps.log
step lm_tests 600 python -m pytest tests/test_lm.py -q -m gpu -x
step kernels 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu
step bench_lm 600 python tools/bench_lm.py --model mistral-7b --new 96 --prompt-len 64
step bench 600 python bench.py --steps 3 --warmup 1
echo ALLDONE
