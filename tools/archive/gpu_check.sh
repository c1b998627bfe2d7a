#!/bin/bash
# GPU validation run: kernel numerics, model parity, smoke, bench (+ optional profile).
# Stops at the first step that crashes/faults/times out (rc not in {0,1}).
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
step kernels 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu
step models 600 python -m pytest tests/test_models_gpu.py -q -m gpu
step smoke 300 python __graft_entry__.py smoke
step bench 600 python bench.py --steps 3 --warmup 1
cat gpurun_out/bench.log | tail -1
if [ "${PROFILE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hip -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --denoise-steps 5 --no-score
fi
echo ALLDONE
