#!/bin/bash
# same-box interleaved bench A/B of an environment knob: KNOB=NAME A=val B=val [TESTS=pytest -k expr]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  env $KNOB=$B timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -m gpu -k "$TESTS" --timeout 200 --timeout-method thread > gpurun_out/envab_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/envab_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
for arm in $A $B $A $B $A $B; do
  env $KNOB=$arm timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-score --no-batch1 > gpurun_out/envab_bench.log 2>&1 || { tail -5 gpurun_out/envab_bench.log; exit 1; }
  echo "$KNOB=$arm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/envab_bench.log)"
done
