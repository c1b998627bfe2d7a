#!/bin/bash
# same-box interleaved bench A/B of the in-tree extension vs an alternative build (ab/$ALT)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ALT=${ALT:-ab/_C_noslp_all.so}
CASSMANTLE_EXT_SO=$ALT timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests.log
[ $rc -ne 0 ] && exit $rc
for arm in base alt base alt base alt; do
  if [ $arm = alt ]; then so=$ALT; else so=; fi
  CASSMANTLE_EXT_SO=$so timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-score --no-batch1 > gpurun_out/ab_bench.log 2>&1 || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  echo "$arm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bench.log)"
done
