#!/bin/bash
# Full-state GPU check: every gpu test (as the driver runs them), smoke, default bench, in-situ kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/state_tests.log 2>&1
rc=$?; tail -3 gpurun_out/state_tests.log; echo "gpu tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/state_smoke.log 2>&1 || { tail -5 gpurun_out/state_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python -u bench.py > gpurun_out/state_bench.log 2>&1 || { tail -5 gpurun_out/state_bench.log; exit 1; }
tail -1 gpurun_out/state_bench.log
bash tools/gpu_prof_now.sh
