#!/bin/bash
# captured VAE decode: pipeline tests + bench, then the live round at Python's default GIL
# switch interval and at 0.5 ms (is the scorer tail host-side?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "graph or overlap or end_to_end or fp8_cross" > gpurun_out/r3_live_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_live_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-score --no-batch1 > gpurun_out/r3_b.log 2>&1 || { tail -20 gpurun_out/r3_b.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"stage_mean_ms": {[^}]*}' gpurun_out/r3_b.log
for sw in 5 0.5; do
  timeout -k 10 150 python -u tools/bench_live.py --seconds 20 --idle-s 5 --switch-ms $sw > gpurun_out/live_sw$sw.log 2>&1 || { tail -5 gpurun_out/live_sw$sw.log; exit 1; }
  grep '^{' gpurun_out/live_sw$sw.log >> gpurun_out/r3_live_switch.jsonl
done
cat gpurun_out/r3_live_switch.jsonl
