#!/bin/bash
# live round after the batcher drain fix: default GIL interval, 0.5 ms, and CU reservation 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for args in "" "--switch-ms 0.5" "--switch-ms 1" "--reserve-cus 8"; do
  timeout -k 10 150 python -u tools/bench_live.py --seconds 20 --idle-s 5 $args > gpurun_out/live2.log 2>&1 || { tail -5 gpurun_out/live2.log; exit 1; }
  grep '^{' gpurun_out/live2.log | tee -a gpurun_out/r3_live_drain.jsonl
done
