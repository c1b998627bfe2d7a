#!/bin/bash
# pipeline smoke after the glue-kernel changes, then the live round with the generation stream
# masked off 0 / 8 / 16 CUs (scorer on all CUs, high priority) and 8 exclusive
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-score --no-batch1 > gpurun_out/r3_b.log 2>&1 || { tail -20 gpurun_out/r3_b.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3_b.log
for rc_ in 0 8 16; do
  timeout -k 10 150 python -u tools/bench_live.py --seconds 20 --idle-s 5 --reserve-cus $rc_ > gpurun_out/live_$rc_.log 2>&1 || { tail -5 gpurun_out/live_$rc_.log; exit 1; }
  grep '^{' gpurun_out/live_$rc_.log >> gpurun_out/r3_live_cumask2.jsonl
done
timeout -k 10 150 python -u tools/bench_live.py --seconds 20 --idle-s 5 --reserve-cus 8 --exclusive-scorer > gpurun_out/live_x8.log 2>&1 || { tail -5 gpurun_out/live_x8.log; exit 1; }
grep '^{' gpurun_out/live_x8.log >> gpurun_out/r3_live_cumask2.jsonl
cat gpurun_out/r3_live_cumask2.jsonl
