#!/bin/bash
# CU-mask bit -> XCD mapping probe, glue-kernel tests, live round with the generation stream
# masked off 0 / 8 / 16 CUs (scorer on all CUs, high priority) and 8 exclusive
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "copy or finalize or latent_init or cu_mask" > gpurun_out/r3_cumask_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_cumask_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/cumask_probe.py > gpurun_out/r3_cumask_probe.jsonl 2>&1 || { tail -5 gpurun_out/r3_cumask_probe.jsonl; exit 1; }
cat gpurun_out/r3_cumask_probe.jsonl
for rc_ in 0 8 16; do
  timeout -k 10 300 python -u tools/bench_live.py --seconds 20 --idle-s 5 --reserve-cus $rc_ > gpurun_out/live_$rc_.log 2>&1 || { tail -5 gpurun_out/live_$rc_.log; exit 1; }
  grep '^{' gpurun_out/live_$rc_.log | tee -a gpurun_out/r3_live_cumask2.jsonl
done
timeout -k 10 300 python -u tools/bench_live.py --seconds 20 --idle-s 5 --reserve-cus 8 --exclusive-scorer > gpurun_out/live_x8.log 2>&1 || { tail -5 gpurun_out/live_x8.log; exit 1; }
grep '^{' gpurun_out/live_x8.log | tee -a gpurun_out/r3_live_cumask2.jsonl
