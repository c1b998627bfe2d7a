#!/bin/bash
# end-of-session check: every gpu test, smoke, the driver-contract bench, a 2-rank rehearsal of
# the torchrun path on one GPU (gloo), and the in-situ kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?; tail -2 gpurun_out/final_tests.log; echo "gpu tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python -u bench.py > gpurun_out/final_bench.log 2>&1 || { tail -5 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log
CASSMANTLE_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 2 --warmup 1 --no-score --no-batch1 > gpurun_out/final_dp2.log 2>&1 || { tail -8 gpurun_out/final_dp2.log; exit 1; }
grep '^{' gpurun_out/final_dp2.log | tail -1
bash tools/gpu_prof_now.sh
