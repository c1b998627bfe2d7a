#!/bin/bash
# round 5: GPU tests of the new supervisor modes + batch-8 numerics, the driver bench, the
# 2-rank oversubscribed launcher, and the 1-GPU live round: supervised async vs lockstep vs in-process
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_models_gpu.py::test_sd15_unet_bench_batch8_plans tests/test_parallel_gpu.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
grep -E "cos\(b8|passed|failed" $O/tests.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python bench.py --gpus 2 --oversubscribe --steps 3 --warmup 1 --no-batch1 > $O/bench_os2.json 2> $O/bench_os2.err || { tail -20 $O/bench_os2.err; exit 1; }
cat $O/bench_os2.json
for d in async lockstep; do
  timeout -k 10 400 python tools/bench_live.py --gpus 1 --dispatch $d --seconds 20 --idle-s 4 > $O/live_$d.json 2> $O/live_$d.err || { tail -20 $O/live_$d.err; exit 1; }
  tail -1 $O/live_$d.json
done
timeout -k 10 400 python tools/bench_live.py --seconds 20 --idle-s 4 > $O/live_inproc.json 2> $O/live_inproc.err || { tail -20 $O/live_inproc.err; exit 1; }
tail -1 $O/live_inproc.json
