#!/bin/bash
# round 5, first box: new GPU tests (batch-8 UNet plans, supervised cuda:0), the driver bench,
# and the shipped launcher with 2 ranks on one GPU (--oversubscribe, gloo)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5a
O=gpurun_out/r5a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_models_gpu.py::test_sd15_unet_bench_batch8_plans tests/test_parallel_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -5 $O/tests.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python bench.py --gpus 2 --oversubscribe --steps 3 --warmup 1 --no-batch1 > $O/bench_os2.json 2> $O/bench_os2.err || { tail -20 $O/bench_os2.err; exit 1; }
cat $O/bench_os2.json
