#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -4 "gpurun_out/$name.log"; echo "rc=$rc"; return $rc; }
run kernels2 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread && \
run models2 1100 python -u -m pytest tests/test_models_gpu.py -x -v -s -m gpu --timeout 400 --timeout-method thread && \
run bench2 600 python -u bench.py --steps 3 --warmup 1 --no-score && \
run prof2 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --denoise-steps 10 --no-score
echo "ALLDONE rc=$?"
