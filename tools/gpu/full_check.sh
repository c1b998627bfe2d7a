#!/bin/bash
# Full-tree check on one box: the GPU test suite, smoke(), the driver-contract bench, and per-eval
# kernel profiles of SD-1.5 and SDXL (fp8 attention).  Usage: tools/gpu/full_check.sh TAG
set -o pipefail
tag=${1:-check}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
bash tools/gpu/profile.sh ${tag}_sd15 sd15 10 24 || exit 1
bash tools/gpu/profile.sh ${tag}_sdxl sdxl 4 10 --batch 1 --fp8-attention || exit 1
