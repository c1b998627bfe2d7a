#!/bin/bash
# Full-tree GPU check: GPU test suite, smoke(), driver-contract bench, SD-1.5 per-eval kernel profile.
#   tools/gpu_check.sh TAG      -> gpurun_out/TAG_{tests,smoke,bench}.txt, gpurun_out/prof_TAG_summary.txt
set -o pipefail
tag=${1:-check}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.txt
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/${tag}_tests.txt | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.txt 2>&1 \
  || { tail -20 gpurun_out/${tag}_smoke.txt; exit 1; }
tail -1 gpurun_out/${tag}_smoke.txt
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.txt 2>&1 || { tail -20 gpurun_out/${tag}_bench.txt; exit 1; }
grep '^{' gpurun_out/${tag}_bench.txt | cut -c1-700
bash tools/gpu_profile.sh $tag sd15 10 24
