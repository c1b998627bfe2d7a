#!/bin/bash
# round 5: steady-state profiles after the batch-1 re-tune + adaptive split-K reduce
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/profile.sh b1w sd15 10 24 --batch 1 > gpurun_out/prof_b1w.txt 2>&1 || { tail -20 gpurun_out/prof_b1w.txt; exit 1; }
head -50 gpurun_out/prof_b1w_steady.txt
rm -rf gpurun_out/prof_b1w
