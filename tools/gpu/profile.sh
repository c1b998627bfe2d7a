#!/bin/bash
# In-situ rocprofv3 kernel trace of the benchmark step for one model, summarised per UNet eval.
#   tools/gpu/profile.sh NAME MODEL DENOISE_STEPS PER_UNITS [extra bench.py args...]
# e.g. tools/gpu/profile.sh sd15 sd15 10 24          (warm-up + timed step = 2 x 12 UNet evals)
#      tools/gpu/profile.sh sdxl sdxl 4 10 --batch 1  (2 x (4 Euler evals + 1 spare))
# writes gpurun_out/prof_NAME_summary.txt (+ the raw trace under gpurun_out/prof_NAME/)
set -o pipefail
name=$1; model=$2; steps=$3; per=$4; shift 4
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- \
  python bench.py --model $model --steps 1 --warmup 1 --denoise-steps $steps --no-score --no-batch1 --no-live --no-sdxl "$@" \
  > gpurun_out/prof_$name.log 2>&1 || { tail -20 gpurun_out/prof_$name.log; exit 1; }
grep '^{' gpurun_out/prof_$name.log | head -c 400; echo
f=$(find gpurun_out/prof_$name -name '*kernel_trace.csv' | head -1)
python tools/prof_summary.py "$f" --per $per --top 60 > gpurun_out/prof_${name}_summary.txt && head -40 gpurun_out/prof_${name}_summary.txt
python tools/prof_summary.py "$f" --last-gen --top 60 > gpurun_out/prof_${name}_steady.txt && head -30 gpurun_out/prof_${name}_steady.txt
