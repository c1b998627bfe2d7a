#!/bin/bash
# Same-box interleaved A/B of environment knobs on bench.py (one JSON line per arm and repeat):
#   tools/gpu_ab_env.sh OUT REPEATS "bench args" "ENV_A" "ENV_B" ["ENV_C" ...]
# e.g. tools/gpu_ab_env.sh gpurun_out/ab_lnfold.txt 2 "--model sdxl --batch 1 --steps 2" \
#        "CASSMANTLE_LN_FOLD_MODE=1" "CASSMANTLE_LN_FOLD_MODE=2"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=$1; reps=$2; bargs=$3; shift 3
: > $out
for r in $(seq 1 $reps); do
  for arm in "$@"; do
    env $arm timeout -k 10 400 python -u bench.py $bargs --warmup 1 --no-score --no-batch1 > gpurun_out/ab_env_run.log 2>&1 || { tail -5 gpurun_out/ab_env_run.log; exit 1; }
    echo "$arm | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_env_run.log) $(grep -o '"stage_mean_ms": {[^}]*}' gpurun_out/ab_env_run.log)" | tee -a $out
  done
done
