#!/bin/bash
# round 6: HIP runtime knob A/B on the bench step (same box, interleaved x2): kernel arguments in
# device memory (HIP_FORCE_DEV_KERNARG=1) vs the runtime default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6s
mkdir -p $O
for rep in 1 2; do
  for v in def dev; do
    if [ $v = dev ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-score --no-live --no-sdxl > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -20 $O/bench_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', $rep, d['ms_per_step'], d['batch1_s_per_image'], d['stage_mean_ms'])"
  done
done
