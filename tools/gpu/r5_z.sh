#!/bin/bash
# round 5: stage overlap (VAE decode of generation i beside the denoise of i+1) with the
# generation stream at high priority: same-box A/B vs no overlap (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5z; mkdir -p $O
for rep in 1 2; do
  for ov in overlap none; do
    a=""; [ $ov = overlap ] && a="--overlap"
    timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-score $a > $O/bench_${ov}_$rep.json 2> $O/bench_${ov}_$rep.err || { tail -5 $O/bench_${ov}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/bench_${ov}_$rep.json'));print('rep $rep $ov ms_per_step', a['ms_per_step'], 'batch1_s', a.get('batch1_s_per_image'), 'stages', a.get('stage_mean_ms'))"
  done
done
