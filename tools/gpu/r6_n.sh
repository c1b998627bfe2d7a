#!/bin/bash
# round 6: the bench's live-round extra with one shared scorer backend and no idle comm stream
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6n
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-sdxl > $O/bench_$rep.json 2> $O/bench_$rep.err || { tail -20 $O/bench_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$rep.json'));print(d['ms_per_step'], d['live_images_per_s'], d['live_score_p50_ms'], d['live_score_p99_ms'], d['live'])"
done
