#!/bin/bash
# round 6: hardware queues per process (GPU_MAX_HW_QUEUES = 1 / 2 / 4 = default) on the 1-GPU bench
# step and the supervised live round: does the number of mapped queues cost throughput?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6o
mkdir -p $O
for rep in 1 2; do
  for q in 4 2 1; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-score --no-live --no-sdxl > $O/sd15_q${q}_$rep.json 2> $O/sd15_q${q}_$rep.err || { tail -5 $O/sd15_q${q}_$rep.err; exit 1; }
    echo "sd15 q=$q rep=$rep $(python -c "import json;d=json.load(open('$O/sd15_q${q}_$rep.json'));print(d['ms_per_step'], d['batch1_s_per_image'])")"
  done
done
for q in 4 2; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/bench_live.py --gpus 1 --seconds 15 --idle-s 3 > $O/live_q$q.json 2> $O/live_q$q.err || { tail -20 $O/live_q$q.err; exit 1; }
  echo "live q=$q $(python -c "import json;d=json.loads(open('$O/live_q$q.json').read().strip().splitlines()[-1]);print(d['images_per_s'], d['load_p50_ms'], d['load_p99_ms'])")"
done
