#!/bin/bash
# round 6: live round (config 5, 1 GPU): supervised async with the ipc data plane (images land on
# GPU 0 from the worker's HBM outbox) vs the pipe transport vs in-process, same box, x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6e
mkdir -p $O
for rep in 1 2; do
  for v in ipc pipe inproc; do
    if [ $v = inproc ]; then args=""; else args="--gpus 1 --transport $v"; fi
    timeout -k 10 300 python tools/bench_live.py $args --seconds 20 --idle-s 4 > $O/live_${v}_$rep.json 2> $O/live_${v}_$rep.err || { tail -20 $O/live_${v}_$rep.err; exit 1; }
    echo "live v=$v rep=$rep $(python -c "import json;d=json.loads(open('$O/live_${v}_$rep.json').read().strip().splitlines()[-1]);print(d['images_per_s'], d['load_p50_ms'], d['load_p99_ms'], d.get('transport'), d.get('land_us_p50'))")"
  done
done
