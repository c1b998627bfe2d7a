#!/bin/bash
# round 6: the defaults after the stream finding -- ipc + device landing on the current stream
# (front-end), outbox copy on the worker's current stream -- vs pipe vs in-process, x2; ipc tests;
# then the GroupNorm apply variants (tools/gpu/r6_k.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_parallel_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  for v in ipc pipe inproc; do
    if [ $v = inproc ]; then args=""; else args="--gpus 1 --transport $v"; fi
    timeout -k 10 300 python tools/bench_live.py $args --seconds 15 --idle-s 3 > $O/live_${v}_$rep.json 2> $O/live_${v}_$rep.err || { tail -20 $O/live_${v}_$rep.err; exit 1; }
    echo "live v=$v rep=$rep $(python -c "import json;d=json.loads(open('$O/live_${v}_$rep.json').read().strip().splitlines()[-1]);print(d['images_per_s'], d['load_p50_ms'], d['load_p99_ms'], d.get('transport'), d.get('land_us_p50'))")"
  done
done
bash tools/gpu/r6_k.sh
