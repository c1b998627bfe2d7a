#!/bin/bash
# round 6: the ipc landing without a stream of its own (the supervisor thread's current stream,
# now the default) vs with one (CASSMANTLE_IPC_STREAM=own), host and device landing, vs pipe; x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6j
mkdir -p $O
for rep in 1 2; do
  for v in host device host_own pipe; do
    t=ipc; [ $v = pipe ] && t=pipe
    l=host; [ $v = device ] && l=device
    st=current; [ $v = host_own ] && st=own
    CASSMANTLE_IPC_STREAM=$st timeout -k 10 300 python tools/bench_live.py --gpus 1 --transport $t --land $l --seconds 15 --idle-s 3 > $O/live_${v}_$rep.json 2> $O/live_${v}_$rep.err || { tail -20 $O/live_${v}_$rep.err; exit 1; }
    echo "live v=$v rep=$rep $(python -c "import json;d=json.loads(open('$O/live_${v}_$rep.json').read().strip().splitlines()[-1]);print(d['images_per_s'], d['load_p50_ms'], d['load_p99_ms'], d.get('transport'), d.get('land_us_p50'), d['rounds'])")"
  done
done
