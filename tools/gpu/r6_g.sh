#!/bin/bash
# round 6: why is the supervised live round slower with the ipc data plane (6.29 vs 7.27 images/s
# with pipe, r6_f)?  ipc as built, ipc without the landing copy (noland), ipc landing to the host
# (hostland), pipe -- same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6g
mkdir -p $O
for v in ipc noland hostland pipe; do
  t=ipc; [ $v = pipe ] && t=pipe
  d=""; [ $v = noland ] && d=noland; [ $v = hostland ] && d=hostland
  CASSMANTLE_IPC_DIAG=$d timeout -k 10 300 python tools/bench_live.py --gpus 1 --transport $t --seconds 15 --idle-s 3 > $O/live_$v.json 2> $O/live_$v.err || { tail -20 $O/live_$v.err; exit 1; }
  echo "live v=$v $(python -c "import json;d=json.loads(open('$O/live_$v.json').read().strip().splitlines()[-1]);print(d['images_per_s'], d['load_p50_ms'], d['load_p99_ms'], d.get('transport'), d.get('land_us_p50'), d['rounds'])")"
done
