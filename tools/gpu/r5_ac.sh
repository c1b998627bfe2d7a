#!/bin/bash
# round 5 final tree: live round (config 5) in-process and supervised (async dispatch), one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ac; mkdir -p $O
timeout -k 10 400 python tools/bench_live.py --gpus 1 --dispatch async --seconds 20 --idle-s 4 > $O/live_async.json 2> $O/live_async.err || { tail -20 $O/live_async.err; exit 1; }
tail -c 600 $O/live_async.json; echo
timeout -k 10 400 python tools/bench_live.py --seconds 20 --idle-s 4 > $O/live_inproc.json 2> $O/live_inproc.err || { tail -20 $O/live_inproc.err; exit 1; }
tail -c 600 $O/live_inproc.json; echo
