#!/bin/bash
# round 5: in-tree top-k + GroupNorm concat cases, then the in-process live round for the A/B row
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py -k "cosine_topk or concat_free or scorer" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 400 python tools/bench_live.py --seconds 20 --idle-s 4 > $O/live_inproc.json 2> $O/live_inproc.err || { tail -20 $O/live_inproc.err; exit 1; }
tail -1 $O/live_inproc.json
