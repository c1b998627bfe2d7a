#!/bin/bash
# round 5: GroupNorm apply block count on large tensors (A/B), then the supervisor GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5aj
mkdir -p $O
for cfg in "0 1024" "32 2048" "32 4096"; do
  set -- $cfg
  for sh in "" "--sdxl"; do
    CASSMANTLE_GN_BIG_MB=$1 CASSMANTLE_GN_BIG_BLOCKS=$2 timeout -k 10 120 python tools/bench_membound.py --gn-only $sh \
      2>>$O/err.txt | sed "s/^/{\"big_mb\": $1, \"big_blocks\": $2, \"row\": /; s/\$/}/" >> $O/gn_ab.jsonl || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests/test_parallel_gpu.py -x -v --timeout 240 --timeout-method thread -m gpu \
  > $O/tests.txt 2>&1 || exit 1
