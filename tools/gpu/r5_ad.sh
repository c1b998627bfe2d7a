#!/bin/bash
# round 5 final tree: three back-to-back driver-contract bench runs (box variance) and the
# 2-rank launcher on one GPU (gloo, --oversubscribe)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ad; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
  python -c "import json;a=json.load(open('$O/bench_$i.json'));print('run $i', a['value'], a['ms_per_step'], a['batch1_s_per_image'], a['finite'])"
done
timeout -k 10 500 python bench.py --gpus 2 --oversubscribe --steps 2 --warmup 1 --no-score --no-batch1 > $O/bench_g2.json 2> $O/bench_g2.err || { tail -20 $O/bench_g2.err; exit 1; }
tail -c 700 $O/bench_g2.json; echo
