#!/bin/bash
# round 6: in-situ value of MALL-warm weights -- every GEMM / conv weight read by ops.prefetch right
# before its launch (CASSMANTLE_PF_SERIAL=1) vs the tree, same box: bench x2 interleaved + steady
# per-eval kernel profiles of both
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6c
mkdir -p $O
for rep in 1 2; do
  for v in tree pf; do
    e=""; [ $v = pf ] && e="CASSMANTLE_PF_SERIAL=1"
    env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-score --no-live --no-sdxl > $O/sd15_${v}_$rep.json 2> $O/sd15_${v}_$rep.err || { tail -5 $O/sd15_${v}_$rep.err; exit 1; }
    echo "sd15 v=$v rep=$rep $(python -c "import json;d=json.load(open('$O/sd15_${v}_$rep.json'));print(d['ms_per_step'], d['batch1_s_per_image'])")"
  done
done
bash tools/gpu/profile.sh r6c_tree sd15 10 24 && CASSMANTLE_PF_SERIAL=1 bash tools/gpu/profile.sh r6c_pf sd15 10 24
rm -rf gpurun_out/prof_r6c_tree gpurun_out/prof_r6c_pf
