#!/bin/bash
# round 5: raster groups spanning every M panel (G = 16: an XCD's 32 tiles = all 16 M-panels x 2
# N-panels, so each (cold) weight panel is fetched by one XCD) vs the default G = 4, same box x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5ae; mkdir -p $O
for rep in 1 2; do
  for r in 4,4 16,4 16,16 32,4; do
    CASSMANTLE_GEMM_RASTER=$r timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-score --no-batch1 > $O/sd15_${r}_$rep.json 2> $O/sd15_${r}_$rep.err || { tail -5 $O/sd15_${r}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/sd15_${r}_$rep.json'));print('rep $rep raster $r sd15', a['ms_per_step'])"
  done
  for r in 4,4 16,4; do
    CASSMANTLE_GEMM_RASTER=$r timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 2 --warmup 1 --no-score --no-batch1 > $O/sdxl_${r}_$rep.json 2> $O/sdxl_${r}_$rep.err || { tail -5 $O/sdxl_${r}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/sdxl_${r}_$rep.json'));print('rep $rep raster $r sdxl', a['ms_per_step'])"
  done
done
