#!/bin/bash
# round 5: GEMM tile raster group per call class (CASSMANTLE_GEMM_RASTER="plain,gated"), same box:
# SD-1.5 bench and SDXL (fp8 attention) over G = 1 (row raster), 2, 4 (tree default), 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5j
mkdir -p $O
for rep in 1 2; do
  for r in 4,4 1,1 2,2 8,8; do
    CASSMANTLE_GEMM_RASTER=$r timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-score --no-batch1 > $O/sd15_${r}_$rep.json 2> $O/sd15_${r}_$rep.err || { tail -5 $O/sd15_${r}_$rep.err; exit 1; }
    echo "sd15 raster $r rep $rep $(python -c "import json;print(json.load(open('$O/sd15_${r}_$rep.json'))['ms_per_step'])")"
  done
done
for rep in 1 2; do
  for r in 4,4 4,1 4,2 4,8 8,8 2,2; do
    CASSMANTLE_GEMM_RASTER=$r timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 3 --warmup 1 --no-score --no-batch1 > $O/sdxl_${r}_$rep.json 2> $O/sdxl_${r}_$rep.err || { tail -5 $O/sdxl_${r}_$rep.err; exit 1; }
    echo "sdxl raster $r rep $rep $(python -c "import json;print(json.load(open('$O/sdxl_${r}_$rep.json'))['ms_per_step'])")"
  done
done
