#!/bin/bash
# round 5: feed-forward row statistics chained to the next block's folded LayerNorm (SDXL):
# the model test, then same-box A/B of SDXL (x2) and one SD-1.5 check
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5aa; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py -k "chained or sdxl_unet_reduced" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2; do
  for ff in 1 0; do
    CASSMANTLE_FF_ROWSTATS=$ff timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 2 --warmup 1 --no-score --no-batch1 > $O/sdxl_${ff}_$rep.json 2> $O/sdxl_${ff}_$rep.err || { tail -5 $O/sdxl_${ff}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/sdxl_${ff}_$rep.json'));print('rep $rep ff_rowstats $ff sdxl ms_per_step', a['ms_per_step'], a.get('finite'))"
  done
done
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-score --no-batch1 > $O/sd15.json 2> $O/sd15.err || { tail -5 $O/sd15.err; exit 1; }
python -c "import json;a=json.load(open('$O/sd15.json'));print('sd15 ms_per_step', a['ms_per_step'], a.get('finite'))"
