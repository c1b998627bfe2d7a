#!/bin/bash
# round 6: GroupNorm apply with non-temporal output stores + the 8-row rule (tree) vs NT only vs
# round-5 apply (gn_old), in situ: GN / norm tests, SD-1.5 (incl. batch 1) and SDXL benches x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu \
  -k "norm or gn or group or vae or unet" -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 200 python tools/bench_membound.py --gn-only --vae > $O/gn_vae_tree.jsonl 2>&1 || { tail -5 $O/gn_vae_tree.jsonl; exit 1; }
for rep in 1 2; do
  for v in tree gn_ntonly gn_old; do
    so=""; [ $v != tree ] && so=variants/$v.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-score --no-live --no-sdxl > $O/sd15_${v}_$rep.json 2> $O/sd15_${v}_$rep.err || { tail -5 $O/sd15_${v}_$rep.err; exit 1; }
    echo "sd15 v=$v rep=$rep $(python -c "import json;d=json.load(open('$O/sd15_${v}_$rep.json'));print(d['ms_per_step'], d['batch1_s_per_image'], d['stage_mean_ms'])")"
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 3 --warmup 1 --no-score --no-batch1 --no-live --no-sdxl > $O/sdxl_${v}_$rep.json 2> $O/sdxl_${v}_$rep.err || { tail -5 $O/sdxl_${v}_$rep.err; exit 1; }
    echo "sdxl v=$v rep=$rep $(python -c "import json;d=json.load(open('$O/sdxl_${v}_$rep.json'));print(d['ms_per_step'], d['stage_mean_ms'])")"
  done
done
