#!/bin/bash
# SDXL (config 4): in-situ autotune of the SDXL shapes, merge only the shapes the committed table
# lacks, then same-box SDXL bench: committed table vs merged table (bf16), and fp8 attention
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/autotune_gemm.py --models sdxl --batch 1 --out gpurun_out/tune_sdxl.json > gpurun_out/autotune_sdxl.jsonl 2> gpurun_out/autotune_sdxl.err
rc=$?; echo "autotune rc=$rc"; tail -2 gpurun_out/autotune_sdxl.err
[ $rc -ne 0 ] && exit $rc
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/table_merged.json
python tools/merge_tuning.py gpurun_out/tune_sdxl.json --table gpurun_out/table_merged.json --model sdxl || exit 1
for arm in "base " "merged " "base " "merged " "merged --fp8-attention"; do
  set -- $arm
  if [ "$1" = merged ]; then tp=gpurun_out/table_merged.json; else tp=; fi
  CASSMANTLE_GEMM_TUNE_PATH=$tp timeout -k 10 400 python -u bench.py --model sdxl --batch 1 --steps 2 --warmup 1 --no-score --no-batch1 $2 > gpurun_out/sdxl_bench.log 2>&1 || { tail -5 gpurun_out/sdxl_bench.log; exit 1; }
  echo "sdxl table=$1 $2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sdxl_bench.log) $(grep -o '"value": [0-9.]*' gpurun_out/sdxl_bench.log)"
done
