#!/bin/bash
# Numerics of the forced-config tests, then an in-situ tune of the given tile configs against the
# current table plans (SD-1.5 batch 4 + SDXL batch 1), then same-box A/B old vs new table x2.
#   tools/gpu_tune_cfgs.sh 29,30 tag
set -o pipefail
cfgs=$1; tag=${2:-cfgs}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -m gpu -k "_pp" > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
cp cassmantle_amd/ops/gemm_tuning.json gpurun_out/tune_${tag}.json
timeout -k 10 600 python -u tools/autotune_gemm.py --models sd15 --merge --cfgs $cfgs --out gpurun_out/tune_${tag}.json \
  > gpurun_out/autotune_${tag}_sd15.log 2>&1 || { tail -5 gpurun_out/autotune_${tag}_sd15.log; exit 1; }
tail -1 gpurun_out/autotune_${tag}_sd15.log
timeout -k 10 600 python -u tools/autotune_gemm.py --models sdxl --batch 1 --merge --cfgs $cfgs --out gpurun_out/tune_${tag}.json \
  > gpurun_out/autotune_${tag}_sdxl.log 2>&1 || { tail -5 gpurun_out/autotune_${tag}_sdxl.log; exit 1; }
tail -1 gpurun_out/autotune_${tag}_sdxl.log
rm -f gpurun_out/tune_${tag}_ab.txt
for r in 1 2; do
  for t in old new; do
    if [ $t = new ]; then e=CASSMANTLE_GEMM_TUNE_PATH=gpurun_out/tune_${tag}.json; else e=X=0; fi
    env $e timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-score --no-batch1 \
      > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
    echo "sd15 table=$t | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_one.log)" >> gpurun_out/tune_${tag}_ab.txt
    env $e timeout -k 10 400 python -u bench.py --model sdxl --batch 1 --fp8-attention --steps 2 --warmup 1 --no-score --no-batch1 \
      > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
    echo "sdxl table=$t | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_one.log)" >> gpurun_out/tune_${tag}_ab.txt
  done
done
cat gpurun_out/tune_${tag}_ab.txt
