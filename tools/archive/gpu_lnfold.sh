#!/bin/bash
# in-kernel LayerNorm fold: kernel numerics, model parity, bench A/B (CASSMANTLE_LN_FOLD 0/1 interleaved)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "layer_norm or areg" --timeout 120 --timeout-method thread > gpurun_out/ln_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ln_tests.log; echo "kernel tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -x -q -m gpu -k "full_size or end_to_end or sdxl" --timeout 240 --timeout-method thread > gpurun_out/ln_models.log 2>&1
rc=$?; tail -3 gpurun_out/ln_models.log; grep -o "psnr [0-9.]* dB, mean |diff| [0-9.]*" gpurun_out/ln_models.log; echo "model tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
for f in 1 0 1 0; do
  CASSMANTLE_LN_FOLD=$f timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-score --no-batch1 > gpurun_out/ln_bench.log 2>&1 || { tail -5 gpurun_out/ln_bench.log; exit 1; }
  echo "lnfold=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ln_bench.log)"
done
exit 0
