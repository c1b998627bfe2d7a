#!/bin/bash
# ping-pong SCHED 3 (LDS-DMA issued inside the MFMA clusters; s3p1 mid-cluster, s3p0 at its start):
# GEMM/conv numerics on each variant, then same-box A/Bs of the ResNet convs, the residual
# projections and the bench step; then the supervised live round with the early-closing window
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in s3p1 s3p0; do
  CASSMANTLE_EXT_SO=variants/$v.so timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "pp or conv or gemm" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i_tests_$v.log 2>&1 || { tail -30 gpurun_out/r4i_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r4i_tests_$v.log
done
bash tools/gpu/so_ab.sh s3c shape us "python tools/bench_resnet_convs.py --rounds 3" tree s3p1 s3p0 || exit 1
bash tools/gpu/so_ab.sh s3l shape us "python tools/bench_resnet_convs.py --rounds 3 --linear" tree s3p1 s3p0 || exit 1
bash tools/gpu/so_ab.sh s3b config.model ms_per_step "python bench.py --steps 6 --warmup 2 --no-score --no-batch1" tree s3p1 s3p0 || exit 1
grep -h stage_mean gpurun_out/s3b_tree_*.jsonl | python -c "import sys,json; [print(json.loads(l)['stage_mean_ms'], json.loads(l)['ms_per_step']) for l in sys.stdin]"
timeout -k 10 400 python tools/bench_live.py --gpus 1 --players 64 --seconds 25 --idle-s 6 > gpurun_out/r4i_live.json 2> gpurun_out/r4i_live.err || { tail -20 gpurun_out/r4i_live.err; exit 1; }
grep '^{' gpurun_out/r4i_live.json
