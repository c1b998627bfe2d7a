#!/bin/bash
# GEMM tile A/B: numerics with each forced tile config, then the gemm/conv microbench per config.
#   CFGS="5 6" bash tools/gpu_gemm_cfg_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for c in ${CFGS:-5 6}; do
  CASSMANTLE_GEMM_CFG=$c timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm or conv" \
    --timeout 120 --timeout-method thread > gpurun_out/ab_test_$c.log 2>&1 || { echo "cfg $c numerics FAILED"; tail -30 gpurun_out/ab_test_$c.log; exit 1; }
  echo "cfg $c: $(tail -1 gpurun_out/ab_test_$c.log)"
done
for c in auto ${CFGS:-5 6}; do
  if [ "$c" = auto ]; then unset CASSMANTLE_GEMM_CFG; else export CASSMANTLE_GEMM_CFG=$c; fi
  timeout -k 10 600 python -u tools/bench_ops.py --only ${ONLY:-gemm,conv} > gpurun_out/ab_ops_$c.log 2>&1 || { tail -20 gpurun_out/ab_ops_$c.log; exit 1; }
  echo "== cfg $c"; grep '^{' gpurun_out/ab_ops_$c.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(f\"{d['op']:12s} {str(d['shape']):34s} {d['ours_us']:8.1f}us {d.get('ours_tflops',0):7.1f}TF\")"
done
unset CASSMANTLE_GEMM_CFG
echo ABDONE
