#!/bin/bash
# ping-pong GEMM: numerics of every config, then the interleaved A/B microbenchmark
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "pp" --timeout 120 --timeout-method thread \
  > gpurun_out/pp_tests.log 2>&1
rc=$?; tail -15 gpurun_out/pp_tests.log; echo "pp tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_gemm_pp.py ${PP_ARGS} > gpurun_out/pp_bench.jsonl 2> gpurun_out/pp_bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/pp_bench.err
python - <<'PY'
import json
for l in open("gpurun_out/pp_bench.jsonl"):
    d = json.loads(l)
    print(d["shape"], "auto", d["auto_us"], "best", d["best_pp"], d["best_pp_us"], "torch", d["torch_us"], "x%.2f" % d["speedup_vs_auto"], d["best_pp_tflops"], "TF err", d["max_err"])
PY
exit $rc
