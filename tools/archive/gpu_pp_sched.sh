#!/bin/bash
# A/B of the ping-pong GEMM fragment-read schedule (CASSMANTLE_PP_SCHED=0 four quadrant phases / 2 two phases per k-tile),
# interleaved processes on one box: numerics tests, per-shape op bench, then bench.py
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "pp" --timeout 120 --timeout-method thread > gpurun_out/pps_tests.log 2>&1
rc=$?; tail -2 gpurun_out/pps_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for m in 0 2 0 2; do
  CASSMANTLE_PP_SCHED=$m timeout -k 10 400 python -u tools/bench_gemm_pp.py --rounds 2 --iters 20 --splits 1,2,4 > gpurun_out/pps_ops$m.jsonl 2> gpurun_out/pps_ops$m.err || { tail gpurun_out/pps_ops$m.err; exit 1; }
  echo "sched=$m"
  python - "$m" <<'PY'
import json, sys
for l in open(f"gpurun_out/pps_ops{sys.argv[1]}.jsonl"):
    d = json.loads(l); t = d["table"]
    print(f'{d["shape"]:28s} auto {d["auto_us"]:7.1f}  pp7/1 {t["pp7/1"]:7.1f}  pp8/1 {t["pp8/1"]:7.1f} pp8/2 {t["pp8/2"]:7.1f} pp8/4 {t["pp8/4"]:7.1f}  best {d["best_pp"]} {d["best_pp_us"]} err {d["max_err"]}')
PY
done
for m in 0 2 0 2; do
  CASSMANTLE_PP_SCHED=$m timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-score --no-batch1 > gpurun_out/pps_b.log 2>&1 || { tail -5 gpurun_out/pps_b.log; exit 1; }
  echo "sched=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pps_b.log)"
done
