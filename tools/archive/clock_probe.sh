#!/bin/bash
# Sample GPU clocks/power while the headline bench runs (is the sustained denoise loop clock-capped?).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
( for i in $(seq 1 40); do rocm-smi --showclocks --showpower --showuse 2>/dev/null | grep -E "sclk|Power|GPU use" | tr '\n' ' '; echo; sleep 0.5; done ) > gpurun_out/clock_probe.log 2>&1 &
PROBE=$!
timeout -k 10 300 python -u tools/bench_ops.py --only conv --iters 500 > gpurun_out/clock_ops.log 2>&1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-score > gpurun_out/clock_bench.log 2>&1
kill $PROBE 2>/dev/null
grep '^{' gpurun_out/clock_ops.log | head -8
grep '^{' gpurun_out/clock_bench.log
cat gpurun_out/clock_probe.log
