#!/bin/bash
# full round check: every GPU test, smoke, the driver-contract bench (with scorer + batch-1), a kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -4 "gpurun_out/$name.log"; echo "rc=$rc"; return $rc; }
run tests3 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread && \
run smoke3 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" && \
run bench3 600 python -u bench.py && \
run prof3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --denoise-steps 10 --no-score --no-batch1
echo "ALLDONE rc=$?"
