#!/bin/bash
# full round check: every GPU test, smoke, the driver-contract bench, and a 2-rank rehearsal of the
# multi-GPU bench path on the one GPU (gloo process group, both ranks on cuda:0)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -4 "gpurun_out/$name.log"; echo "rc=$rc"; return $rc; }
run tests4 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread && \
run smoke4 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" && \
run bench4 600 python -u bench.py && \
CASSMANTLE_DIST_BACKEND=gloo run dp2_rehearsal 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --no-score --no-batch1
echo "ALLDONE rc=$?"
