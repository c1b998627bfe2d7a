#!/bin/bash
# round 6: (1) exp pipe probe (is a polynomial exp2 on the FMA path cheaper than v_exp_f32?),
# (2) weight-prefetch probe (graph-branch concurrency, MALL-warm GEMMs), (3) the driver's bench
# command with the config-4 / config-5 extras
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 120 tools/bin/exp_pipe_probe > $O/exp_pipe_probe.jsonl 2>&1 || { cat $O/exp_pipe_probe.jsonl; exit 1; }
cat $O/exp_pipe_probe.jsonl
timeout -k 10 300 python tools/probe_weight_prefetch.py > $O/prefetch_probe.jsonl 2> $O/prefetch_probe.err || { tail -20 $O/prefetch_probe.err; exit 1; }
cat $O/prefetch_probe.jsonl
t0=$(date +%s)
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - t0 )) s"
cat $O/bench.json
