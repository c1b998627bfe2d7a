#!/bin/bash
# in-situ kernel trace of a short generation + epilogue A/B + PMC of the ping-pong GEMM
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm_pp.py --only epi --splits 1,2 > gpurun_out/epi.jsonl 2> gpurun_out/epi.err || { tail gpurun_out/epi.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/epi.jsonl"):
    d = json.loads(l); print(d["shape"], "auto", d["auto_us"], "best", d["best_pp"], d["best_pp_us"], d["table"])
PY
for pp in 0 1; do
CASSMANTLE_GEMM_PP=$pp timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pp$pp -o run --output-format csv -- \
  python bench.py --steps 1 --warmup 1 --denoise-steps 10 --no-score > gpurun_out/prof_pp$pp.log 2>&1 || { tail -20 gpurun_out/prof_pp$pp.log; exit 1; }
grep '^{' gpurun_out/prof_pp$pp.log | head -c 300; echo
done
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES"
for cfg in 7 -1; do
  for op in "gemm 4096 4096 4096" "conv 8 64 320 320"; do
    tag=$(echo $op | tr ' ' '_')_c$cfg
    CASSMANTLE_GEMM_CFG=$cfg ITERS=5 timeout -s KILL 90 rocprofv3 --pmc $A --output-format csv -d gpurun_out/pmc_${tag}_a -o run -- python tools/one_op.py $op > gpurun_out/pmc_${tag}_a.log 2>&1 || exit 1
    CASSMANTLE_GEMM_CFG=$cfg ITERS=5 timeout -s KILL 90 rocprofv3 --pmc $B --output-format csv -d gpurun_out/pmc_${tag}_b -o run -- python tools/one_op.py $op > gpurun_out/pmc_${tag}_b.log 2>&1 || exit 1
  done
done
echo PROFDONE
