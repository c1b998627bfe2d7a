#!/bin/bash
# PMC table of one command (tools/pmc_table.py): a kernel trace plus four counter passes (each
# within the per-block limits: <= 8 SQ, <= 4 TCC, <= 2 GRBM), every pass its own rocprofv3 run
# under its own time limit.
#   tools/gpu/pmc_table.sh NAME [bench.py args...]          (eager bench step: --no-graphs)
#   CMD="python tools/one_op.py gemm 2048 1280 1280" tools/gpu/pmc_table.sh NAME
set -o pipefail
name=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/pmc_$name
mkdir -p $out
CMD=${CMD:-"python bench.py --steps 1 --warmup 0 --no-score --no-batch1 --no-live --no-sdxl --no-graphs $*"}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- $CMD > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
i=0
for cnt in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_BUSY_CU_CYCLES TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $cnt --output-format csv -d $out/pmc_p$i -o run -- $CMD > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
python tools/pmc_table.py $out --top ${TOP:-14} --title "$name: ${CFG_NOTE:-}$CMD" > $out/table.txt && cat $out/table.txt
