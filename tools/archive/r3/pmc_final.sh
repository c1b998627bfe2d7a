#!/bin/bash
# PMC counters of the final tree's three hottest kernel families: ping-pong level-1 conv (cfg 8),
# LayerNorm-folded GEGLU in the A-in-registers kernel, level-1 self-attention (d 40, K/V
# double-buffered).  One counter group per rocprofv3 pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"
for spec in "pp_conv:8:conv 8 64 320 320" "areg_geglu:-1:lngeglu 32768 1280 320" "attn_l1:-1:attn 8 4096 8 40"; do
  tag=${spec%%:*}; rest=${spec#*:}; cfg=${rest%%:*}; op=${rest#*:}
  for part in a b; do
    if [ $part = a ]; then cnt=$A; else cnt=$B; fi
    CASSMANTLE_GEMM_CFG=$cfg ITERS=5 timeout -s KILL 90 rocprofv3 --pmc $cnt --output-format csv -d gpurun_out/pmcf_${tag}_$part -o run -- python tools/one_op.py $op > gpurun_out/pmcf_${tag}_$part.log 2>&1 || { echo "fail $tag $part"; tail -3 gpurun_out/pmcf_${tag}_$part.log; exit 1; }
  done
  echo "$tag done"
done
python tools/pmc_summary.py gpurun_out pmcf_pp_conv gemm_pp_kernel > gpurun_out/pmcf_summary.txt
python tools/pmc_summary.py gpurun_out pmcf_areg_geglu gemm_areg_kernel >> gpurun_out/pmcf_summary.txt
python tools/pmc_summary.py gpurun_out pmcf_attn_l1 attn_fwd_kernel >> gpurun_out/pmcf_summary.txt
cat gpurun_out/pmcf_summary.txt
