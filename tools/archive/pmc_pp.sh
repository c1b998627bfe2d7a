#!/bin/bash
# PMC counters on the ping-pong GEMM kernel: 4096^3 (cfg 7) and the SD-1.5 level-1 conv (cfg 8)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"
C="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum"
for spec in "7:gemm 4096 4096 4096" "8:conv 8 64 320 320"; do
  cfg=${spec%%:*}; op=${spec#*:}
  tag=pp${cfg}_$(echo $op | tr ' ' '_')
  for part in A B C; do
    eval cnt=\$$part
    CASSMANTLE_GEMM_CFG=$cfg ITERS=5 timeout -s KILL 90 rocprofv3 --pmc $cnt --output-format csv -d gpurun_out/pmc_${tag}_$part -o run -- python tools/one_op.py $op > gpurun_out/pmc_${tag}_$part.log 2>&1 || { echo "fail $tag $part"; tail -3 gpurun_out/pmc_${tag}_$part.log; exit 1; }
  done
  echo "$tag done"
done
echo PMCDONE
