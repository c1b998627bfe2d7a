#!/bin/bash
# PMC counters on the flash-attention kernels (2 passes per shape, one rocprofv3 run each)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC"
for op in "attn 8 4096 8 40" "attn 2 4096 10 64" "attn8 2 4096 10 64" "attn 2 1024 20 64" "attn8 2 1024 20 64"; do
  tag=$(echo $op | tr ' ' '_')
  ITERS=5 timeout -s KILL 90 rocprofv3 --pmc $A --output-format csv -d gpurun_out/pmc_${tag}_a -o run -- python tools/one_op.py $op > gpurun_out/pmc_${tag}_a.log 2>&1 || exit 1
  ITERS=5 timeout -s KILL 90 rocprofv3 --pmc $B --output-format csv -d gpurun_out/pmc_${tag}_b -o run -- python tools/one_op.py $op > gpurun_out/pmc_${tag}_b.log 2>&1 || exit 1
  echo "$tag done"
done
echo PMCDONE
