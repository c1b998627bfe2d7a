set -e
export TMPDIR=/tmp
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES"
for op in "conv 8 64 320 320" "gemm 32768 320 320"; do
  tag=$(echo $op | tr ' ' '_')
  ITERS=5 timeout -s KILL 90 rocprofv3 --pmc $A --output-format csv -d gpurun_out/pmc_${tag}_a -o run -- python tools/one_op.py $op > gpurun_out/pmc_${tag}_a.log 2>&1
  ITERS=5 timeout -s KILL 90 rocprofv3 --pmc $B --output-format csv -d gpurun_out/pmc_${tag}_b -o run -- python tools/one_op.py $op > gpurun_out/pmc_${tag}_b.log 2>&1
done
