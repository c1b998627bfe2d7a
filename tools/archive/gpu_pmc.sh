#!/bin/bash
# PMC counters for the hot GEMM/conv/attention kernels (kernel-trace + pmc only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
run() {  # name counters... -- cmd
  local name=$1; shift
  local ctrs=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d gpurun_out/pmc/$name -o run --output-format csv -- "$@" > gpurun_out/pmc/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/$name.log; exit $rc; fi
}
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
C2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM"
C3="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS TA_BUSY_avr"
for c in "$C1" "$C2" "$C3"; do
  tag=$(echo $c | cut -d' ' -f1)
  run conv_$tag "$c" python tools/one_op.py conv 8 64 320 320
  run gemm_$tag "$c" python tools/one_op.py gemm 4096 4096 4096
  run attn_$tag "$c" python tools/one_op.py attn 8 4096 8 40
done
echo PMCDONE
