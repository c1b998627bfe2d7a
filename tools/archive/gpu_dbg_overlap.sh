#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for kn in "" "CASSMANTLE_PP_SCHED=0" "CASSMANTLE_LN_INKERNEL=0" "CASSMANTLE_GEMM_TUNE=0"; do
  echo "=== $kn"
  env $kn timeout -k 10 240 python -u tools/dbg_overlap.py > gpurun_out/dbg_overlap.log 2>&1
  rc=$?; grep -v "^knobs" gpurun_out/dbg_overlap.log | tail -16
  [ $rc -ne 0 ] && { echo "rc=$rc"; exit $rc; }
done
exit 0
