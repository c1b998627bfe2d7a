#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dbg_lnk_conc.py none c0 conv > gpurun_out/dbg_lnk2.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/dbg_lnk2.log | tail -6
[ $rc -ne 0 ] && exit $rc
ITERS=36 timeout -k 10 300 python -u tools/dbg_lnk_rows.py > gpurun_out/dbg_rows.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/dbg_rows.log | tail -12
[ $rc -ne 0 ] && exit $rc
for arm in noslp slp noslp slp; do
  if [ $arm = slp ]; then so=ab/_C_slp.so; else so=; fi
  CASSMANTLE_EXT_SO=$so timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-score --no-batch1 > gpurun_out/ab_bench.log 2>&1 || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  echo "$arm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bench.log)"
done
