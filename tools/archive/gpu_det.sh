cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/dbg_det_lnk.py > gpurun_out/det_lnk.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/det_lnk.log | tail -6; echo "rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q -m gpu -k "determin" --timeout 200 --timeout-method thread > gpurun_out/det_t.log 2>&1; rc=$?; tail -1 gpurun_out/det_t.log; [ $rc -ne 0 ] && exit $rc
for m in 0 1 0 1; do
  CASSMANTLE_LN_INKERNEL=$m timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-score --no-batch1 > gpurun_out/det_b.log 2>&1 || { tail -5 gpurun_out/det_b.log; exit 1; }
  echo "inkernel=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/det_b.log)"
done
