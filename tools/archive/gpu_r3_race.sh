#!/bin/bash
# LNK (in-kernel LayerNorm A-in-registers GEMM) race screen: control = round-2 source built WITH
# SLP (expected to reproduce the concurrency failures), fix = padded permlane swaps with SLP on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out/r3_race.txt
: > $O
for so in ab/_C_old_slp.so cassmantle_amd/_C.cpython-310-x86_64-linux-gnu.so; do
  echo "== so=$so  concurrency screen (tools/race_lnk_concurrency.py none c0 conv)" | tee -a $O
  CASSMANTLE_EXT_SO=$PWD/$so timeout -k 10 240 python -u tools/race_lnk_concurrency.py none c0 conv >> $O 2>&1 || exit 1
done
echo "== fix: rows screen ITERS=36 (1440 concurrent runs)" | tee -a $O
ITERS=36 timeout -k 10 300 python -u tools/race_lnk_rows.py >> $O 2>&1 || exit 1
for so in ab/_C_old_slp.so ab/_C_old_noslp.so cassmantle_amd/_C.cpython-310-x86_64-linux-gnu.so; do
  echo "== so=$so determinism, 16-row LNK variant (CASSMANTLE_AREG_LNK16=1; old builds ignore it)" | tee -a $O
  CASSMANTLE_AREG_LNK16=1 CASSMANTLE_EXT_SO=$PWD/$so timeout -k 10 200 python -u tools/race_lnk_determinism.py >> $O 2>&1 || exit 1
done
echo "== tests" | tee -a $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_kernels_gpu.py -k "areg or layer_norm or concurrency" \
  tests/test_models_gpu.py::test_stage_overlap_decode_matches_serial \
  tests/test_models_gpu.py::test_fp8_cross_kv_survives_batch_size_change_under_graphs >> $O 2>&1
rc=$?
tail -5 $O
grep -E "^==|diff|differing|passed|failed" $O | head -60
exit $rc
