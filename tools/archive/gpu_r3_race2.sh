#!/bin/bash
# LNK race screen, step 2: LayerNorm prologue in scalar fp32 (no v_pk_* before the first DMA),
# SLP on for the rest of the file
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out/r3_race2.txt
: > $O
echo "== concurrency screen x2" | tee -a $O
timeout -k 10 240 python -u tools/race_lnk_concurrency.py none c0 conv >> $O 2>&1 || exit 1
timeout -k 10 240 python -u tools/race_lnk_concurrency.py c0 conv >> $O 2>&1 || exit 1
echo "== rows screen ITERS=36 (1440 concurrent runs)" | tee -a $O
ITERS=36 timeout -k 10 300 python -u tools/race_lnk_rows.py >> $O 2>&1 || exit 1
grep -E "^==|diff|differing|iter" $O | head -60
