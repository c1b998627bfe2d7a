#!/bin/bash
# round 5: bf16 attention (attn_fwd, d <= 80) with the K fragments of a half read in one batch before
# its MFMA chain (main) vs read-wait-MFMA per k-step (variants/attn_kseq.so, -DATTN_KBATCH=0):
# attention GPU tests, graph-timed probe at the UNet shapes, SD-1.5 bench incl. batch 1 (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5an
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -m gpu -k "attention" -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for v in main kseq main kseq; do
  so=""; [ $v = kseq ] && so=variants/attn_kseq.so
  CASSMANTLE_EXT_SO=$so timeout -k 10 240 python -u tools/probe_attn_overhead.py 2>>$O/err.txt \
    | sed "s/^/{\"v\": \"$v\", \"row\": /; s/\$/}/" >> $O/attn_ab.jsonl || exit 1
done
for rep in 1 2; do
  for v in main kseq; do
    so=""; [ $v = kseq ] && so=variants/attn_kseq.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py > $O/sd15_${v}_$rep.json 2> $O/sd15_${v}_$rep.err || { tail -5 $O/sd15_${v}_$rep.err; exit 1; }
    echo "v=$v rep=$rep $(python -c "import json;d=json.load(open('$O/sd15_${v}_$rep.json'));print(d['ms_per_step'], d['batch1_s_per_image'])")"
  done
done
