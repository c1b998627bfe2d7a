#!/bin/bash
# round 6: what share of a small-K GEMM is its epilogue?  tree vs variants/noepi.so (GEMM_DIAG_NOEPI:
# the tile epilogue skipped, results wrong), tools/probe_small_gemm.py, same box x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6u
mkdir -p $O
for rep in 1 2; do
  for v in tree noepi; do
    so=""; [ $v = noepi ] && so=variants/noepi.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 200 python tools/probe_small_gemm.py --m 32768 --n 320 --ks 320,640,1280 --cfgs 20 --splits 1 --rotate 8 > $O/pp_${v}_$rep.jsonl 2> $O/pp_${v}_$rep.err || { tail -5 $O/pp_${v}_$rep.err; exit 1; }
    CASSMANTLE_EXT_SO=$so timeout -k 10 200 python tools/probe_small_gemm.py --m 2048 --n 1280 --ks 320,640,1280 --cfgs 31 --splits 1 --rotate 8 > $O/d31_${v}_$rep.jsonl 2> $O/d31_${v}_$rep.err || { tail -5 $O/d31_${v}_$rep.err; exit 1; }
    echo "== $v $rep"; grep -h '"M"' $O/pp_${v}_$rep.jsonl $O/d31_${v}_$rep.jsonl
  done
done
