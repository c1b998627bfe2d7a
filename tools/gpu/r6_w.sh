#!/bin/bash
# round 6: weight-operand LDS-DMA with the nt cache policy (variants/wnt.so, GEMM_W_CPOL=2) vs the tree:
# small-K probe + bench, same box x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6w
mkdir -p $O
timeout -k 10 300 env CASSMANTLE_EXT_SO=variants/wnt.so python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "gemm or conv or linear" -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  for v in tree wnt; do
    so=""; [ $v = wnt ] && so=variants/wnt.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 200 python tools/probe_small_gemm.py --m 32768 --n 320 --ks 320,1280 --cfgs 20 --splits 1 --rotate 8 > $O/pp_${v}_$rep.jsonl 2> $O/pp_${v}_$rep.err || { tail -5 $O/pp_${v}_$rep.err; exit 1; }
    CASSMANTLE_EXT_SO=$so timeout -k 10 200 python tools/probe_small_gemm.py --m 2048 --n 1280 --ks 1280 --cfgs 31 --splits 1 --rotate 8 > $O/d31_${v}_$rep.jsonl 2> $O/d31_${v}_$rep.err || { tail -5 $O/d31_${v}_$rep.err; exit 1; }
    echo "== $v $rep"; grep -h '"M"' $O/pp_${v}_$rep.jsonl $O/d31_${v}_$rep.jsonl
  done
done
for rep in 1 2; do
  for v in tree wnt; do
    so=""; [ $v = wnt ] && so=variants/wnt.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-score --no-live --no-sdxl > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -20 $O/bench_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', $rep, d['ms_per_step'], d['batch1_s_per_image'], d['stage_mean_ms'])"
  done
done
