#!/bin/bash
# round 5: grouped tile raster (GEMM_RASTER_G=4, variants/rg4.so) vs the in-tree row raster:
# small-GEMM probe warm / cold (rotating 40 weight + activation copies), then the bench x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5f
mkdir -p $O
for v in tree rg4; do
  so=""; [ "$v" != tree ] && so=variants/$v.so
  for rot in 1 40; do
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python tools/probe_small_gemm.py --m 2048 --n 1280 --ks 640,1280,2560 --cfgs 31,26,16,3 --splits 1 --rotate $rot > $O/probe_${v}_r$rot.jsonl 2> $O/probe_${v}_r$rot.err || { tail -20 $O/probe_${v}_r$rot.err; exit 1; }
    echo "$v rot$rot"; grep '"M"' $O/probe_${v}_r$rot.jsonl
  done
done
for rep in 1 2; do
  for v in tree rg4; do
    so=""; [ "$v" != tree ] && so=variants/$v.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-score --no-batch1 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -20 $O/bench_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', $rep, d['ms_per_step'], d['stage_mean_ms'])"
  done
done
