#!/bin/bash
# round 6: (1) fp8 attention with the P.V MFMAs software-pipelined into the next step (tree) vs
# F8_PIPE=0 (variants/f8_nopipe.so): attention tests, micro-bench, SDXL x2 interleaved;
# (2) supervised live round: ipc landing by DMA to pinned host (default) vs device landing vs pipe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_parallel_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu \
  -k "attention or attn or ipc" -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for v in tree nopipe; do
  so=""; [ $v = nopipe ] && so=variants/f8_nopipe.so
  CASSMANTLE_EXT_SO=$so timeout -k 10 300 python tools/bench_attn.py --only-d 64 > $O/attn_$v.jsonl 2> $O/attn_$v.err || { tail -5 $O/attn_$v.err; exit 1; }
  python -c "
import json
for l in open('$O/attn_$v.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print('$v', d['shape'], {k: x for k, x in d['us'].items() if k != 'sdpa'})"
done
for rep in 1 2; do
  for v in tree nopipe; do
    so=""; [ $v = nopipe ] && so=variants/f8_nopipe.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 3 --warmup 1 --no-score --no-batch1 --no-live --no-sdxl > $O/sdxl_${v}_$rep.json 2> $O/sdxl_${v}_$rep.err || { tail -5 $O/sdxl_${v}_$rep.err; exit 1; }
    echo "sdxl v=$v rep=$rep $(python -c "import json;d=json.load(open('$O/sdxl_${v}_$rep.json'));print(d['ms_per_step'])")"
  done
done
for rep in 1 2; do
  for v in host device pipe; do
    t=ipc; [ $v = pipe ] && t=pipe
    l=host; [ $v = device ] && l=device
    timeout -k 10 300 python tools/bench_live.py --gpus 1 --transport $t --land $l --seconds 15 --idle-s 3 > $O/live_${v}_$rep.json 2> $O/live_${v}_$rep.err || { tail -20 $O/live_${v}_$rep.err; exit 1; }
    echo "live v=$v rep=$rep $(python -c "import json;d=json.loads(open('$O/live_${v}_$rep.json').read().strip().splitlines()[-1]);print(d['images_per_s'], d['load_p50_ms'], d['load_p99_ms'], d.get('transport'), d.get('land_us_p50'), d['rounds'])")"
  done
done
