#!/bin/bash
# round 6: attention masks as real branches (tree) vs the round-5 attention (variants/attn_old.so,
# the masks if-converted into every tile): attention tests, attention micro-bench, SD-1.5 and SDXL
# benches interleaved x2; then the live-round transport A/B (tools/gpu/r6_e.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "attention or attn" -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for v in tree old; do
  so=""; [ $v = old ] && so=variants/attn_old.so
  CASSMANTLE_EXT_SO=$so timeout -k 10 300 python tools/bench_attn.py > $O/attn_$v.jsonl 2> $O/attn_$v.err || { tail -5 $O/attn_$v.err; exit 1; }
done
python - <<'PY'
import json
for v in ("tree", "old"):
    for l in open(f"gpurun_out/r6f/attn_{v}.jsonl"):
        if l.startswith("{"):
            d = json.loads(l); print(v, d["shape"], {k: x for k, x in d["us"].items() if k != "sdpa"})
PY
for rep in 1 2; do
  for v in tree old; do
    so=""; [ $v = old ] && so=variants/attn_old.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-score --no-live --no-sdxl > $O/sd15_${v}_$rep.json 2> $O/sd15_${v}_$rep.err || { tail -5 $O/sd15_${v}_$rep.err; exit 1; }
    echo "sd15 v=$v rep=$rep $(python -c "import json;d=json.load(open('$O/sd15_${v}_$rep.json'));print(d['ms_per_step'], d['batch1_s_per_image'])")"
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 2 --warmup 1 --no-score --no-batch1 --no-live --no-sdxl > $O/sdxl_${v}_$rep.json 2> $O/sdxl_${v}_$rep.err || { tail -5 $O/sdxl_${v}_$rep.err; exit 1; }
    echo "sdxl v=$v rep=$rep $(python -c "import json;d=json.load(open('$O/sdxl_${v}_$rep.json'));print(d['ms_per_step'])")"
  done
done
bash tools/gpu/r6_e.sh
