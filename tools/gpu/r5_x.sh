#!/bin/bash
# round 5: cold in-situ re-tune of the SDXL pass (batch 1); only its conv keys (SDXL-only shapes)
# are kept (filter below), then same-box A/B current vs filtered table: SDXL + SD-1.5 (x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5x; mkdir -p $O
cp cassmantle_amd/ops/gemm_tuning.json $O/tune_cur.json
cp cassmantle_amd/ops/gemm_tuning.json $O/tune_raw.json
timeout -k 10 900 python -u tools/autotune_gemm.py --models sdxl --batch 1 --merge --cold 512 --out $O/tune_raw.json > $O/autotune_sdxl.jsonl 2> $O/autotune_sdxl.err || { tail -5 $O/autotune_sdxl.err; exit 1; }
tail -1 $O/autotune_sdxl.jsonl
python - <<'PY'
import json
O = "gpurun_out/r5x"
cur = {e["key"]: e for e in json.load(open(f"{O}/tune_cur.json"))["entries"]}
raw = json.load(open(f"{O}/tune_raw.json"))
out = dict(cur)
n = 0
for e in raw["entries"]:
    k = e["key"]
    if " c1:" in k and (k not in cur or (cur[k]["cfg"], cur[k]["split"]) != (e["cfg"], e["split"])):
        out[k] = dict(e, model="sdxl-cold")
        n += 1
raw["entries"] = sorted(out.values(), key=lambda e: e["key"])
json.dump(raw, open(f"{O}/tune_new.json", "w"), indent=1)
print("conv keys changed / added:", n)
PY
for rep in 1 2; do
  for t in cur new; do
    CASSMANTLE_GEMM_TUNE_PATH=$O/tune_$t.json timeout -k 10 300 python bench.py --model sdxl --fp8-attention --batch 1 --steps 2 --warmup 1 --no-score --no-batch1 > $O/sdxl_${t}_$rep.json 2> $O/sdxl_${t}_$rep.err || { tail -5 $O/sdxl_${t}_$rep.err; exit 1; }
    python -c "import json;a=json.load(open('$O/sdxl_${t}_$rep.json'));print('rep $rep table $t sdxl ms_per_step', a['ms_per_step'])"
  done
done
for t in cur new; do
  CASSMANTLE_GEMM_TUNE_PATH=$O/tune_$t.json timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-score > $O/sd15_${t}.json 2> $O/sd15_${t}.err || { tail -5 $O/sd15_${t}.err; exit 1; }
  python -c "import json;a=json.load(open('$O/sd15_${t}.json'));print('table $t sd15 ms_per_step', a['ms_per_step'], 'batch1', a.get('batch1_s_per_image'))"
done
