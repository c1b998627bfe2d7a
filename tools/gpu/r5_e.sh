#!/bin/bash
# round 5: batch-size efficiency curve of the SD-1.5 step (images per room 1/2/4/8), the current
# SDXL fp8 number, and the PyTorch-eager SDXL baseline (BASELINE config 4's comparison row)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5e
mkdir -p $O
for b in 1 2 4 8; do
  timeout -k 10 300 python bench.py --batch $b --steps 3 --warmup 1 --no-score --no-batch1 > $O/b$b.json 2> $O/b$b.err || { tail -20 $O/b$b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b$b.json'));print($b, d['ms_per_step'], d['stage_mean_ms'])"
done
timeout -k 10 400 python bench.py --model sdxl --fp8-attention --batch 1 --steps 3 --warmup 1 --no-score --no-batch1 > $O/sdxl.json 2> $O/sdxl.err || { tail -20 $O/sdxl.err; exit 1; }
python -c "import json;d=json.load(open('$O/sdxl.json'));print('sdxl fp8', d['ms_per_step'], d['stage_mean_ms'])"
timeout -k 10 600 python bench.py --model sdxl --baseline --batch 1 --steps 1 --warmup 1 --no-score --no-batch1 > $O/sdxl_eager.json 2> $O/sdxl_eager.err || { tail -20 $O/sdxl_eager.err; exit 1; }
python -c "import json;d=json.load(open('$O/sdxl_eager.json'));print('sdxl eager', d['ms_per_step'], d['stage_mean_ms'])"
