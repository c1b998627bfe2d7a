set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_profile.sh sd15 sd15 10 24 && \
bash tools/gpu_profile.sh sdxl_bf16 sdxl 4 8 --batch 1 && \
bash tools/gpu_profile.sh sdxl_fp8 sdxl 4 8 --batch 1 --fp8-attention && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_r3_start.log 2>&1; tail -c 1500 gpurun_out/bench_r3_start.log
