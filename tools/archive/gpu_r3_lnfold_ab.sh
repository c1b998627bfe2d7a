set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_ab_env.sh gpurun_out/r3_ab_lnfold_sdxl.txt 2 "--model sdxl --batch 1 --steps 2" "CASSMANTLE_LN_FOLD_MODE=1" "CASSMANTLE_LN_FOLD_MODE=2" && \
bash tools/gpu_ab_env.sh gpurun_out/r3_ab_lnfold_sd15.txt 2 "--steps 4" "CASSMANTLE_LN_FOLD_MODE=1" "CASSMANTLE_LN_FOLD_MODE=2"
