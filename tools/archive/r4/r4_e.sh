#!/bin/bash
# GroupNorm+SiLU A-prologue cost probe: the ResNet convs with and without the probe (same box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu/so_ab.sh apro shape us "python tools/bench_resnet_convs.py" tree apro || exit 1
bash tools/gpu/so_ab.sh gnap shape us "python tools/bench_membound.py --gn-only" tree || exit 1
