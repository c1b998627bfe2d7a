#!/bin/bash
# Same-box interleaved A/B of extension builds: runs CMD once per .so per repetition (the in-tree
# build is "tree"; others are variants/NAME.so from tools/build_variant.py) and prints a table of
# the JSON field FIELD keyed by KEY (tools/ab_table.py).
#   tools/gpu/so_ab.sh TAG KEY FIELD "CMD" tree v1 v2 ...
set -o pipefail
tag=$1; key=$2; field=$3; cmd=$4; shift 4
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    so=""; [ "$v" != tree ] && so=variants/$v.so
    CASSMANTLE_EXT_SO=$so timeout -k 10 300 $cmd > gpurun_out/${tag}_${v}_$rep.jsonl 2> gpurun_out/${tag}_${v}_$rep.err || { tail -5 gpurun_out/${tag}_${v}_$rep.err; exit 1; }
  done
done
python tools/ab_table.py "$key" "$field" gpurun_out/${tag} "$@" | tee gpurun_out/${tag}_table.txt
