#!/bin/bash
# kernel trace of the fp8 attention calls: pack kernel vs attention kernel time
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for op in "attn8 2 4096 10 64" "attn8 2 1024 20 64" "attn 2 4096 10 64" "attn 2 1024 20 64"; do
  tag=$(echo $op | tr ' ' '_')
  ITERS=20 timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${tag} -o run -- python tools/one_op.py $op > gpurun_out/kt_${tag}.log 2>&1 || exit 1
done
echo KTDONE
