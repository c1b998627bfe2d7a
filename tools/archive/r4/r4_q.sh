#!/bin/bash
# live round, same box: in-process topology vs supervised topology (front-end scorer process + worker
# process), and the supervised one with a normal-priority scorer stream
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_live.py --players 64 --seconds 25 --idle-s 6 > gpurun_out/r4q_inproc.json 2> gpurun_out/r4q_inproc.err || { tail -20 gpurun_out/r4q_inproc.err; exit 1; }
grep '^{' gpurun_out/r4q_inproc.json
timeout -k 10 400 python tools/bench_live.py --gpus 1 --players 64 --seconds 25 --idle-s 6 > gpurun_out/r4q_sup.json 2> gpurun_out/r4q_sup.err || { tail -20 gpurun_out/r4q_sup.err; exit 1; }
grep '^{' gpurun_out/r4q_sup.json
timeout -k 10 400 python tools/bench_live.py --gpus 1 --players 64 --seconds 25 --idle-s 6 --no-priority > gpurun_out/r4q_sup_np.json 2> gpurun_out/r4q_sup_np.err || { tail -20 gpurun_out/r4q_sup_np.err; exit 1; }
grep '^{' gpurun_out/r4q_sup_np.json
