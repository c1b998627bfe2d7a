set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0).multi_processor_count)" > gpurun_out/devinfo.txt 2>&1
timeout -k 10 600 python bench.py --baseline --steps 2 --warmup 1 > gpurun_out/baseline.json 2> gpurun_out/baseline.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_baseline -o run --output-format csv -- python bench.py --baseline --steps 1 --warmup 1 --denoise-steps 5 --no-score > gpurun_out/baseline_prof.log 2>&1
echo done
