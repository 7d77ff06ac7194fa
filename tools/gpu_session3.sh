#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_fused_kernels_gpu.py tests/test_fused_dp_gpu.py -x -q > gpurun_out/t3.log 2>&1; rc=$?; echo "tests rc $rc"; tail -30 gpurun_out/t3.log
[ $rc -eq 0 ] || exit 1
for spg in 1 8; do timeout -k 10 240 python bench.py --steps 400 --warmup 40 --steps_per_graph $spg 2>&1 | tail -1; done
timeout -k 10 240 python bench.py --steps 400 --warmup 40 --batch_size 8192 2>&1 | tail -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 20 > gpurun_out/prof3.log 2>&1; echo "prof rc $?"
