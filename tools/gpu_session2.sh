#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_fused_kernels_gpu.py tests/test_fused_dp_gpu.py -x -q > gpurun_out/t2.log 2>&1; echo "tests rc $?"; tail -30 gpurun_out/t2.log
timeout -k 10 240 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_fused.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_fused.log; exit 1; }
tail -1 gpurun_out/bench_fused.log
timeout -k 10 240 python bench.py --steps 300 --warmup 30 --batch_size 8192 2>&1 | tail -1
timeout -k 10 240 python bench.py --embedding_update exact --steps 100 --warmup 10 2>&1 | tail -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 > gpurun_out/prof2.log 2>&1; echo "prof rc $?"
