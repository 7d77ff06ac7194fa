#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_fused_kernels_gpu.py -x -q > gpurun_out/t15.log 2>&1; rc=$?; echo "tests rc $rc"; tail -15 gpurun_out/t15.log
[ $rc -eq 0 ] || exit 1
for spg in 8 16 32; do
timeout -k 10 240 python bench.py --steps 640 --warmup 64 --steps_per_graph $spg > gpurun_out/b15_$spg.log 2>&1 || exit 1; tail -1 gpurun_out/b15_$spg.log | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof15 -o single -- python bench.py --steps 160 --warmup 32 --steps_per_graph 16 > gpurun_out/p15s.log 2>&1 || exit 1
