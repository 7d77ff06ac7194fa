#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_fused_kernels_gpu.py -x -q > gpurun_out/t25.log 2>&1; rc=$?; echo "tests rc $rc"; tail -25 gpurun_out/t25.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 240 python bench.py --steps 640 --warmup 64 --compute_dtype fp8 > gpurun_out/b25.log 2>&1 || exit 1; tail -1 gpurun_out/b25.log | cut -c1-260
