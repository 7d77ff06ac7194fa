#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_fused_kernels_gpu.py tests/test_fused_dp_gpu.py -x -q > gpurun_out/t21.log 2>&1; rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/t21.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 320 --warmup 32 --feature_size 100000000 > gpurun_out/b21_100m.log 2>&1 || exit 1; tail -1 gpurun_out/b21_100m.log | cut -c1-330
timeout -k 10 500 python bench.py --steps 320 --warmup 32 --feature_size 1000000000 > gpurun_out/b21_1b.log 2>&1 || exit 1; tail -1 gpurun_out/b21_1b.log | cut -c1-330
rocm-smi --showmeminfo vram 2>/dev/null | head -5 || true
