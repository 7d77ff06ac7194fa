#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_fused_kernels_gpu.py tests/test_fused_dp_gpu.py -x -q > gpurun_out/t19.log 2>&1; rc=$?; echo "tests rc $rc"; tail -15 gpurun_out/t19.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/diag_phases.py > gpurun_out/diag19.log 2>&1 || exit 1; grep -v amdgpu gpurun_out/diag19.log | tail -22
timeout -k 10 240 python bench.py --steps 640 --warmup 64 > gpurun_out/b19.log 2>&1 || exit 1; tail -1 gpurun_out/b19.log | cut -c1-200
