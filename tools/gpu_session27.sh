#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_fused_kernels_gpu.py -x -q -k "batch_norm" > gpurun_out/t27a.log 2>&1 || { tail -60 gpurun_out/t27a.log; exit 1; }
tail -3 gpurun_out/t27a.log
timeout -k 10 500 python -m pytest tests/test_fused_kernels_gpu.py tests/test_estimator_gpu.py -x -q > gpurun_out/t27.log 2>&1 || { tail -60 gpurun_out/t27.log; exit 1; }
tail -3 gpurun_out/t27.log
N=4000000 timeout -k 10 600 python tools/train_e2e.py > gpurun_out/e2e27.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/e2e27.log | tail -12; exit $rc
