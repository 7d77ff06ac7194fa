#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_fused_kernels_gpu.py tests/test_estimator_gpu.py -x -q > gpurun_out/t26.log 2>&1 || { tail -40 gpurun_out/t26.log; exit 1; }
tail -3 gpurun_out/t26.log
N=4000000 timeout -k 10 600 python tools/train_e2e.py > gpurun_out/e2e26.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/e2e26.log | tail -12; exit $rc
