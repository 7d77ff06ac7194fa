#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_fused_kernels_gpu.py tests/test_fused_dp_gpu.py -x -q > gpurun_out/t5.log 2>&1; rc=$?; echo "tests rc $rc"; tail -15 gpurun_out/t5.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/diag_phases.py > gpurun_out/diag5.log 2>&1; echo "diag rc $?"; grep -v amdgpu.ids gpurun_out/diag5.log
timeout -k 10 240 python bench.py --steps 400 --warmup 40 2>&1 | tail -1
timeout -k 10 240 python bench.py --steps 400 --warmup 40 --batch_size 8192 2>&1 | tail -1
