#!/bin/bash
# triage: streamed-vs-per-step equality (twice) + fused kernel tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python -u -m pytest tests/test_estimator_gpu.py -x -q -k streamed --timeout 200 --timeout-method thread > gpurun_out/t36_$i.log 2>&1; echo "run $i rc=$?"; grep -E "Error|passed|failed" gpurun_out/t36_$i.log | head -3
done
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t36k.log 2>&1; echo "kernels rc=$?"; tail -3 gpurun_out/t36k.log
