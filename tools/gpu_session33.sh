#!/bin/bash
# p2p push exchange: unit tests (2 procs on 1 GPU), DP equality incl. p2p multi-step graphs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_p2p_gpu.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/t33a.log 2>&1 || { tail -60 gpurun_out/t33a.log; exit 1; }
grep -E "rank|passed|failed" gpurun_out/t33a.log | tail -6
timeout -k 10 400 python -u -m pytest tests/test_fused_dp_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t33b.log 2>&1 || { tail -60 gpurun_out/t33b.log; exit 1; }
tail -8 gpurun_out/t33b.log
