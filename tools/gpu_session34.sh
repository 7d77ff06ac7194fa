#!/bin/bash
# DP over the p2p push: equality tests + N>1 bench rehearsal (ranks share the one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_dp_gpu.py tests/test_p2p_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t34.log 2>&1 || { tail -60 gpurun_out/t34.log; exit 1; }
tail -2 gpurun_out/t34.log
for g in 2 4; do
  ROCFM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus $g --steps 640 --warmup 64 > gpurun_out/b34_$g.log 2>&1 || { tail -30 gpurun_out/b34_$g.log; exit 1; }
  echo "[gloo+p2p N=$g] $(tail -1 gpurun_out/b34_$g.log | cut -c80-330)"
done
