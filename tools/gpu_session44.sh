#!/bin/bash
# FTRL sqrt special case, p2p spin bounds, estimator save barrier: full suite + benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t44.log 2>&1 || { tail -40 gpurun_out/t44.log; exit 1; }
tail -1 gpurun_out/t44.log
for st in "--optimizer ftrl" "--optimizer Momentum" "--optimizer GD"; do
  timeout -k 10 180 python bench.py $st > gpurun_out/b44.log 2>&1 || { tail -30 gpurun_out/b44.log; exit 1; }
  echo "[$st] $(tail -1 gpurun_out/b44.log | cut -c80-200)"
done
ROCFM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 640 --warmup 64 > gpurun_out/b44_2.log 2>&1 || { tail -30 gpurun_out/b44_2.log; exit 1; }
echo "[gloo+p2p N=2] $(tail -1 gpurun_out/b44_2.log | cut -c80-200)"
