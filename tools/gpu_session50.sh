#!/bin/bash
# exact mode: step-tagged touched rows (dense update reads/clears gradient rows only where written)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t50.log 2>&1 || { tail -40 gpurun_out/t50.log; exit 1; }
tail -1 gpurun_out/t50.log
for st in "--embedding_update exact" "--embedding_update exact --parallelism dense_dp" "--embedding_update exact --parallelism rowshard"; do
  timeout -k 10 180 python bench.py $st > gpurun_out/b50.log 2>&1 || { tail -30 gpurun_out/b50.log; exit 1; }
  echo "[$st] $(tail -1 gpurun_out/b50.log | cut -c80-200)"
done
