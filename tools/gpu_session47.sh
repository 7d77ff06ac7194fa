#!/bin/bash
# re-measure BASELINE configs 4/5 with the current kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for st in "--feature_size 100000000" "--feature_size 100000000 --parallelism rowshard" "--parallelism rowshard" "--feature_size 1000000000"; do
  timeout -k 10 400 python bench.py $st > gpurun_out/b47.log 2>&1 || { tail -30 gpurun_out/b47.log; exit 1; }
  echo "[$st] $(tail -1 gpurun_out/b47.log | cut -c80-200)"
done
