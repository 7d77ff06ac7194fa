#!/bin/bash
# 1-GPU bench matrix after the re-entry build: engines, update modes, optimizers, parallelism at world 1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/m61.jsonl
for st in "" "--embedding_update exact" "--optimizer Adagrad" "--optimizer ftrl" "--optimizer Momentum" \
          "--parallelism dp" "--parallelism dense_dp --embedding_update exact" "--parallelism rowshard" \
          "--batch_size 4096" "--engine torch --steps 50"; do
  timeout -k 10 180 python bench.py $st > gpurun_out/b61.log 2>&1 || { tail -30 gpurun_out/b61.log; exit 1; }
  echo "{\"flags\": \"$st\", \"result\": $(tail -1 gpurun_out/b61.log)}" >> gpurun_out/m61.jsonl
  echo "[$st] $(tail -1 gpurun_out/b61.log | cut -c100-200)"
done
echo done
