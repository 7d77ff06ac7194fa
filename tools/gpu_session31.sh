#!/bin/bash
# split side/main multi-step graphs: tests, bench (default + long), dp/rowshard benches, profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t31.log 2>&1 || { tail -60 gpurun_out/t31.log; exit 1; }
tail -2 gpurun_out/t31.log
for st in "" "--steps 1600 --warmup 32" "--parallelism dp" "--parallelism rowshard"; do
  timeout -k 10 180 python bench.py $st > gpurun_out/b31.log 2>&1 || { tail -30 gpurun_out/b31.log; exit 1; }
  echo "[$st] $(tail -1 gpurun_out/b31.log | cut -c1-230)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof31 -o single -- python bench.py --steps 320 --warmup 32 > gpurun_out/p31.log 2>&1 || { tail -30 gpurun_out/p31.log; exit 1; }
