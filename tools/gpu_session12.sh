#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_fused_dp_gpu.py tests/test_rowshard_gpu.py -x -q > gpurun_out/t12.log 2>&1; rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/t12.log
[ $rc -eq 0 ] || exit 1
for par in dp rowshard; do
  timeout -k 10 240 python bench.py --steps 400 --warmup 40 --parallelism $par > gpurun_out/b12_$par.log 2>&1 || exit 1; tail -1 gpurun_out/b12_$par.log | cut -c1-200
done
timeout -k 10 240 python bench.py --steps 400 --warmup 40 > gpurun_out/b12_single.log 2>&1 || exit 1; tail -1 gpurun_out/b12_single.log | cut -c1-200
