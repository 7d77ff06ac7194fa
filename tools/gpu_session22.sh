#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_rowshard_gpu.py -x -q > gpurun_out/t22.log 2>&1; rc=$?; echo "tests rc $rc"; tail -15 gpurun_out/t22.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 240 python bench.py --steps 640 --warmup 64 --parallelism rowshard > gpurun_out/b22_rs.log 2>&1 || exit 1; tail -1 gpurun_out/b22_rs.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 320 --warmup 32 --parallelism rowshard --feature_size 100000000 > gpurun_out/b22_rs100m.log 2>&1 || exit 1; tail -1 gpurun_out/b22_rs100m.log | cut -c1-200
