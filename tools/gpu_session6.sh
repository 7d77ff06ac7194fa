#!/bin/bash
# row-shard validation + baseline measurements
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_rowshard_gpu.py -x -q > gpurun_out/t6.log 2>&1; rc=$?; echo "rowshard tests rc $rc"; tail -25 gpurun_out/t6.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 240 python bench.py --steps 400 --warmup 40 > gpurun_out/b6_dp1.log 2>&1 || exit 1; tail -1 gpurun_out/b6_dp1.log
timeout -k 10 240 python bench.py --steps 200 --warmup 20 --parallelism rowshard > gpurun_out/b6_rs1.log 2>&1 || exit 1; tail -1 gpurun_out/b6_rs1.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --parallelism rowshard --feature_size 100000000 > gpurun_out/b6_rs100m.log 2>&1 || exit 1; tail -1 gpurun_out/b6_rs100m.log
timeout -k 10 240 python bench.py --steps 100 --warmup 10 --engine torch > gpurun_out/b6_torch_sparse.log 2>&1 || exit 1; tail -1 gpurun_out/b6_torch_sparse.log
timeout -k 10 240 python bench.py --steps 100 --warmup 10 --engine torch --embedding_update exact > gpurun_out/b6_torch_exact.log 2>&1 || exit 1; tail -1 gpurun_out/b6_torch_exact.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --engine torch --parallelism rowshard --feature_size 100000000 > gpurun_out/b6_torch_rs100m.log 2>&1 || exit 1; tail -1 gpurun_out/b6_torch_rs100m.log
