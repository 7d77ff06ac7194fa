#!/bin/bash
# merge kernels (dp + rowshard), N>1 bench rehearsal over gloo on one GPU, rowshard profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests/test_fused_dp_gpu.py tests/test_rowshard_gpu.py -x -q > gpurun_out/t7.log 2>&1; rc=$?; echo "tests rc $rc"; tail -25 gpurun_out/t7.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 240 python bench.py --steps 200 --warmup 20 --parallelism rowshard > gpurun_out/b7_rs1.log 2>&1 || exit 1; tail -1 gpurun_out/b7_rs1.log
ROCFM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/b7_dp2_gloo.log 2>&1 || exit 1; tail -1 gpurun_out/b7_dp2_gloo.log
ROCFM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --parallelism rowshard > gpurun_out/b7_rs2_gloo.log 2>&1 || exit 1; tail -1 gpurun_out/b7_rs2_gloo.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof7 -o rs -- python bench.py --steps 100 --warmup 10 --parallelism rowshard > gpurun_out/p7.log 2>&1 || exit 1; tail -1 gpurun_out/p7.log
ls -R gpurun_out/prof7 | head -20
