#!/bin/bash
# whole-step graphs with captured collectives (world=1 nccl via torchrun), fork-order change
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_fused_kernels_gpu.py tests/test_fused_dp_gpu.py tests/test_rowshard_gpu.py -x -q > gpurun_out/t10.log 2>&1; rc=$?; echo "tests rc $rc"; tail -5 gpurun_out/t10.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 240 python bench.py --steps 400 --warmup 40 > gpurun_out/b10_single.log 2>&1 || exit 1; tail -1 gpurun_out/b10_single.log
for par in dp rowshard; do
  timeout -k 10 240 python bench.py --steps 300 --warmup 30 --parallelism $par > gpurun_out/b10_$par.log 2>&1 || exit 1; tail -1 gpurun_out/b10_$par.log
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29544 bench.py --steps 300 --warmup 30 --parallelism $par > gpurun_out/b10_${par}_nccl1.log 2>&1 || exit 1; grep metric gpurun_out/b10_${par}_nccl1.log | tail -1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof10 -o dp -- python bench.py --steps 100 --warmup 10 --parallelism dp > gpurun_out/p10.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof10 -o single -- python bench.py --steps 100 --warmup 10 > gpurun_out/p10s.log 2>&1 || exit 1
