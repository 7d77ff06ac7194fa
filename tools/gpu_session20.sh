#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_fused_dp_gpu.py tests/test_rowshard_gpu.py -x -q > gpurun_out/t20.log 2>&1; rc=$?; echo "tests rc $rc"; tail -15 gpurun_out/t20.log
[ $rc -eq 0 ] || exit 1
for par in dp dense_dp; do
  up=sparse; [ $par = dense_dp ] && up=exact
  timeout -k 10 240 python bench.py --steps 640 --warmup 64 --parallelism $par --embedding_update $up > gpurun_out/b20_$par.log 2>&1 || exit 1; tail -1 gpurun_out/b20_$par.log | cut -c1-200
done
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29544 bench.py --steps 640 --warmup 64 --parallelism dp > gpurun_out/b20_dp_nccl1.log 2>&1 || exit 1; grep metric gpurun_out/b20_dp_nccl1.log | tail -1 | cut -c1-200
