#!/bin/bash
# row-shard engine with 4 ranks sharing one GPU (4-way table split, 3-peer all-to-all pushes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rowshard_gpu.py -k 4ranks -x -v --timeout 300 --timeout-method thread > gpurun_out/t57.log 2>&1 || { tail -40 gpurun_out/t57.log; exit 1; }
tail -3 gpurun_out/t57.log
export ROCFM_BENCH_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29557 bench.py --gpus 4 --parallelism rowshard > gpurun_out/b57g.log 2>&1 || { tail -30 gpurun_out/b57g.log; exit 1; }
echo "[gloo+p2p N=4 rowshard, one GPU] $(grep metric gpurun_out/b57g.log | cut -c1-200)"
