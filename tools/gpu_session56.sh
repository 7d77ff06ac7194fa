#!/bin/bash
# 4 ranks sharing one GPU: p2p fan-out to 3 peers + 4-way merge (the W>2 paths of the 8-GPU node)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_dp_gpu.py -k world4 -x -v --timeout 300 --timeout-method thread > gpurun_out/t56.log 2>&1 || { tail -40 gpurun_out/t56.log; exit 1; }
tail -3 gpurun_out/t56.log
export ROCFM_BENCH_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29556 bench.py --gpus 4 > gpurun_out/b56g.log 2>&1 || { tail -30 gpurun_out/b56g.log; exit 1; }
echo "[gloo+p2p N=4 default, one GPU] $(grep metric gpurun_out/b56g.log | cut -c1-400)"
