#!/bin/bash
# row-shard over p2p push exchanges (X1-X3 all-to-all, X4 all-gather+sum): tests + rehearsals
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rowshard_gpu.py tests/test_fused_dp_gpu.py tests/test_p2p_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t46.log 2>&1 || { tail -50 gpurun_out/t46.log; exit 1; }
tail -1 gpurun_out/t46.log
timeout -k 10 180 python bench.py --parallelism rowshard > gpurun_out/b46.log 2>&1 || { tail -30 gpurun_out/b46.log; exit 1; }
echo "[rowshard 1] $(tail -1 gpurun_out/b46.log | cut -c80-200)"
for x in p2p rccl; do
ROCFM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 320 --warmup 64 --parallelism rowshard --dp_exchange $x > gpurun_out/b46_2.log 2>&1 || { tail -30 gpurun_out/b46_2.log; exit 1; }
echo "[gloo+$x rowshard N=2] $(tail -1 gpurun_out/b46_2.log | cut -c80-200)"
done
