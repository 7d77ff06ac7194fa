#!/bin/bash
# DP exact update over the sparse exchange; p2p push publish recipe
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t51.log 2>&1 || { tail -40 gpurun_out/t51.log; exit 1; }
tail -1 gpurun_out/t51.log
for st in "" "--embedding_update exact --parallelism dp" "--parallelism dp"; do
  timeout -k 10 180 python bench.py $st > gpurun_out/b51.log 2>&1 || { tail -30 gpurun_out/b51.log; exit 1; }
  echo "[$st] $(tail -1 gpurun_out/b51.log | cut -c1-220)"
done
export ROCFM_BENCH_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --embedding_update exact > gpurun_out/b51g.log 2>&1 || { tail -30 gpurun_out/b51g.log; exit 1; }
echo "[gloo+p2p N=2 exact] $(grep metric gpurun_out/b51g.log | cut -c1-220)"
