#!/bin/bash
# round-end rehearsal: full GPU suite, smoke, N=1 benches (incl. DP at world 1 with recv aliasing send), N=2 gloo+p2p
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t55.log 2>&1 || { tail -40 gpurun_out/t55.log; exit 1; }
tail -1 gpurun_out/t55.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s55.log 2>&1 || { tail -30 gpurun_out/s55.log; exit 1; }
tail -1 gpurun_out/s55.log
for st in "" "--parallelism dp" "--parallelism dp --embedding_update exact"; do
  timeout -k 10 180 python bench.py $st > gpurun_out/b55.log 2>&1 || { tail -30 gpurun_out/b55.log; exit 1; }
  echo "[$st] $(tail -1 gpurun_out/b55.log | cut -c1-200)"
done
export ROCFM_BENCH_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 > gpurun_out/b55g.log 2>&1 || { tail -30 gpurun_out/b55g.log; exit 1; }
echo "[gloo+p2p N=2 default] $(grep metric gpurun_out/b55g.log | cut -c1-260)"
