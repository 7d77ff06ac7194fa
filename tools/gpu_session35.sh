#!/bin/bash
# emb-update row prefetch + DP union-list merge: full gpu suite, benches, dp profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t35.log 2>&1 || { tail -60 gpurun_out/t35.log; exit 1; }
tail -2 gpurun_out/t35.log
for st in "" "--parallelism dp" ; do
  timeout -k 10 180 python bench.py --steps 1280 --warmup 128 $st > gpurun_out/b35.log 2>&1 || { tail -30 gpurun_out/b35.log; exit 1; }
  echo "[$st] $(tail -1 gpurun_out/b35.log | cut -c80-200)"
done
ROCFM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 640 --warmup 64 > gpurun_out/b35_2.log 2>&1 || { tail -30 gpurun_out/b35_2.log; exit 1; }
echo "[gloo+p2p N=2] $(tail -1 gpurun_out/b35_2.log | cut -c80-200)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof35 -o dp -- python bench.py --steps 640 --warmup 128 --parallelism dp > gpurun_out/p35.log 2>&1 || { tail -30 gpurun_out/p35.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof35 -o single -- python bench.py --steps 640 --warmup 128 > gpurun_out/p35b.log 2>&1 || { tail -30 gpurun_out/p35b.log; exit 1; }
