#!/bin/bash
# step-merge_apply early table loads, shard_serve without scratch: dp/rowshard tests, dp benches, dp profile, p2p N=2 rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t42.log 2>&1 || { tail -40 gpurun_out/t42.log; exit 1; }
tail -1 gpurun_out/t42.log
for st in "--parallelism dp" "--parallelism rowshard"; do
  timeout -k 10 180 python bench.py $st > gpurun_out/b42.log 2>&1 || { tail -30 gpurun_out/b42.log; exit 1; }
  echo "[$st] $(tail -1 gpurun_out/b42.log | cut -c80-200)"
done
ROCFM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 640 --warmup 64 > gpurun_out/b42_2.log 2>&1 || { tail -30 gpurun_out/b42_2.log; exit 1; }
echo "[gloo+p2p N=2] $(tail -1 gpurun_out/b42_2.log | cut -c80-200)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof42 -o dp -- python bench.py --steps 640 --warmup 128 --parallelism dp > gpurun_out/p42.log 2>&1 || { tail -30 gpurun_out/p42.log; exit 1; }
