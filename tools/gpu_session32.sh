#!/bin/bash
# steps-per-graph sweep with split side/main graphs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for spg in 16 32 64 128; do
  timeout -k 10 180 python bench.py --steps 1280 --warmup 128 --steps_per_graph $spg > gpurun_out/b32.log 2>&1 || { tail -30 gpurun_out/b32.log; exit 1; }
  echo "[$spg] $(tail -1 gpurun_out/b32.log | cut -c100-200)"
done
timeout -k 10 180 python bench.py --steps 1280 --warmup 128 --steps_per_graph 64 --parallelism dp > gpurun_out/b32.log 2>&1 || { tail -30 gpurun_out/b32.log; exit 1; }
echo "[dp 64] $(tail -1 gpurun_out/b32.log | cut -c100-200)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof32 -o s64 -- python bench.py --steps 640 --warmup 128 --steps_per_graph 64 > gpurun_out/p32.log 2>&1 || { tail -30 gpurun_out/p32.log; exit 1; }
