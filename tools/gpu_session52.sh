#!/bin/bash
# phase stamps of the current kernels; DP (sparse / exact) step profiles at world 1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python tools/diag_phases.py > gpurun_out/d52.log 2>&1 || { tail -30 gpurun_out/d52.log; exit 1; }
cat gpurun_out/d52.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof52 -o dp -- python bench.py --steps 640 --warmup 128 --parallelism dp > gpurun_out/p52a.log 2>&1 || { tail -30 gpurun_out/p52a.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof52 -o dpx -- python bench.py --steps 640 --warmup 128 --parallelism dp --embedding_update exact > gpurun_out/p52b.log 2>&1 || { tail -30 gpurun_out/p52b.log; exit 1; }
echo done
