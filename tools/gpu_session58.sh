#!/bin/bash
# DP step profile at world 1 after the recv/send alias (no exchange copy)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof58 -o dp -- python bench.py --steps 640 --warmup 128 --parallelism dp > gpurun_out/p58a.log 2>&1 || { tail -30 gpurun_out/p58a.log; exit 1; }
tail -1 gpurun_out/p58a.log | cut -c1-200
echo done
