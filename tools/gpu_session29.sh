#!/bin/bash
# regression hunt: bench x2 + kernel-trace profile of the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python bench.py > gpurun_out/b29a.log 2>&1 || { tail -30 gpurun_out/b29a.log; exit 1; }
tail -1 gpurun_out/b29a.log
timeout -k 10 180 python bench.py --steps 1000 --warmup 50 > gpurun_out/b29b.log 2>&1 || { tail -30 gpurun_out/b29b.log; exit 1; }
tail -1 gpurun_out/b29b.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof29 -o single -- python bench.py --steps 200 --warmup 20 > gpurun_out/p29.log 2>&1 || { tail -30 gpurun_out/p29.log; exit 1; }
tail -1 gpurun_out/p29.log
