#!/bin/bash
# Re-entry check after a container rebuild: full GPU suite, smoke, default 1-GPU bench, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t60.log 2>&1 || { tail -40 gpurun_out/t60.log; exit 1; }
tail -1 gpurun_out/t60.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s60.log 2>&1 || { tail -30 gpurun_out/s60.log; exit 1; }
tail -1 gpurun_out/s60.log
timeout -k 10 180 python bench.py > gpurun_out/b60.log 2>&1 || { tail -30 gpurun_out/b60.log; exit 1; }
tail -1 gpurun_out/b60.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof60 -o single -- python bench.py --steps 640 --warmup 128 > gpurun_out/p60.log 2>&1 || { tail -30 gpurun_out/p60.log; exit 1; }
echo done
