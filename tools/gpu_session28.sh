#!/bin/bash
# full GPU regression after container re-creation: gpu tests, smoke, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t28.log 2>&1 || { tail -60 gpurun_out/t28.log; exit 1; }
tail -5 gpurun_out/t28.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke28.log 2>&1 || { tail -30 gpurun_out/smoke28.log; exit 1; }
tail -2 gpurun_out/smoke28.log
timeout -k 10 180 python bench.py > gpurun_out/bench28.log 2>&1 || { tail -30 gpurun_out/bench28.log; exit 1; }
tail -3 gpurun_out/bench28.log
