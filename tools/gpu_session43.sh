#!/bin/bash
# embedding update: run heads own their row's optimizer with phase-1 table loads
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t43.log 2>&1 || { tail -40 gpurun_out/t43.log; exit 1; }
tail -1 gpurun_out/t43.log
for st in "" "--parallelism dp" "--optimizer Adagrad" "--optimizer ftrl"; do
  timeout -k 10 180 python bench.py $st > gpurun_out/b43.log 2>&1 || { tail -30 gpurun_out/b43.log; exit 1; }
  echo "[$st] $(tail -1 gpurun_out/b43.log | cut -c80-200)"
done
timeout -k 10 200 python tools/diag_phases.py > gpurun_out/diag43.log 2>&1 || { tail -30 gpurun_out/diag43.log; exit 1; }
grep -v amdgpu.ids gpurun_out/diag43.log | tail -6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof43 -o single -- python bench.py --steps 640 --warmup 128 > gpurun_out/p43.log 2>&1 || { tail -30 gpurun_out/p43.log; exit 1; }
