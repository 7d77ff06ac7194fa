#!/bin/bash
# A/B: HEAD vs HEAD~1 (pre batch_norm) row kernel / step time
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for d in . wt_old; do
  for st in "--steps 1600 --warmup 32" "--steps 200 --warmup 20"; do
    (cd $d && timeout -k 10 180 python bench.py $st) > gpurun_out/b30.log 2>&1 || { tail -30 gpurun_out/b30.log; exit 1; }
    echo "$d $st $(tail -1 gpurun_out/b30.log | cut -c1-200)"
  done
done
(cd wt_old && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof30 -o old -- python bench.py --steps 320 --warmup 32) > gpurun_out/p30.log 2>&1 || { tail -30 gpurun_out/p30.log; exit 1; }
