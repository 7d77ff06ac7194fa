#!/bin/bash
# merge_apply with one-wave workgroups and no loads for absent ranks: DP tests (world 1/2/4) + DP bench + profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fused_dp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t59.log 2>&1 || { tail -40 gpurun_out/t59.log; exit 1; }
tail -1 gpurun_out/t59.log
for st in "--parallelism dp" "--parallelism dp --embedding_update exact"; do
  timeout -k 10 180 python bench.py $st > gpurun_out/b59.log 2>&1 || { tail -30 gpurun_out/b59.log; exit 1; }
  echo "[$st] $(tail -1 gpurun_out/b59.log | cut -c150-260)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof59 -o dp -- python bench.py --steps 640 --warmup 128 --parallelism dp > gpurun_out/p59a.log 2>&1 || { tail -30 gpurun_out/p59a.log; exit 1; }
echo done
