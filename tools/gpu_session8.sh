#!/bin/bash
# multi-WG route; dp and rowshard single-GPU step profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests/test_fused_dp_gpu.py tests/test_rowshard_gpu.py -x -q > gpurun_out/t8.log 2>&1; rc=$?; echo "tests rc $rc"; tail -5 gpurun_out/t8.log
[ $rc -eq 0 ] || exit 1
for par in rowshard dp dense_dp; do
  up=sparse; [ $par = dense_dp ] && up=exact
  timeout -k 10 240 python bench.py --steps 300 --warmup 30 --parallelism $par --embedding_update $up > gpurun_out/b8_$par.log 2>&1 || exit 1; tail -1 gpurun_out/b8_$par.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof8rs -o rs -- python bench.py --steps 100 --warmup 10 --parallelism rowshard > gpurun_out/p8a.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof8dp -o dp -- python bench.py --steps 100 --warmup 10 --parallelism dp > gpurun_out/p8b.log 2>&1 || exit 1
ls -R gpurun_out/prof8rs | head
