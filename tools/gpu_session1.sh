#!/bin/bash
# first measurement session: fused bench, eager baselines, rocprof kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_fused.log 2>&1 || { echo "fused bench failed"; tail -30 gpurun_out/bench_fused.log; exit 1; }
cat gpurun_out/bench_fused.log
timeout -k 10 240 python bench.py --steps 300 --warmup 30 --batch_size 8192 > gpurun_out/bench_fused_b8k.log 2>&1; tail -2 gpurun_out/bench_fused_b8k.log
timeout -k 10 240 python bench.py --engine torch --steps 50 --warmup 5 > gpurun_out/bench_torch_sparse.log 2>&1; tail -2 gpurun_out/bench_torch_sparse.log
timeout -k 10 240 python bench.py --engine torch --embedding_update exact --steps 30 --warmup 5 > gpurun_out/bench_torch_exact.log 2>&1; tail -2 gpurun_out/bench_torch_exact.log
timeout -k 10 240 python bench.py --embedding_update exact --steps 100 --warmup 10 > gpurun_out/bench_fused_exact.log 2>&1; tail -2 gpurun_out/bench_fused_exact.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 > gpurun_out/prof1.log 2>&1; echo "prof rc $?"
ls -R gpurun_out/prof1 | head -20
