#!/bin/bash
# instruction-cache misses on the fused kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES -d gpurun_out/pmc54 -o a --output-format csv -- python bench.py --steps 64 --warmup 16 > gpurun_out/p54a.log 2>&1 || { tail -20 gpurun_out/p54a.log; exit 1; }
echo pass-a-ok
