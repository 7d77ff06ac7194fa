#!/bin/bash
# instruction-fetch counters on the fused kernels (is the 100 KB step_tail / 19 KB rows code icache-bound?)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > gpurun_out/avail53.txt 2>&1 || { tail -20 gpurun_out/avail53.txt; exit 1; }
grep -o -E "\b(SQC?_[A-Z_]*(ICACHE|IFETCH|INST)[A-Z_]*)\b" gpurun_out/avail53.txt | sort -u | tr '\n' ' '; echo
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/pmc53 -o a --output-format csv -- python bench.py --steps 64 --warmup 16 > gpurun_out/p53a.log 2>&1 || { tail -20 gpurun_out/p53a.log; exit 1; }
echo pass-a-ok
