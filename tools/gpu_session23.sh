#!/bin/bash
# full GPU suite + profiles of the three step pipelines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t23.log 2>&1; rc=$?; echo "gpu tests rc $rc"; tail -3 gpurun_out/t23.log
[ $rc -eq 0 ] || exit 1
rm -rf gpurun_out/prof23
for par in auto dp rowshard; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof23 -o $par -- python bench.py --steps 160 --warmup 32 --parallelism $par > gpurun_out/p23_$par.log 2>&1 || exit 1
done
timeout -k 10 200 python tools/diag_phases.py > gpurun_out/diag23.log 2>&1 || exit 1
for par in auto dp rowshard; do python tools/prof_report.py gpurun_out/prof23/$par --title "bench.py --parallelism $par (B=1024, 1M vocab)" > gpurun_out/report_$par.md; done
rm -f gpurun_out/prof23/*_kernel_trace.csv
ls gpurun_out
