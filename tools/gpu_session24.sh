#!/bin/bash
# profiles of the three step pipelines → markdown reports (traces deleted on the box)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof24
for par in auto dp rowshard; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof24 -o $par -- python bench.py --steps 160 --warmup 32 --parallelism $par > gpurun_out/p24_$par.log 2>&1 || exit 1
python tools/prof_report.py gpurun_out/prof24/$par --title "bench.py --parallelism $par (B=1024, 1M vocab, 1 MI355X)" > gpurun_out/report24_$par.md || exit 1
done
timeout -k 10 200 python tools/diag_phases.py > gpurun_out/diag24.log 2>&1 || exit 1
rm -f gpurun_out/prof24/*_kernel_trace.csv
