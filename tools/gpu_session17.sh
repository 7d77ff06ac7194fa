#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 128 512 1024 4096; do
B=$b timeout -k 10 200 python tools/diag_phases.py > gpurun_out/diag17b_$b.log 2>&1 || exit 1; echo "B=$b"; grep -A4 "deepfm_rows:" gpurun_out/diag17b_$b.log | head -5
done
