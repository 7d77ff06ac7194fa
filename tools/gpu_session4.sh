#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python tools/diag_phases.py > gpurun_out/diag4.log 2>&1; echo "diag rc $?"; cat gpurun_out/diag4.log | grep -v amdgpu.ids
timeout -k 10 240 python bench.py --steps 400 --warmup 40 2>&1 | tail -1
