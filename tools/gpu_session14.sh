#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/step_variants.py > gpurun_out/v14.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/v14.log | tail -20; exit $rc
