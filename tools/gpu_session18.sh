#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python tools/frag_probe.py > gpurun_out/fp18.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/fp18.log; exit $rc
