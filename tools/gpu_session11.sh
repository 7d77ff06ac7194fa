#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t11.log 2>&1; rc=$?; echo "gpu tests rc $rc"; tail -25 gpurun_out/t11.log
exit $rc
