#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in delgraph delgraph_nodestroy nobarrier plain; do
PROBE_EXIT=$m timeout -k 5 60 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 tools/probe_graph_collectives.py > gpurun_out/g9_$m.log 2>&1; rc=$?; echo "probe $m rc $rc"; grep -E "rank|deleted|barrier|destroyed" gpurun_out/g9_$m.log | grep -v "^\[W"
[ $rc -eq 124 ] && break
done
exit 0
