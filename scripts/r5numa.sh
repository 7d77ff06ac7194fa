cd $GRAFT_REPO_ROOT
O=gpurun_out/r5numa
mkdir -p $O
timeout -k 10 120 python tools/probe_numa.py > $O/probe.log 2>&1 || exit 1
