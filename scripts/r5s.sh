cd $GRAFT_REPO_ROOT
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 200 python tools/debug_pre.py > $O/dbg.log 2>&1
exit 0
