# Round 6 (q): the 20-step window's fixed costs (graph launch, side graph)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6q
mkdir -p $O
S=20 timeout -k 10 200 python tools/probe_graph_launch.py > $O/probe20.txt 2>&1 || exit 1
S=64 timeout -k 10 200 python tools/probe_graph_launch.py > $O/probe64.txt 2>&1 || exit 1
