# Round 6 (bh): what the overlapped side chain costs the main chain (main graph GPU time/step)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bh
mkdir -p $O
timeout -k 10 200 python tools/probe_side_overlap.py 10 20 > $O/k10.json 2> $O/k10.err || exit 1
timeout -k 10 200 python tools/probe_side_overlap.py 32 20 > $O/k32.json 2> $O/k32.err || exit 1
