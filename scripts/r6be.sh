# Round 6 (be): row-kernel entry skew (notebook and headline, multi-step path)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6be
mkdir -p $O
MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_d.txt 2>&1 || exit 1
K=32 V=117581 MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_n.txt 2>&1 || exit 1
K=32 V=117581 timeout -k 10 200 python tools/diag_phases.py > $O/phases_n_perstep.txt 2>&1 || exit 1
