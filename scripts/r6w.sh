# Round 6 (w): which tail workgroups exit last (role, entry, exit)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6w
mkdir -p $O
for rep in 1 2; do
  MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_d_$rep.txt 2>&1 || exit 1
done
K=32 V=117581 MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_n.txt 2>&1 || exit 1
