# Round 4 (j): determinism of the step tail with the spare-thread table loads (graphs vs per-step,
# each twice; 1 step and 40 steps)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4j
mkdir -p $O
STEPS=1 timeout -k 10 200 python tools/diag_determinism.py > $O/det1.log 2>&1
STEPS=40 timeout -k 10 200 python tools/diag_determinism.py > $O/det40.log 2>&1
ROCFM_TAIL_CHUNK=512 STEPS=40 timeout -k 10 200 python tools/diag_determinism.py > $O/det40_c512.log 2>&1
