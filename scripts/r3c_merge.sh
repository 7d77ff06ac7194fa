# Merge microbenchmark incl. the owner-sharded DP merge at W = 1..8 (one GPU)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c
timeout -k 10 300 python tools/bench_merge.py > gpurun_out/r3c/bench_merge.log 2>&1
timeout -k 10 300 python tools/bench_merge.py --hash > gpurun_out/r3c/bench_merge_hash.log 2>&1
