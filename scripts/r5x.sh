# Round 5 (x): DP rehearsal phase times, plan-ahead vs direct maps vs search merges (4 and 2 ranks
# sharing the GPU, gloo bootstrap, p2p copy push)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5x
mkdir -p $O
for m in direct auto; do
  ROCFM_BENCH_BACKEND=gloo ROCFM_MERGE=$m ROCFM_BENCH_SECONDARY_S=60 timeout -k 10 600 python bench.py --gpus 4 --steps 32 --warmup 8 --steps_per_graph 16 > $O/r4_$m.log 2>&1 || exit 1
  ROCFM_BENCH_BACKEND=gloo ROCFM_MERGE=$m ROCFM_BENCH_SECONDARY_S=60 timeout -k 10 600 python bench.py --gpus 2 --steps 32 --warmup 8 --steps_per_graph 16 > $O/r2_$m.log 2>&1 || exit 1
done
