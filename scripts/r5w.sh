# Round 5 (w): the DP rehearsal through bench.py (4 and 2 ranks sharing the GPU, gloo bootstrap,
# p2p exchange: phase_ms with the plan-ahead merge); per-tile dedup A/B on the k = 32 notebook shape
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5w
mkdir -p $O
ROCFM_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 4 --steps 32 --warmup 8 --steps_per_graph 16 > $O/rehearsal4.log 2>&1 || exit 1
ROCFM_BENCH_BACKEND=gloo ROCFM_MERGE=direct timeout -k 10 600 python bench.py --gpus 4 --steps 32 --warmup 8 --steps_per_graph 16 --no_secondary > $O/rehearsal4_direct.log 2>&1 || exit 1
for d in 0 1 0 1; do
  ROCFM_DEDUP=$d timeout -k 10 300 python bench.py --steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --no_secondary >> $O/notebook_dedup$d.log 2>&1 || exit 1
done
