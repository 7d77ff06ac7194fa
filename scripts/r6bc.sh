# Round 6 (bc): capture-first warm-up order (ROCFM_BENCH_CAPTURE_FIRST) x lean launch, driver-shaped
# bench processes interleaved (headline k=10, notebook k=32)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bc
mkdir -p $O
B="python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5"
NB="--embedding_size 32 --feature_size 117581"
for rep in 1 2 3; do
  for cf in 0 1; do
    for v in 0 3; do
      ROCFM_BENCH_CAPTURE_FIRST=$cf ROCFM_LEAN_LAUNCH=$v timeout -k 10 150 $B > $O/d20_c${cf}_v${v}_$rep.json 2>$O/d20_c${cf}_v${v}_$rep.err || exit 1
      ROCFM_BENCH_CAPTURE_FIRST=$cf ROCFM_LEAN_LAUNCH=$v timeout -k 10 150 $B $NB > $O/n20_c${cf}_v${v}_$rep.json 2>$O/n20_c${cf}_v${v}_$rep.err || exit 1
    done
  done
done
