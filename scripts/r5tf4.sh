# Round 5 (tf4): TFRecord window — the copy stream split into its H2D copies and its parse kernel
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5tf4
mkdir -p $O
for first in 1 0 1 0; do
  ROCFM_BENCH_TF_FIRST=$first timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/tf_first$first.log 2>&1 || exit 1
done
