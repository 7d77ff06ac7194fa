# Round 5 (tf): TFRecord window order in separate processes, GPU state recorded around the window
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5tf
mkdir -p $O
for first in 0 1 0 1; do
  ROCFM_BENCH_GPU_STATE=1 ROCFM_BENCH_TF_FIRST=$first timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/tf_first$first.log 2>&1 || exit 1
done
