# Round 5 (tf3): TFRecord window order with the NUMA binding default, separate processes
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5tf3
mkdir -p $O
for first in 1 0 1 0; do
  ROCFM_BENCH_GPU_STATE=1 ROCFM_BENCH_TF_FIRST=$first timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/tf_first$first.log 2>&1 || exit 1
done
