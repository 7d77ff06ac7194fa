# Round 5 (tf2): TFRecord window first, with / without binding to the GPU's NUMA node
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5tf2
mkdir -p $O
for b in 1 0 1 0 1; do
  ROCFM_NUMA_BIND=$b ROCFM_BENCH_GPU_STATE=1 ROCFM_BENCH_TF_FIRST=1 timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bind$b.log 2>&1 || exit 1
done
