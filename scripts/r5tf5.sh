# Round 5 (tf5): TFRecord window — loader slots held in flight (hold 2 vs 4)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5tf5
mkdir -p $O
for h in 4 2 4 2; do
  timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 --loader_hold $h >> $O/hold$h.log 2>&1 || exit 1
done
