# Round 5 (y): k = 32 notebook shape — tail chunk size and wgrad tile width knobs, 200-step windows
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5y
mkdir -p $O
NB="--steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --no_secondary"
for i in 1 2; do
  timeout -k 10 300 python bench.py $NB >> $O/base.log 2>&1 || exit 1
  ROCFM_TAIL_CHUNK=512 timeout -k 10 300 python bench.py $NB >> $O/chunk512.log 2>&1 || exit 1
  ROCFM_WGRAD_TW=1 timeout -k 10 300 python bench.py $NB >> $O/tw1.log 2>&1 || exit 1
  ROCFM_WGRAD_TW=auto timeout -k 10 300 python bench.py $NB >> $O/twauto.log 2>&1 || exit 1
done
