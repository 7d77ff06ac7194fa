# Round 5 (opt): notebook shape, optimizer A/B (diagnostic: how much of the tail is the row update)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5opt
mkdir -p $O
NB="--steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --no_secondary"
for o in Adam GD Adagrad Adam; do
  timeout -k 10 300 python bench.py $NB --optimizer $o >> $O/nb_$o.log 2>&1 || exit 1
done
