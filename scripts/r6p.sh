# Round 6 (p): main graphs on a high-priority stream (A/B)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6p
mkdir -p $O
python -c "import torch; print(torch.cuda.Stream.priority_range())" > $O/prio.txt 2>&1
NB="--embedding_size 32 --feature_size 117581"
B="python bench.py --gpus 1 --no_secondary"
for rep in 1 2 3; do
  ROCFM_MAIN_PRIORITY=1 timeout -k 10 150 $B --steps 20 --warmup 5 > $O/hp_d20_$rep.json 2>/dev/null || exit 1
  timeout -k 10 150 $B --steps 20 --warmup 5 > $O/np_d20_$rep.json 2>/dev/null || exit 1
  ROCFM_MAIN_PRIORITY=1 timeout -k 10 150 $B --steps 20 --warmup 5 $NB > $O/hp_n20_$rep.json 2>/dev/null || exit 1
  timeout -k 10 150 $B --steps 20 --warmup 5 $NB > $O/np_n20_$rep.json 2>/dev/null || exit 1
done
ROCFM_MAIN_PRIORITY=1 timeout -k 10 150 $B --steps 200 --warmup 20 > $O/hp_d200.json 2>/dev/null || exit 1
timeout -k 10 150 $B --steps 200 --warmup 20 > $O/np_d200.json 2>/dev/null || exit 1
