# Round 6 (z): lsplit sweep with the head-key slab (headline 20/200, notebook 200)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6z
mkdir -p $O
B="python bench.py --gpus 1 --no_secondary"
NB="--embedding_size 32 --feature_size 117581"
for rep in 1 2 3; do
  for ls in 512 256 128; do
    ROCFM_EMB_LSPLIT=$ls timeout -k 10 150 $B --steps 20 --warmup 5 > $O/l${ls}_d20_$rep.json 2>/dev/null || exit 1
  done
done
for ls in 512 256 128; do
  ROCFM_EMB_LSPLIT=$ls timeout -k 10 150 $B --steps 200 --warmup 20 > $O/l${ls}_d200.json 2>/dev/null || exit 1
  ROCFM_EMB_LSPLIT=$ls timeout -k 10 150 $B --steps 200 --warmup 20 $NB > $O/l${ls}_n200.json 2>/dev/null || exit 1
  ROCFM_EMB_LSPLIT=$ls MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_d_l${ls}.txt 2>&1 || exit 1
done
