# Round 6 (i): planned tail split threshold sweep (reserve 16)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6i
mkdir -p $O
NB="--embedding_size 32 --feature_size 117581"
B="python bench.py --gpus 1 --no_secondary"
export ROCFM_EMB_PLAN_RESERVE=16
for rep in 1 2 3; do
  for l in 128 512 1024; do
    ROCFM_EMB_LSPLIT=$l timeout -k 10 150 $B --steps 20 --warmup 5 > $O/l${l}_d20_$rep.json 2>/dev/null || exit 1
    ROCFM_EMB_LSPLIT=$l timeout -k 10 150 $B --steps 20 --warmup 5 $NB > $O/l${l}_n20_$rep.json 2>/dev/null || exit 1
  done
done
for l in 128 512 1024; do
  ROCFM_EMB_LSPLIT=$l timeout -k 10 150 $B --steps 200 --warmup 20 > $O/l${l}_d200.json 2>/dev/null || exit 1
  ROCFM_EMB_LSPLIT=$l timeout -k 10 150 $B --steps 200 --warmup 20 $NB > $O/l${l}_n200.json 2>/dev/null || exit 1
done
ROCFM_EMB_LSPLIT=1024 MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_default_l1024.txt 2>&1 || exit 1
ROCFM_EMB_LSPLIT=1024 MULTI=1 K=32 V=117581 timeout -k 10 200 python tools/diag_phases.py > $O/phases_notebook_l1024.txt 2>&1 || exit 1
