# Round 6 (h): planned tail CU reserve sweep with the wave-segmented plan kernel
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6h
mkdir -p $O
NB="--embedding_size 32 --feature_size 117581"
B="python bench.py --gpus 1 --no_secondary"
for rep in 1 2 3; do
  for r in 0 8 16 32; do
    ROCFM_EMB_PLAN_RESERVE=$r timeout -k 10 150 $B --steps 20 --warmup 5 > $O/r${r}_d20_$rep.json 2>/dev/null || exit 1
  done
  ROCFM_EMB_PLAN=0 timeout -k 10 150 $B --steps 20 --warmup 5 > $O/noplan_d20_$rep.json 2>/dev/null || exit 1
done
for r in 0 8 16 32; do
  ROCFM_EMB_PLAN_RESERVE=$r timeout -k 10 150 $B --steps 200 --warmup 20 > $O/r${r}_d200.json 2>/dev/null || exit 1
  ROCFM_EMB_PLAN_RESERVE=$r timeout -k 10 150 $B --steps 20 --warmup 5 $NB > $O/r${r}_n20.json 2>/dev/null || exit 1
done
ROCFM_EMB_PLAN=0 timeout -k 10 150 $B --steps 200 --warmup 20 > $O/noplan_d200.json 2>/dev/null || exit 1
ROCFM_EMB_PLAN_RESERVE=16 MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_default_r16.txt 2>&1 || exit 1
