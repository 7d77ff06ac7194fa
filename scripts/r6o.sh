# Round 6 (o): next-step input prefetch from the tail (on / off), head-cost sweep
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_emb_plan_gpu.py tests/test_fused_kernels_gpu.py -x -q --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || exit 1
NB="--embedding_size 32 --feature_size 117581"
B="python bench.py --gpus 1 --no_secondary"
for rep in 1 2 3; do
  timeout -k 10 150 $B --steps 20 --warmup 5 > $O/pf1_d20_$rep.json 2>/dev/null || exit 1
  ROCFM_TAIL_PREFETCH_INPUTS=0 timeout -k 10 150 $B --steps 20 --warmup 5 > $O/pf0_d20_$rep.json 2>/dev/null || exit 1
  timeout -k 10 150 $B --steps 20 --warmup 5 $NB > $O/pf1_n20_$rep.json 2>/dev/null || exit 1
  ROCFM_TAIL_PREFETCH_INPUTS=0 timeout -k 10 150 $B --steps 20 --warmup 5 $NB > $O/pf0_n20_$rep.json 2>/dev/null || exit 1
done
for b in 3 6; do
  for rep in 1 2; do
    ROCFM_EMB_BETA=$b timeout -k 10 150 $B --steps 20 --warmup 5 > $O/b${b}_d20_$rep.json 2>/dev/null || exit 1
    ROCFM_EMB_BETA=$b timeout -k 10 150 $B --steps 20 --warmup 5 $NB > $O/b${b}_n20_$rep.json 2>/dev/null || exit 1
  done
done
timeout -k 10 150 $B --steps 200 --warmup 20 > $O/pf1_d200.json 2>/dev/null || exit 1
ROCFM_TAIL_PREFETCH_INPUTS=0 timeout -k 10 150 $B --steps 200 --warmup 20 > $O/pf0_d200.json 2>/dev/null || exit 1
MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_pf1.txt 2>&1 || exit 1
ROCFM_TAIL_PREFETCH_INPUTS=0 MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_pf0.txt 2>&1 || exit 1
