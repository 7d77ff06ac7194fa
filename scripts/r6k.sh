# Round 6 (k): split runs combined by their head item after fire-and-forget lead arrivals
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_emb_plan_gpu.py tests/test_fused_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
NB="--embedding_size 32 --feature_size 117581"
B="python bench.py --gpus 1 --no_secondary"
export ROCFM_EMB_PLAN_RESERVE=16
for rep in 1 2 3; do
  for l in 128 512; do
    ROCFM_EMB_LSPLIT=$l timeout -k 10 150 $B --steps 20 --warmup 5 > $O/l${l}_d20_$rep.json 2>/dev/null || exit 1
    ROCFM_EMB_LSPLIT=$l timeout -k 10 150 $B --steps 20 --warmup 5 $NB > $O/l${l}_n20_$rep.json 2>/dev/null || exit 1
  done
  ROCFM_EMB_PLAN=0 timeout -k 10 150 $B --steps 20 --warmup 5 > $O/noplan_d20_$rep.json 2>/dev/null || exit 1
done
for l in 128 512; do
  ROCFM_EMB_LSPLIT=$l timeout -k 10 150 $B --steps 200 --warmup 20 > $O/l${l}_d200.json 2>/dev/null || exit 1
  ROCFM_EMB_LSPLIT=$l timeout -k 10 150 $B --steps 200 --warmup 20 $NB > $O/l${l}_n200.json 2>/dev/null || exit 1
done
MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_default.txt 2>&1 || exit 1
MULTI=1 K=32 V=117581 timeout -k 10 200 python tools/diag_phases.py > $O/phases_notebook.txt 2>&1 || exit 1
