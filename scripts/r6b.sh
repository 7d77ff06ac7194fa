# Round 6 (b): the planned step tail — plan kernel vs replica, bitwise vs per-step, the existing
# multi-step tests, then the driver-shaped bench and phase stamps at the default and notebook shapes
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_emb_plan_gpu.py -x -v --timeout 200 --timeout-method thread > $O/plan_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fused_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > $O/fused_tests.log 2>&1 || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no_secondary"
for rep in 1 2 3; do
  timeout -k 10 150 $B > $O/plan_$rep.json 2> $O/plan_$rep.err || exit 1
  ROCFM_EMB_PLAN=0 timeout -k 10 150 $B > $O/noplan_$rep.json 2> $O/noplan_$rep.err || exit 1
done
NB="--embedding_size 32 --feature_size 117581"
timeout -k 10 150 $B $NB > $O/nb_plan.json 2> $O/nb_plan.err || exit 1
ROCFM_EMB_PLAN=0 timeout -k 10 150 $B $NB > $O/nb_noplan.json 2> $O/nb_noplan.err || exit 1
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary > $O/plan200.json 2>&1 || exit 1
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary $NB > $O/nb_plan200.json 2>&1 || exit 1
MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_default.txt 2>&1 || exit 1
MULTI=1 K=32 V=117581 timeout -k 10 200 python tools/diag_phases.py > $O/phases_notebook.txt 2>&1 || exit 1
