# Round 6 (bs): the plan kernel on 256-thread workgroups (fits beside the split k = 32 row tiles too)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bs
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_emb_plan_gpu.py -x -q --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/probe_side_overlap.py 32 20 > $O/k32.json 2> $O/k32.err || exit 1
B="python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5"
NB="--embedding_size 32 --feature_size 117581"
for rep in 1 2 3; do
  timeout -k 10 150 $B > $O/d20_$rep.json 2>/dev/null || exit 1
  timeout -k 10 150 $B $NB > $O/n20_$rep.json 2>/dev/null || exit 1
  timeout -k 10 150 $B $NB --deep_layers 256,128,64 > $O/r20_$rep.json 2>/dev/null || exit 1
done
