# Round 6 (x): row prefetch issued after phase 1's first loads; outliers with / without the slab
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_emb_plan_gpu.py tests/test_fused_kernels_gpu.py -x -q --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in 1 0; do
    ROCFM_EMB_HSLAB=$v MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_d_s${v}_$rep.txt 2>&1 || exit 1
  done
done
B="python bench.py --gpus 1 --no_secondary"
NB="--embedding_size 32 --feature_size 117581"
for rep in 1 2 3; do
  for v in 1 0; do
    ROCFM_EMB_HSLAB=$v timeout -k 10 150 $B --steps 20 --warmup 5 > $O/s${v}_d20_$rep.json 2>/dev/null || exit 1
  done
done
for v in 1 0; do
  ROCFM_EMB_HSLAB=$v timeout -k 10 150 $B --steps 200 --warmup 20 > $O/s${v}_d200.json 2>/dev/null || exit 1
  ROCFM_EMB_HSLAB=$v timeout -k 10 150 $B --steps 200 --warmup 20 $NB > $O/s${v}_n200.json 2>/dev/null || exit 1
done
