# Round 5 (t): write-through (sc1) stores of the row kernel's gradient rows / h0ᵀ (ROCFM_WT) — does
# a launch that leaves less dirty L2 end sooner?  200-step windows A/B, k = 10 and k = 32
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "multi_step or row_tile or row_split" > $O/tests.log 2>&1 || exit 1
for wt in 0 1 3 0 1 3; do
  ROCFM_WT=$wt timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no_secondary >> $O/default_wt$wt.log 2>&1 || exit 1
  ROCFM_WT=$wt timeout -k 10 300 python bench.py --steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --no_secondary >> $O/notebook_wt$wt.log 2>&1 || exit 1
done
ROCFM_WT=1 ROCFM_TEST_WT=1 timeout -k 10 300 python -u -m pytest tests/test_fused_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "multi_step or row_tile or row_split" > $O/tests_wt.log 2>&1 || exit 1
