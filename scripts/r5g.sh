# Round 5 (g): the reference's k = 32 shapes — examples per row workgroup (ROCFM_ROW_TILE 8 / 4) ×
# weight-gradient tile width (ROCFM_WGRAD_TW 1 / 2), 200-step windows
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5h
mkdir -p $O
for rt in 8 4; do for tw in 1 2; do
  ROCFM_ROW_TILE=$rt ROCFM_WGRAD_TW=$tw timeout -k 10 300 python bench.py --steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 --no_secondary > $O/refdef_rt${rt}_tw${tw}.log 2>&1 || exit 1
  ROCFM_ROW_TILE=$rt ROCFM_WGRAD_TW=$tw timeout -k 10 300 python bench.py --steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --no_secondary > $O/notebook_rt${rt}_tw${tw}.log 2>&1 || exit 1
done; done
for rt in 8 4; do ROCFM_ROW_TILE=$rt timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no_secondary > $O/default_rt${rt}.log 2>&1 || exit 1; done
K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef.txt 2>&1 || exit 1
MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_default.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_fused_kernels_gpu.py tests/test_trajectory_gpu.py tests/test_fused_dp_gpu.py tests/test_rowshard_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
