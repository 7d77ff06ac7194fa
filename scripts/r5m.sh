# Round 5 (m): the row-tile split (2 workgroups per 8-row tile, exchange of layer 0's outputs) for
# the flag-default shape — bitwise tests, phase stamps, 200-step windows; DP plan merge from 2 ranks
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "row_split or row_tile" > $O/split_tests.log 2>&1 || exit 1
K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef_split.txt 2>&1 || exit 1
ROCFM_ROW_SPLIT=1 K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef_nosplit.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 --no_secondary > $O/refdef_split.log 2>&1 || exit 1
ROCFM_ROW_SPLIT=1 timeout -k 10 300 python bench.py --steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 --no_secondary > $O/refdef_nosplit.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_fused_dp_gpu.py tests/test_fused_kernels_gpu.py tests/test_trajectory_gpu.py tests/test_rowshard_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
