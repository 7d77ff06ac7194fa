# Round 5 (v): phase B (FM) on one wave per row, 64 lanes — kernel tests, phase stamps, windows
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_fused_kernels_gpu.py tests/test_trajectory_gpu.py tests/test_bf16_table_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_default.txt 2>&1 || exit 1
K=32 V=117581 LAYERS=128,64,32 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_notebook.txt 2>&1 || exit 1
K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef.txt 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no_secondary >> $O/default.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --no_secondary >> $O/notebook.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 --no_secondary >> $O/refdef.log 2>&1 || exit 1
done
