# Round 4 (t): vectorised LDS stores of the gathered rows in the row kernel (phase A):
# oracle / bitwise tests, determinism, bench (default, driver-shaped,
# k = 32 shapes), phase stamps
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_kernels_gpu.py tests/test_bf16_table_gpu.py tests/test_sort_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
STEPS=40 timeout -k 10 200 python tools/diag_determinism.py > $O/det40.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > $O/b200_$r.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_secondary > $O/b20_$r.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $O/nb_$r.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 > $O/rd_$r.log 2>&1
done
MULTI=1 timeout -k 10 300 python tools/diag_phases.py > $O/phases_default.log 2>&1
MULTI=1 K=32 V=117581 LAYERS=128,64,32 timeout -k 10 300 python tools/diag_phases.py > $O/phases_nb.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_fused_dp_gpu.py tests/test_rowshard_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_dist.log 2>&1
