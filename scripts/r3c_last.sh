# last check of the final tree: smoke, driver-shaped bench, DP + fused-kernel GPU tests
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c/last
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c/last/smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3c/last/b20.log 2>&1
timeout -k 10 500 python -u -m pytest tests/test_fused_kernels_gpu.py tests/test_fused_dp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/last/tests.log 2>&1
