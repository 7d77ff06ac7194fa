# New defaults (tail chunk 256, dedup off): kernel + DP tests, smoke, driver-shaped bench
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_fused_kernels_gpu.py tests/test_fused_dp_gpu.py -k "not world4_hash" > gpurun_out/r3_def_test.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_def_smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_def_b20.log 2>&1
