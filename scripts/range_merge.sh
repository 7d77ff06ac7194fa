# Range merge: kernel test, DP equivalence tests (range at W = 2 / 4), merge microbenchmark
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_kernels_gpu.py -k merge_range > gpurun_out/r3_rm_test.log 2>&1
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_fused_dp_gpu.py >> gpurun_out/r3_rm_test.log 2>&1
timeout -k 10 300 python tools/bench_merge.py > gpurun_out/r3_bench_merge.log 2>&1
