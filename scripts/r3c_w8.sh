# eight ranks sharing the GPU: DP equivalence through the W = 8 paths (one test)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c/w8
timeout -k 10 400 python -u -m pytest tests/test_fused_dp_gpu.py -k "world8 or world4_direct" -x -v --timeout 300 --timeout-method thread > gpurun_out/r3c/w8/tests.log 2>&1
