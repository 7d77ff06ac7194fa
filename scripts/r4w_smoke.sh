# Round 4 (w): smoke + sort / decode / fused-kernel tests on the final in-tree build
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4w
mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_sort_gpu.py tests/test_decode_gpu.py tests/test_fused_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_secondary > $O/b20.log 2>&1
