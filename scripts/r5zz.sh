# Round 5 (z): final-tree validation after the NUMA default — GPU suite, smoke, the driver-shaped bench
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5zz
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.log 2>&1 || exit 1
