# Round 4 (u): final check on HEAD — the whole GPU suite, smoke, the driver-shaped bench with its
# secondary windows
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.log 2>&1
