# Re-entry (session 3) verification at HEAD: GPU suite, smoke, driver-shaped bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/gputests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c/smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3c/b20.log 2>&1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no_secondary > gpurun_out/r3c/b200.log 2>&1
