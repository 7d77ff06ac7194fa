# Full GPU suite, smoke, driver-shaped bench + rocprof of the default bench at HEAD
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c/final
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/final/gputests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c/final/smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3c/final/b20.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3c/final/prof -o default -- python bench.py --steps 200 --warmup 20 --no_secondary > gpurun_out/r3c/final/prof.log 2>&1
