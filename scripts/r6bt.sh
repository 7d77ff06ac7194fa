# Round 6 (bt): final validation (plan kernel 256 threads) on the current tree — GPU suite, smoke, driver-shaped bench (all windows)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bt
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > $O/suite.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_full.json 2> $O/bench_full.err || exit 1
