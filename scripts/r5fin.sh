# Round 5 (fin): the whole GPU suite and smoke on the final tree
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5fin
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
