# Round 5 (u): final validation — the whole GPU suite, smoke, the driver-shaped bench (all
# secondary windows, GPU state around the TFRecord window), a kernel trace of the headline
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
ROCFM_BENCH_GPU_STATE=1 timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_default -o df -- python3 bench.py --steps 200 --warmup 20 --no_secondary > $O/default_prof.log 2>&1 || exit 1
