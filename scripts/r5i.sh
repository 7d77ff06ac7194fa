# Round 5 (i): the GPU suite on the new defaults (widened wgrad tiles, 4-row workgroups at wide
# input layers, emb-role split, process-wide streams), smoke, the plan-ahead merge microbenchmark,
# the bench with the TFRecord window twice (first and last, copy-stream timing)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_merge.py --worlds 1,2,4,8 --memory cached,uncached --skip_owner > $O/bench_merge.log 2>&1 || exit 1
ROCFM_BENCH_TF_TWICE=1 timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_tftwice.log 2>&1 || exit 1
