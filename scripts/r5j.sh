# Round 5 (j): the plan-ahead DP merge (composite-key fix), the GPU suite, smoke, merge
# microbenchmark, bench with the TFRecord window twice
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_dp_gpu.py -x -q --timeout 300 --timeout-method thread -k "plan or world8 or world4_p2p" > $O/dp_plan.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_merge.py --worlds 1,2,4,8 --memory cached,uncached --skip_owner > $O/bench_merge.log 2>&1 || exit 1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
ROCFM_BENCH_TF_TWICE=1 timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_tftwice.log 2>&1 || exit 1
