# Search merge with bucket directories: merge microbenchmark, DP tests, 2-rank rehearsal A/B
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c/sdir
timeout -k 10 300 python tools/bench_merge.py > gpurun_out/r3c/sdir/bench_merge.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_fused_dp_gpu.py tests/test_rccl_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/sdir/tests.log 2>&1
for r in 1 2; do
  for d in 1 0; do
    ROCFM_SEARCH_DIR=$d ROCFM_BENCH_BACKEND=gloo timeout -k 10 200 python bench.py --gpus 2 --steps 64 --warmup 16 > gpurun_out/r3c/sdir/dp2_dir${d}_$r.log 2>&1
  done
done
