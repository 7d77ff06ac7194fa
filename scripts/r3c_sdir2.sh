# search + directory merge through W = 4: DP / RCCL / hazard tests, 4-rank rehearsal
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c/sdir2
timeout -k 10 500 python -u -m pytest tests/test_fused_dp_gpu.py tests/test_rccl_gpu.py tests/test_hazard_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/sdir2/tests.log 2>&1
for d in 1 0; do
  ROCFM_SEARCH_DIR=$d ROCFM_BENCH_BACKEND=gloo timeout -k 10 200 python bench.py --gpus 4 --steps 64 --warmup 16 > gpurun_out/r3c/sdir2/dp4_dir$d.log 2>&1
done
