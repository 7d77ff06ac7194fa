# Round 5 (k): plan-ahead DP merge tests, merge microbenchmark, layer-0 split ablations (k = 32
# shapes), the GPU suite, smoke, bench with the TFRecord window twice
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_dp_gpu.py -x -q --timeout 300 --timeout-method thread -k "plan or world8" > $O/dp_plan.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_merge.py --worlds 1,2,4,8 --memory cached,uncached --skip_owner > $O/bench_merge.log 2>&1 || exit 1
for a in 0 16 32; do
  for rt in 8 4; do
    ROCFM_ROW_TILE=$rt ABLATE=$a K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef_rt${rt}_a${a}.txt 2>&1 || exit 1
    ROCFM_ROW_TILE=$rt ABLATE=$a K=32 V=117581 LAYERS=128,64,32 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_notebook_rt${rt}_a${a}.txt 2>&1 || exit 1
  done
done
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
ROCFM_BENCH_TF_TWICE=1 timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_tftwice.log 2>&1 || exit 1
