# Round 5 (f): 1B-row parse debug, GPU tests of the round's changes, the bench's window-order A/B
# with process-wide engine streams, the 1B-row step
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 400 python tools/debug_1b.py > $O/d1b.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_decode_gpu.py tests/test_hazard_gpu.py tests/test_sort_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
ROCFM_BENCH_TF_FIRST=0 timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_tflast.log 2>&1 || exit 1
ROCFM_BENCH_TF_FIRST=1 timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_tffirst.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --feature_size 1000000000 --steps 200 --warmup 20 --no_secondary > $O/b1b.log 2>&1 || exit 1
