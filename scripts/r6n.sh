# Round 6 (n): the 4-rank gloo bench rehearsal on its own (window progress to a file), then the
# rest of the GPU suite from the rehearsal tests on, verbose
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6n
mkdir -p $O
ROCFM_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 4 --steps 32 --warmup 8 --steps_per_graph 16 > $O/gloo4.json 2> $O/gloo4.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_rccl_gpu.py tests/test_rowshard_gpu.py tests/test_sort_gpu.py tests/test_trajectory_gpu.py -x -v --timeout 170 --timeout-method thread > $O/suite_rest.log 2>&1 || exit 1
