# Round 6 (bm): lean-launch event ring (8 deep) — stream / multi-step / hazard tests, full bench
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bm
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_fused_kernels_gpu.py tests/test_hazard_gpu.py tests/test_decode_gpu.py tests/test_emb_plan_gpu.py -x -v --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_full.json 2> $O/bench_full.err || exit 1
