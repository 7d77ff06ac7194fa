# Round 6 (bg): capture-first warm-up for the DP / row-shard engines — bench rehearsal tests,
# 2-rank gloo rehearsal, and a 1-rank RCCL DP window A/B (ROCFM_FORCE_COLLECTIVES=1)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rccl_gpu.py -x -v --timeout 300 --timeout-method thread > $O/rccl_tests.log 2>&1 || exit 1
ROCFM_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --no_secondary > $O/gloo2.json 2> $O/gloo2.err || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no_secondary --parallelism dp"
for rep in 1 2 3; do
  for cf in 0 1; do
    ROCFM_FORCE_COLLECTIVES=1 ROCFM_BENCH_CAPTURE_FIRST=$cf timeout -k 10 200 $B > $O/dp1_c${cf}_$rep.json 2> $O/dp1_c${cf}_$rep.err || exit 1
  done
done
for cf in 0 1; do
  ROCFM_BENCH_CAPTURE_FIRST=$cf timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no_secondary --parallelism rowshard > $O/rs1_c${cf}.json 2> $O/rs1_c${cf}.err || exit 1
done
