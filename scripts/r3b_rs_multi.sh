# Row-shard: X3+X4(+next X1) in one hand-off launch — GPU tests + 2-rank shared-GPU A/B bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_rowshard_gpu.py -k "2ranks or 4ranks or shadow or staleness1_2ranks" > gpurun_out/r3b/rs_tests.log 2>&1
for v in 1 0 1 0; do
  echo "== ROCFM_P2P_MULTI=$v" >> gpurun_out/r3b/rs_ab.log
  ROCFM_P2P_MULTI=$v ROCFM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 64 --warmup 16 --parallelism rowshard --no_secondary 2>/dev/null | tail -1 | cut -c1-260 >> gpurun_out/r3b/rs_ab.log
done
