# dp_owner (owner-sharded DP) + row-shard regression tests, 2-rank shared-GPU benches
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_rowshard_gpu.py -k "dp_owner or world1 or 2ranks_equals or 4ranks or shadow" > gpurun_out/r3b/owner_tests.log 2>&1
for par in dp dp_owner rowshard; do
  echo "== $par" >> gpurun_out/r3b/owner_bench.log
  ROCFM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 64 --warmup 16 --parallelism $par --no_secondary 2>/dev/null | tail -1 | cut -c100-220 >> gpurun_out/r3b/owner_bench.log
done
echo "== dp_owner world 1" >> gpurun_out/r3b/owner_bench.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --parallelism dp_owner --no_secondary 2>/dev/null | tail -1 | cut -c100-220 >> gpurun_out/r3b/owner_bench.log
