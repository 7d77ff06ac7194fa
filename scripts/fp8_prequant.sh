# Pre-quantised fp8 input-layer copies: fp8 tests, then fp8 vs bf16 step time (200 / 20 steps).
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fused_kernels_gpu.py -k "fp8" > gpurun_out/r3_fp8_tests.log 2>&1
for i in 1 2; do
  for dt in bf16 fp8; do
    timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no_secondary --compute_dtype $dt > gpurun_out/r3_fp8cmp_${dt}_b200_$i.log 2>&1
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no_secondary --compute_dtype $dt > gpurun_out/r3_fp8cmp_${dt}_b20_$i.log 2>&1
  done
done
