# Reference defaults (k=32, 256-128-64) on the compile-time-shape row kernel: tests, bench, phases
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fused_kernels_gpu.py -k "256 or wide or row_tile" > gpurun_out/r3b/wide_tests.log 2>&1
A="--steps 200 --warmup 20 --no_secondary --embedding_size 32 --deep_layers 256,128,64 --feature_size 117581"
for v in "ROCFM_DEDUP=0" "ROCFM_DEDUP=1" "ROCFM_DEDUP=0" "ROCFM_DEDUP=1"; do
  echo "== $v" >> gpurun_out/r3b/wide_bench.log
  env $v timeout -k 10 200 python bench.py $A 2>/dev/null | tail -1 | cut -c1-200 >> gpurun_out/r3b/wide_bench.log
done
MULTI=1 K=32 V=117581 LAYERS=256,128,64 timeout -k 10 300 python tools/diag_phases.py > gpurun_out/r3b/wide_phases.log 2>&1
ROCFM_DEDUP=1 MULTI=1 K=32 V=117581 LAYERS=256,128,64 timeout -k 10 300 python tools/diag_phases.py > gpurun_out/r3b/wide_phases_dedup.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_secondary > gpurun_out/r3b/wide_default_b20.log 2>&1
