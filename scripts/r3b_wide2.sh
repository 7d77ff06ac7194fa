# Wide static kernel + batch norm on compile-time shapes + 2-per-CU tail: tests and A/B benches
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fused_kernels_gpu.py > gpurun_out/r3b/w2_tests.log 2>&1
A="--steps 200 --warmup 20 --no_secondary --embedding_size 32 --deep_layers 256,128,64 --feature_size 117581"
N="--steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581"
for v in 1 0 1 0; do
  echo "== refdef ROCFM_TAIL_OCC2=$v" >> gpurun_out/r3b/w2_bench.log
  ROCFM_TAIL_OCC2=$v timeout -k 10 200 python bench.py $A 2>/dev/null | tail -1 | cut -c100-200 >> gpurun_out/r3b/w2_bench.log
  echo "== notebook ROCFM_TAIL_OCC2=$v" >> gpurun_out/r3b/w2_bench.log
  ROCFM_TAIL_OCC2=$v timeout -k 10 200 python bench.py $N 2>/dev/null | tail -1 | cut -c100-200 >> gpurun_out/r3b/w2_bench.log
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_secondary > gpurun_out/r3b/w2_default_b20.log 2>&1
