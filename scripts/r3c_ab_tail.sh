# A/B on one box: tail emb role with early item loads + two-chunk continuation (new) vs HEAD (old .so)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c/ab
SO=$(ls deepfm-tensorflow-distributed-training-on-amazon-sagemaker_amd/_rocfm_hip*.so)
cp $SO ab/new_hip.so
for r in 1 2; do
  for v in new old; do
    cp ab/${v}_hip.so $SO
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > gpurun_out/r3c/ab/${v}_200_$r.log 2>&1
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_secondary > gpurun_out/r3c/ab/${v}_20_$r.log 2>&1
  done
done
cp ab/new_hip.so $SO
MULTI=1 timeout -k 10 180 python tools/diag_phases.py > gpurun_out/r3c/ab/phases_new.log 2>&1
timeout -k 10 240 python tools/loader_breakdown.py --batches 272,2064 --threads 16 > gpurun_out/r3c/ab/loader_breakdown_new.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels_gpu.py tests/test_fused_dp_gpu.py tests/test_rowshard_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/ab/tests.log 2>&1
