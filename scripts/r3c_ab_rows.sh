# A/B on one box: phase-A paired LDS stores (new) vs HEAD (old .so); oracle tests on the new one
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c/abr
SO=$(ls deepfm-tensorflow-distributed-training-on-amazon-sagemaker_amd/_rocfm_hip*.so)
cp $SO ab/new_hip.so
for r in 1 2; do
  for v in new old; do
    cp ab/${v}_hip.so $SO
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > gpurun_out/r3c/abr/${v}_200_$r.log 2>&1
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_secondary > gpurun_out/r3c/abr/${v}_20_$r.log 2>&1
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > gpurun_out/r3c/abr/${v}_k32_$r.log 2>&1
  done
done
cp ab/new_hip.so $SO
MULTI=1 timeout -k 10 180 python tools/diag_phases.py > gpurun_out/r3c/abr/phases_new.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_fused_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/abr/tests.log 2>&1
