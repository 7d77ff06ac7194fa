# A/B of the fused tail's sorted entries per embedding workgroup (ROCFM_TAIL_CHUNK 512 / 256), with
# the kernel tests under 256 first.
set -e
cd $GRAFT_REPO_ROOT
ROCFM_TAIL_CHUNK=256 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_kernels_gpu.py tests/test_fused_dp_gpu.py -k "multi_step or stream or optimizers or oracle or world1 or union" > gpurun_out/r3_tc_test.log 2>&1
for i in 1 2; do
  for tc in 512 256; do
    ROCFM_TAIL_CHUNK=$tc timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no_secondary > gpurun_out/r3_tc${tc}_b200_$i.log 2>&1
    ROCFM_TAIL_CHUNK=$tc timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no_secondary > gpurun_out/r3_tc${tc}_b20_$i.log 2>&1
  done
done
ROCFM_TAIL_CHUNK=256 MULTI=1 timeout -k 10 300 python tools/diag_phases.py > gpurun_out/r3_tc256_phases.log 2>&1
