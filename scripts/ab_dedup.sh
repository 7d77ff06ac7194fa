# Per-tile dedup: kernel / engine tests, then A/B of ROCFM_DEDUP x ROCFM_TAIL_CHUNK on the bench.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_fused_kernels_gpu.py tests/test_fused_dp_gpu.py tests/test_bf16_table_gpu.py > gpurun_out/r3_dd_test.log 2>&1
for i in 1 2; do
  for dd in 0 1; do
    for tc in 512 256; do
      ROCFM_DEDUP=$dd ROCFM_TAIL_CHUNK=$tc timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no_secondary > gpurun_out/r3_dd${dd}_tc${tc}_b200_$i.log 2>&1
      ROCFM_DEDUP=$dd ROCFM_TAIL_CHUNK=$tc timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no_secondary > gpurun_out/r3_dd${dd}_tc${tc}_b20_$i.log 2>&1
    done
  done
done
ROCFM_DEDUP=1 ROCFM_TAIL_CHUNK=256 MULTI=1 timeout -k 10 300 python tools/diag_phases.py > gpurun_out/r3_dd1_phases.log 2>&1
