# A/B of the row kernel's examples per workgroup (ROCFM_ROW_TILE) on the bench config and the
# notebook shape (k=32, 117,581 rows); the row-tile equivalence test first.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_kernels_gpu.py -k row_tile > gpurun_out/r3_rt_test.log 2>&1
for i in 1 2; do
  for rt in 16 8 4; do
    ROCFM_ROW_TILE=$rt timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no_secondary > gpurun_out/r3_b200_rt${rt}_$i.log 2>&1
    ROCFM_ROW_TILE=$rt timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no_secondary > gpurun_out/r3_b20_rt${rt}_$i.log 2>&1
    ROCFM_ROW_TILE=$rt timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > gpurun_out/r3_nb200_rt${rt}_$i.log 2>&1
  done
done
