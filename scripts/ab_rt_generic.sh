# A/B of the runtime-shape row kernel's examples per workgroup (16 vs 8) on the reference's flag
# defaults (k=32, MLP 256-128-64, 117,581 rows) and a 400-400-400 MLP; the row-tile test first.
set -e
cd $GRAFT_REPO_ROOT
true
for rt in 16 8; do
  ROCFM_ROW_TILE=$rt timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 > gpurun_out/r3_refdef_rt${rt}.log 2>&1
  ROCFM_ROW_TILE=$rt timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 16 --feature_size 117581 --deep_layers 400,400,400 > gpurun_out/r3_r400_rt${rt}.log 2>&1
done
