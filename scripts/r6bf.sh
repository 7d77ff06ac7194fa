# Round 6 (bf): k=32 shapes — 256 row workgroups (entry skew behind side-chain kernels) vs 128:
# notebook row tile 4 vs 8, flag defaults split 2 vs 1; driver-shaped 20-step windows, interleaved
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bf
mkdir -p $O
B="python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5 --embedding_size 32 --feature_size 117581"
for rep in 1 2 3; do
  for rt in 0 8; do
    ROCFM_ROW_TILE=$rt timeout -k 10 150 $B > $O/n_rt${rt}_$rep.json 2>/dev/null || exit 1
  done
  for sp in auto 1; do
    ROCFM_ROW_SPLIT=$sp timeout -k 10 150 $B --deep_layers 256,128,64 > $O/r_sp${sp}_$rep.json 2>/dev/null || exit 1
  done
done
ROCFM_ROW_TILE=8 K=32 V=117581 MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_n_rt8.txt 2>&1 || exit 1
K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_r.txt 2>&1 || exit 1
