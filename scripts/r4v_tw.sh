# Round 4 (v): widened weight-gradient tiles (one dispatch round) at the k = 32 shapes, re-measured
# after the embedding role got faster (continuation, DPP scan)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4v
mkdir -p $O
for r in 1 2; do
for tw in 1 auto; do
ROCFM_WGRAD_TW=$tw timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $O/nb_tw${tw}_$r.log 2>&1
ROCFM_WGRAD_TW=$tw timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 --deep_layers 256,128,64 > $O/rd_tw${tw}_$r.log 2>&1
done
done
ROCFM_WGRAD_TW=auto MULTI=1 K=32 V=117581 LAYERS=128,64,32 timeout -k 10 300 python tools/diag_phases.py > $O/phases_nb_twauto.log 2>&1
