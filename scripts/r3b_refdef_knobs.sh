# Reference-default shape (k=32, 256-128-64, 117,581 vocab): dedup / tail chunk / row tile knobs
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
A="--steps 200 --warmup 20 --no_secondary --embedding_size 32 --deep_layers 256,128,64 --feature_size 117581"
for v in "ROCFM_DEDUP=0" "ROCFM_DEDUP=1" "ROCFM_DEDUP=1 ROCFM_TAIL_CHUNK=512" "ROCFM_DEDUP=0 ROCFM_ROW_TILE=16"; do
  echo "== $v" >> gpurun_out/r3b/knobs.log
  env $v timeout -k 10 200 python bench.py $A 2>/dev/null | tail -1 | cut -c1-200 >> gpurun_out/r3b/knobs.log
done
ROCFM_DEDUP=1 MULTI=1 K=32 V=117581 LAYERS=256,128,64 GENERIC=1 timeout -k 10 300 python tools/diag_phases.py > gpurun_out/r3b/refdef_phases_dedup.log 2>&1
