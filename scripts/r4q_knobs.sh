# Round 4 (q): tail chunk 256 vs 512 entries per embedding workgroup after the DPP scan (A/B)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4q
mkdir -p $O
for r in 1 2; do
for c in 256 512; do
ROCFM_TAIL_CHUNK=$c timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > $O/b200_c${c}_$r.log 2>&1
ROCFM_TAIL_CHUNK=$c timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_secondary > $O/b20_c${c}_$r.log 2>&1
ROCFM_TAIL_CHUNK=$c timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $O/nb_c${c}_$r.log 2>&1
done
done
