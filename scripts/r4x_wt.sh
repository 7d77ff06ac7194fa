# Round 4 (x): the row kernel's per-lookup gradient rows stored write-through (sc1) so the
# kernel boundary has less to write back (A/B, interleaved), + correctness with it on
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4x
mkdir -p $O
ROCFM_WT_CONTRIB=1 timeout -k 10 600 python -u -m pytest tests/test_fused_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_wt.log 2>&1
ROCFM_WT_CONTRIB=1 STEPS=40 timeout -k 10 200 python tools/diag_determinism.py > $O/det40_wt.log 2>&1
for r in 1 2 3; do
for w in 0 1; do
ROCFM_WT_CONTRIB=$w timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary > $O/b200_wt${w}_$r.log 2>&1
ROCFM_WT_CONTRIB=$w timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_secondary > $O/b20_wt${w}_$r.log 2>&1
done
done
for w in 0 1; do
ROCFM_WT_CONTRIB=$w timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $O/nb_wt${w}.log 2>&1
done
