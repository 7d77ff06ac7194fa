# Round 6 (bb): first-launch cost of a precaptured graph pair — hipGraphUpload at capture time
# (ROCFM_GRAPH_UPLOAD) x lean launch (ROCFM_LEAN_LAUNCH), driver-shaped bench processes interleaved
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bb
mkdir -p $O
ROCFM_GRAPH_UPLOAD=1 timeout -k 10 200 python tools/probe_window_lean.py 10 > $O/probe_k10_up.json 2> $O/probe_k10_up.err || exit 1
B="python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5"
for rep in 1 2 3; do
  for up in 0 1; do
    for v in 0 3; do
      ROCFM_GRAPH_UPLOAD=$up ROCFM_LEAN_LAUNCH=$v timeout -k 10 150 $B > $O/d20_u${up}_v${v}_$rep.json 2>$O/d20_u${up}_v${v}_$rep.err || exit 1
    done
  done
done
for up in 0 1; do
  ROCFM_GRAPH_UPLOAD=$up ROCFM_LEAN_LAUNCH=3 timeout -k 10 150 $B --embedding_size 32 --feature_size 117581 > $O/n20_u${up}_v3.json 2>/dev/null || exit 1
done
