# Round 6 (bl): row-tile workgroups with the whole CU's LDS (ROCFM_ROWS_LDS_EXCL) — side-chain
# overlap cost and driver-shaped windows
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bl
mkdir -p $O
for x in 0 1; do
  ROCFM_ROWS_LDS_EXCL=$x timeout -k 10 120 python tools/probe_side_overlap.py 10 20 > $O/k10_x$x.json 2> $O/k10_x$x.err || exit 1
  ROCFM_ROWS_LDS_EXCL=$x timeout -k 10 120 python tools/probe_side_overlap.py 32 20 > $O/k32_x$x.json 2> $O/k32_x$x.err || exit 1
done
B="python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5"
for rep in 1 2 3; do
  for x in 0 1; do
    ROCFM_ROWS_LDS_EXCL=$x timeout -k 10 150 $B > $O/d20_x${x}_$rep.json 2>/dev/null || exit 1
    ROCFM_ROWS_LDS_EXCL=$x timeout -k 10 150 $B --embedding_size 32 --feature_size 117581 > $O/n20_x${x}_$rep.json 2>/dev/null || exit 1
  done
done
