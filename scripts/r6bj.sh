# Round 6 (bj): CU-masked side stream, wider masks; side graph end vs main graph length
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bj
mkdir -p $O
for n in 0 96 128 192; do
  ROCFM_SIDE_CUS=$n timeout -k 10 120 python tools/probe_side_overlap.py 10 20 > $O/k10_$n.json 2> $O/k10_$n.err || exit 1
  ROCFM_SIDE_CUS=$n timeout -k 10 120 python tools/probe_side_overlap.py 32 20 > $O/k32_$n.json 2> $O/k32_$n.err || exit 1
done
B="python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5"
for rep in 1 2 3; do
  for n in 0 128 192; do
    ROCFM_SIDE_CUS=$n timeout -k 10 150 $B > $O/d20_${n}_$rep.json 2>/dev/null || exit 1
    ROCFM_SIDE_CUS=$n timeout -k 10 150 $B --embedding_size 32 --feature_size 117581 > $O/n20_${n}_$rep.json 2>/dev/null || exit 1
  done
done
