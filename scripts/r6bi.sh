# Round 6 (bi): side stream on a CU-masked hardware queue (ROCFM_SIDE_CUS / ROCFM_SIDE_CU_PICK):
# main graph GPU time with the side chain overlapped, and the driver-shaped window
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bi
mkdir -p $O
for cfg in "0 stride" "16 stride" "32 stride" "64 stride" "32 last" "128 stride"; do
  set -- $cfg
  ROCFM_SIDE_CUS=$1 ROCFM_SIDE_CU_PICK=$2 timeout -k 10 120 python tools/probe_side_overlap.py 10 20 > $O/k10_$1_$2.json 2> $O/k10_$1_$2.err || exit 1
  ROCFM_SIDE_CUS=$1 ROCFM_SIDE_CU_PICK=$2 timeout -k 10 120 python tools/probe_side_overlap.py 32 20 > $O/k32_$1_$2.json 2> $O/k32_$1_$2.err || exit 1
done
B="python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5"
for rep in 1 2; do
  for n in 0 32 64; do
    ROCFM_SIDE_CUS=$n timeout -k 10 150 $B > $O/d20_${n}_$rep.json 2>/dev/null || exit 1
    ROCFM_SIDE_CUS=$n timeout -k 10 150 $B --embedding_size 32 --feature_size 117581 > $O/n20_${n}_$rep.json 2>/dev/null || exit 1
  done
done
