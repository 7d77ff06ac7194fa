# Round 6 (y): kernel-argument placement (HIP_FORCE_DEV_KERNARG) and graph packet capture vs the per-kernel overhead
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6y
mkdir -p $O
B="python bench.py --gpus 1 --no_secondary"
for rep in 1 2 3; do
  timeout -k 10 150 $B --steps 20 --warmup 5 > $O/def_d20_$rep.json 2>/dev/null || exit 1
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 150 $B --steps 20 --warmup 5 > $O/dk1_d20_$rep.json 2>/dev/null || exit 1
  HIP_FORCE_DEV_KERNARG=0 timeout -k 10 150 $B --steps 20 --warmup 5 > $O/dk0_d20_$rep.json 2>/dev/null || exit 1
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 150 $B --steps 20 --warmup 5 > $O/pc0_d20_$rep.json 2>/dev/null || exit 1
done
timeout -k 10 150 $B --steps 200 --warmup 20 > $O/def_d200.json 2>/dev/null || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 150 $B --steps 200 --warmup 20 > $O/dk1_d200.json 2>/dev/null || exit 1
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 150 $B --steps 200 --warmup 20 > $O/dk0_d200.json 2>/dev/null || exit 1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 150 $B --steps 200 --warmup 20 > $O/pc0_d200.json 2>/dev/null || exit 1
