# Round 6 (a): headline regression bisect on the round-5 tree — driver-shaped 20-step window,
# interleaved A/B of the env-switchable round-5 changes, 3 processes each; tail kernel means by rocprof
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6a
mkdir -p $O
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no_secondary"
for rep in 1 2 3; do
  timeout -k 10 150 $B > $O/def_$rep.json 2> $O/def_$rep.err || exit 1
  ROCFM_WGRAD_TW=1 timeout -k 10 150 $B > $O/tw1_$rep.json 2> $O/tw1_$rep.err || exit 1
  ROCFM_NUMA_BIND=0 timeout -k 10 150 $B > $O/numa0_$rep.json 2> $O/numa0_$rep.err || exit 1
done
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary > $O/def200.json 2>&1 || exit 1
ROCFM_WGRAD_TW=1 timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary > $O/tw1_200.json 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_def -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary > $GRAFT_REPO_ROOT/$O/prof_def.log 2>&1 || exit 1
ROCFM_WGRAD_TW=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_tw1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary > $GRAFT_REPO_ROOT/$O/prof_tw1.log 2>&1 || exit 1
