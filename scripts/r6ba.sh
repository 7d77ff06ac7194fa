# Round 6 (ba): the 20-step window's fixed cost — ROCFM_LEAN_LAUNCH variants (probe interleaved in
# one process; driver-shaped bench processes interleaved)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ba
mkdir -p $O
timeout -k 10 200 python tools/probe_window_lean.py 10 > $O/probe_k10.json 2> $O/probe_k10.err || exit 1
timeout -k 10 200 python tools/probe_window_lean.py 32 > $O/probe_k32.json 2> $O/probe_k32.err || exit 1
B="python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5"
for rep in 1 2 3; do
  for v in 0 3; do
    ROCFM_LEAN_LAUNCH=$v timeout -k 10 150 $B > $O/d20_v${v}_$rep.json 2>/dev/null || exit 1
  done
done
