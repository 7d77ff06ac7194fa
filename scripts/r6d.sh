# Round 6 (d): kernel traces of the planned vs unplanned tail (driver-shaped bench, 200 and 20 steps),
# summarised on the box (per-kernel mean / p50 / p90 / max)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6d
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in plan noplan; do
  if [ $v = noplan ]; then export ROCFM_EMB_PLAN=0; else unset ROCFM_EMB_PLAN; fi
  for st in 200 20; do
    w=$([ $st = 200 ] && echo 20 || echo 5)
    timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/p_${v}_$st -o run -- python3 $R/bench.py --gpus 1 --steps $st --warmup $w --no_secondary > $R/$O/prof${st}_$v.log 2>&1 || exit 1
    python3 $R/tools/rocpd_summary.py $(find /tmp/p_${v}_$st -name "*.db" | head -1) > $R/$O/prof${st}_$v.txt 2>&1 || exit 1
  done
done
