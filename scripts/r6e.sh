# Round 6 (e): coalesced plan kernel — tests, A/B windows, kernel-trace summary
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6e
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_emb_plan_gpu.py -x -q --timeout 200 --timeout-method thread > $O/plan_tests.log 2>&1 || exit 1
NB="--embedding_size 32 --feature_size 117581"
for rep in 1 2 3; do
  timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5 > $O/plan_d20_$rep.json 2>/dev/null || exit 1
  ROCFM_EMB_PLAN=0 timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5 > $O/noplan_d20_$rep.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5 $NB > $O/plan_n20_$rep.json 2>/dev/null || exit 1
  ROCFM_EMB_BETA=2 timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5 > $O/b2_d20_$rep.json 2>/dev/null || exit 1
  ROCFM_EMB_BETA=2 timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5 $NB > $O/b2_n20_$rep.json 2>/dev/null || exit 1
done
timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 200 --warmup 20 > $O/plan_d200.json 2>/dev/null || exit 1
ROCFM_EMB_PLAN=0 timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 200 --warmup 20 > $O/noplan_d200.json 2>/dev/null || exit 1
timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 200 --warmup 20 $NB > $O/plan_n200.json 2>/dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/p_plan -o run -- python3 $R/bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary > $R/$O/prof_plan.log 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $(find /tmp/p_plan -name "*.db" | head -1) > $R/$O/prof_plan.txt 2>&1 || exit 1
