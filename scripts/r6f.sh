# Round 6 (f): tile-prefetched plan kernel — tests, A/B windows, phases, kernel-trace summary
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6f
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_emb_plan_gpu.py -x -q --timeout 200 --timeout-method thread > $O/plan_tests.log 2>&1 || exit 1
NB="--embedding_size 32 --feature_size 117581"
for rep in 1 2 3; do
  timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5 > $O/plan_d20_$rep.json 2>/dev/null || exit 1
  ROCFM_EMB_PLAN=0 timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5 > $O/noplan_d20_$rep.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5 $NB > $O/plan_n20_$rep.json 2>/dev/null || exit 1
done
timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 200 --warmup 20 > $O/plan_d200.json 2>/dev/null || exit 1
timeout -k 10 150 python bench.py --gpus 1 --no_secondary --steps 200 --warmup 20 $NB > $O/plan_n200.json 2>/dev/null || exit 1
MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_default.txt 2>&1 || exit 1
MULTI=1 K=32 V=117581 timeout -k 10 200 python tools/diag_phases.py > $O/phases_notebook.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/p_plan -o run -- python3 $R/bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary > $R/$O/prof_plan.log 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $(find /tmp/p_plan -name "*.db" | head -1) > $R/$O/prof_plan.txt 2>&1 || exit 1
export ROCFM_EMB_PLAN=0
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/p_noplan -o run -- python3 $R/bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary > $R/$O/prof_noplan.log 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $(find /tmp/p_noplan -name "*.db" | head -1) > $R/$O/prof_noplan.txt 2>&1 || exit 1
