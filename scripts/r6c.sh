# Round 6 (c): planned tail knobs — CU reserve for the side chain, head cost, split threshold —
# driver-shaped windows (20 steps) and 200-step windows, default and notebook shapes
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_emb_plan_gpu.py -x -q --timeout 200 --timeout-method thread > $O/plan_tests.log 2>&1 || exit 1
run() {  # name, env..., then bench args after --
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 150 python bench.py --gpus 1 --no_secondary "$@" > $O/$name.json 2> $O/$name.err
}
NB="--embedding_size 32 --feature_size 117581"
for rep in 1 2; do
  for cfg in "noplan ROCFM_EMB_PLAN=0" "r0 ROCFM_EMB_PLAN_RESERVE=0" "r32 ROCFM_EMB_PLAN_RESERVE=32" "r64 ROCFM_EMB_PLAN_RESERVE=64" \
             "r32b2 ROCFM_EMB_PLAN_RESERVE=32 ROCFM_EMB_BETA=2" "r32b8 ROCFM_EMB_PLAN_RESERVE=32 ROCFM_EMB_BETA=8" \
             "r32l256 ROCFM_EMB_PLAN_RESERVE=32 ROCFM_EMB_LSPLIT=256"; do
    set -- $cfg
    name=$1; shift
    run ${name}_d20_$rep "$@" X=1 -- --steps 20 --warmup 5 || exit 1
    run ${name}_n20_$rep "$@" X=1 -- --steps 20 --warmup 5 $NB || exit 1
  done
done
for cfg in "noplan ROCFM_EMB_PLAN=0" "r0 ROCFM_EMB_PLAN_RESERVE=0" "r32 ROCFM_EMB_PLAN_RESERVE=32" "r64 ROCFM_EMB_PLAN_RESERVE=64"; do
  set -- $cfg
  name=$1; shift
  run ${name}_d200 "$@" X=1 -- --steps 200 --warmup 20 || exit 1
  run ${name}_n200 "$@" X=1 -- --steps 200 --warmup 20 $NB || exit 1
done
MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_default.txt 2>&1 || exit 1
MULTI=1 K=32 V=117581 timeout -k 10 200 python tools/diag_phases.py > $O/phases_notebook.txt 2>&1 || exit 1
ROCFM_EMB_PLAN_RESERVE=32 MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_default_r32.txt 2>&1 || exit 1
ROCFM_EMB_PLAN_RESERVE=32 MULTI=1 K=32 V=117581 timeout -k 10 200 python tools/diag_phases.py > $O/phases_notebook_r32.txt 2>&1 || exit 1
