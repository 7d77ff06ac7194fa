# Round 6 (bq): the plan kernel on 512-thread workgroups (co-resident with the k = 32 row tiles)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bq
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_emb_plan_gpu.py tests/test_fused_kernels_gpu.py -x -q --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || exit 1
K=32 V=117581 MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_n.txt 2>&1 || exit 1
MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_d.txt 2>&1 || exit 1
timeout -k 10 120 python tools/probe_side_overlap.py 32 20 > $O/k32.json 2> $O/k32.err || exit 1
timeout -k 10 120 python tools/probe_side_overlap.py 10 20 > $O/k10.json 2> $O/k10.err || exit 1
B="python bench.py --gpus 1 --no_secondary --steps 20 --warmup 5"
for rep in 1 2 3; do
  timeout -k 10 150 $B > $O/d20_$rep.json 2>/dev/null || exit 1
  timeout -k 10 150 $B --embedding_size 32 --feature_size 117581 > $O/n20_$rep.json 2>/dev/null || exit 1
done
