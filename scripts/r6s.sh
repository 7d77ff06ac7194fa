# Round 6 (s): where the planned tail's slow workgroups run (XCC / CU placement stamps)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hazard_gpu.py -x -q --timeout 170 --timeout-method thread > $O/hazard_tests.log 2>&1 || exit 1
for rep in 1 2 3; do
  MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_default_$rep.txt 2>&1 || exit 1
done
K=32 V=117581 MULTI=1 timeout -k 10 200 python tools/diag_phases.py > $O/phases_notebook.txt 2>&1 || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/p_nb -o run -- python3 $R/bench.py --gpus 1 --steps 200 --warmup 20 --no_secondary --embedding_size 32 --feature_size 117581 > $R/$O/prof_nb.log 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $(find /tmp/p_nb -name "*.db" | head -1) > $R/$O/prof_nb.txt 2>&1 || exit 1
