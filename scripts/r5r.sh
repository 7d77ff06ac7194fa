cd $GRAFT_REPO_ROOT
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "multi_step_graph_equals_per_step and sparse and composite" > $O/dbg.log 2>&1
exit 0
