cd $GRAFT_REPO_ROOT
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 200 python tools/debug_hkeys.py > $O/hkeys.log 2>&1
ROCFM_TAIL_CHUNK=512 timeout -k 10 300 python -u -m pytest tests/test_fused_kernels_gpu.py -q --timeout 120 --timeout-method thread -k "multi_step_graph_equals_per_step" > $O/pre512.log 2>&1
exit 0
