# Round 5 (p): isolate the multi-step ≡ per-step mismatch (tail prefetch on / off)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5p
mkdir -p $O
ROCFM_TAIL_PREFETCH=0 timeout -k 10 300 python -u -m pytest tests/test_fused_kernels_gpu.py -q --timeout 120 --timeout-method thread -k "multi_step_graph_equals_per_step" > $O/nopre.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels_gpu.py -q --timeout 120 --timeout-method thread -k "multi_step_graph_equals_per_step" > $O/pre.log 2>&1
exit 0
