# Round 5 (h): the copy-stream ordering fix (1B-row wide-vocab test, hazard plans), the emb-role
# column split, GPU clock-ramp probe, k = 32 tile / width A/B, phase stamps
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_sort_gpu.py tests/test_hazard_gpu.py tests/test_decode_gpu.py tests/test_fused_kernels_gpu.py tests/test_trajectory_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/probe_clock_ramp.py > $O/clock.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/probe_clock_ramp.py >> $O/clock.jsonl 2>&1 || exit 1
bash scripts/r5g.sh
