cd $GRAFT_REPO_ROOT
O=gpurun_out/r5est
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_estimator_gpu.py tests/test_decode_gpu.py tests/test_hazard_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
