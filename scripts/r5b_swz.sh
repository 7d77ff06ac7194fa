# Round 5 (b): fragment-swizzled actT / dzT (common.h act_swz) — oracle tests, phase stamps at the
# three shapes, the driver-shaped bench
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_kernels_gpu.py tests/test_trajectory_gpu.py tests/test_sort_gpu.py tests/test_hazard_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef.txt 2>&1
ROCFM_WGRAD_TW=auto K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef_twauto.txt 2>&1
MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_default.txt 2>&1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.log 2>&1
