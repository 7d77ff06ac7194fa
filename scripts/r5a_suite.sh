# Round 5 (a): the GPU suite after the halted-step / decode gate / WGRAD_TW changes, smoke, the
# driver-shaped bench, and the reference-shape phase stamps (baseline for the layer-0 GEMM work)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.log 2>&1
K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef.txt 2>&1
K=32 V=117581 LAYERS=128,64,32 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_notebook.txt 2>&1
ROCFM_WGRAD_TW=auto K=32 V=117581 LAYERS=256,128,64 MULTI=1 timeout -k 10 120 python tools/diag_phases.py > $O/phases_refdef_twauto.txt 2>&1
