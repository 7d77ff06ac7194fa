# Round 4 (m): the whole GPU suite on HEAD, smoke, and the driver-shaped bench with its secondary
# windows (TFRecord window first, 32 steps per graph)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/b20.log 2>&1
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1
MULTI=1 K=32 V=117581 LAYERS=128,64,32 timeout -k 10 300 python tools/diag_phases.py > $O/phases_nb_static.log 2>&1
MULTI=1 K=32 V=117581 LAYERS=256,128,64 timeout -k 10 300 python tools/diag_phases.py > $O/phases_refdef_static.log 2>&1
