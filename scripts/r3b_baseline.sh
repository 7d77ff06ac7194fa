# Re-entry baseline: smoke, driver-shaped bench, reference-default shape bench + phase stamps
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b/smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3b/b20.log 2>&1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --deep_layers 256,128,64 --feature_size 117581 > gpurun_out/r3b/refdef.log 2>&1
MULTI=1 K=32 V=117581 LAYERS=256,128,64 GENERIC=1 timeout -k 10 300 python tools/diag_phases.py > gpurun_out/r3b/refdef_phases.log 2>&1
