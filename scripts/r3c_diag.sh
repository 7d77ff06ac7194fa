# Session 3: loader breakdown on the box (CPU only), phase stamps of the default and the
# reference-default shapes on the multi-step path, rocprof of the reference-default bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c
timeout -k 10 240 python tools/loader_breakdown.py --batches 272,2064 --threads 8,16 > gpurun_out/r3c/loader_breakdown.log 2>&1
MULTI=1 timeout -k 10 180 python tools/diag_phases.py > gpurun_out/r3c/phases_default.log 2>&1
MULTI=1 K=32 V=117581 LAYERS=256,128,64 timeout -k 10 180 python tools/diag_phases.py > gpurun_out/r3c/phases_refdef.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3c/prof_refdef -o refdef -- python bench.py --steps 200 --warmup 20 --no_secondary --embedding_size 32 --deep_layers 256,128,64 --feature_size 117581 > gpurun_out/r3c/prof_refdef.log 2>&1
